/*
 * mqr_oracle.c -- CPU restatement of the reference hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * This file is the parity oracle (and the "port" CPU baseline timed by bench.py).  It is
 * never linked into, loaded by, or called from the product library; only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg use it.
 *
 * What it restates (reference = lszmer/metaquest-3d-reconstruction @ /root/reference):
 *   - TSDF touch / integrate / extract: the reference calls Open3D 0.19.0
 *     (environment.yml:17, a pip dependency that is NOT vendored and NOT installed here) at
 *       scripts/processing/reconstruction/utils/o3d_utils.py:170-179   VoxelBlockGrid(...)
 *       scripts/processing/reconstruction/utils/o3d_utils.py:212-219   compute_unique_block_coordinates
 *       scripts/processing/reconstruction/utils/o3d_utils.py:221-229   integrate
 *       scripts/processing/reconstruction/reconstruct_scene.py:90      extract_point_cloud
 *       scripts/processing/reconstruction/reconstruct_scene.py:105-108 extract_triangle_mesh
 *     The arithmetic below follows the published Open3D 0.19 algorithm (VoxelBlockGrid.cpp,
 *     kernel/VoxelBlockGridImpl.h, TransformIndexer.h, MarchingCubesConst.h) as restated in
 *     SURVEY.md Appendix A.  Open3D cannot be run here, so this part is PARITY UNPINNED
 *     against real Open3D; it is pinned by the known-answer tests in tests/test_oracle_tsdf.py.
 *   - Depth confidence: scripts/processing/reconstruction/confidence_estimation/
 *       compute_pixel_error_map.py:4-92 (bilinear_interpolate_depth), :95-117
 *       (depth_to_pointcloud_numpy), :120-220 (compute_pixel_error_map) and
 *       estimate_depth_confidences.py:15-79 (build_confidence_map).
 *     numpy's dtype promotion is mirrored exactly (float64 arithmetic, float32 rounding of
 *     the interpolated depth and of the error) and the result is pinned by golden vectors
 *     generated from the reference itself (tests/golden/, tests/golden/make_golden.py).
 *
 * Build: see oracle/Makefile (gcc -O2 -ffp-contract=off -fopenmp).  No FMA contraction, so
 * every float op rounds exactly as written -- the HIP library is compiled the same way.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "../include/mqr_mc_tables.h"

#define ORC_EMPTY UINT64_MAX
#define ORC_BIAS (1 << 20)

typedef struct orc_vbg {
    float voxel_size;
    int R;
    int64_t R3;
    /* hash: open addressing, linear probing */
    uint64_t* hkeys;
    int64_t* hvals;
    int64_t hcap; /* power of two */
    /* blocks in activation order */
    int32_t* keys; /* n*3 */
    float* tsdf;   /* n*R3 */
    float* weight; /* n*R3 */
    int64_t n, cap;
} orc_vbg;

static uint64_t pack_key(int32_t x, int32_t y, int32_t z) {
    return ((uint64_t)(uint32_t)(x + ORC_BIAS) << 42) | ((uint64_t)(uint32_t)(y + ORC_BIAS) << 21) |
           (uint64_t)(uint32_t)(z + ORC_BIAS);
}

static uint64_t mix64(uint64_t k) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdULL;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ULL;
    k ^= k >> 33;
    return k;
}

static int64_t h_find(const orc_vbg* v, uint64_t k) {
    uint64_t m = (uint64_t)v->hcap - 1, h = mix64(k) & m;
    for (;;) {
        if (v->hkeys[h] == k) return v->hvals[h];
        if (v->hkeys[h] == ORC_EMPTY) return -1;
        h = (h + 1) & m;
    }
}

static void h_insert_raw(uint64_t* hk, int64_t* hv, int64_t cap, uint64_t k, int64_t val) {
    uint64_t m = (uint64_t)cap - 1, h = mix64(k) & m;
    while (hk[h] != ORC_EMPTY) h = (h + 1) & m;
    hk[h] = k;
    hv[h] = val;
}

static int h_grow(orc_vbg* v) {
    int64_t ncap = v->hcap * 2;
    uint64_t* nk = (uint64_t*)malloc(sizeof(uint64_t) * ncap);
    int64_t* nv = (int64_t*)malloc(sizeof(int64_t) * ncap);
    if (!nk || !nv) return -1;
    memset(nk, 0xff, sizeof(uint64_t) * ncap);
    for (int64_t i = 0; i < v->hcap; ++i)
        if (v->hkeys[i] != ORC_EMPTY) h_insert_raw(nk, nv, ncap, v->hkeys[i], v->hvals[i]);
    free(v->hkeys);
    free(v->hvals);
    v->hkeys = nk;
    v->hvals = nv;
    v->hcap = ncap;
    return 0;
}

/* Activate: return the buffer index of key, allocating a zero-initialised block if new (with
 * `created` given, the caller zeroes the new block itself: orc_integrate does it in parallel). */
static int64_t activate(orc_vbg* v, int32_t x, int32_t y, int32_t z, int* created) {
    uint64_t k = pack_key(x, y, z);
    int64_t idx = h_find(v, k);
    if (created) *created = 0;
    if (idx >= 0) return idx;
    if ((v->n + 1) * 2 > v->hcap && h_grow(v)) return -1;
    if (v->n == v->cap) {
        int64_t ncap = v->cap ? v->cap * 2 : 64;
        int32_t* nk = (int32_t*)realloc(v->keys, sizeof(int32_t) * 3 * ncap);
        if (!nk) return -1;
        v->keys = nk;
        float* nt = (float*)realloc(v->tsdf, sizeof(float) * ncap * v->R3);
        if (!nt) return -1;
        v->tsdf = nt;
        float* nw = (float*)realloc(v->weight, sizeof(float) * ncap * v->R3);
        if (!nw) return -1;
        v->weight = nw;
        v->cap = ncap;
    }
    idx = v->n++;
    v->keys[3 * idx + 0] = x;
    v->keys[3 * idx + 1] = y;
    v->keys[3 * idx + 2] = z;
    if (!created) {
        memset(v->tsdf + idx * v->R3, 0, sizeof(float) * v->R3);
        memset(v->weight + idx * v->R3, 0, sizeof(float) * v->R3);
    }
    h_insert_raw(v->hkeys, v->hvals, v->hcap, k, idx);
    if (created) *created = 1;
    return idx;
}

orc_vbg* orc_vbg_create(float voxel_size, int R, int64_t capacity) {
    orc_vbg* v = (orc_vbg*)calloc(1, sizeof(orc_vbg));
    if (!v) return NULL;
    v->voxel_size = voxel_size;
    v->R = R;
    v->R3 = (int64_t)R * R * R;
    v->hcap = 1024;
    while (v->hcap < 2 * capacity && v->hcap < (1LL << 26)) v->hcap *= 2;
    v->hkeys = (uint64_t*)malloc(sizeof(uint64_t) * v->hcap);
    v->hvals = (int64_t*)malloc(sizeof(int64_t) * v->hcap);
    memset(v->hkeys, 0xff, sizeof(uint64_t) * v->hcap);
    return v;
}

void orc_vbg_destroy(orc_vbg* v) {
    if (!v) return;
    free(v->hkeys);
    free(v->hvals);
    free(v->keys);
    free(v->tsdf);
    free(v->weight);
    free(v);
}

int64_t orc_vbg_size(const orc_vbg* v) { return v->n; }

void orc_set_threads(int n) {
#ifdef _OPENMP
    if (n > 0) omp_set_num_threads(n);
#else
    (void)n;
#endif
}

int orc_get_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

/* TransformIndexer (float32 state, as upstream): extrinsic 3x4, fx, fy, cx, cy, scale. */
typedef struct {
    float e[3][4];
    float fx, fy, cx, cy, scale;
} tindexer;

static void ti_init(tindexer* t, const double* K, const double* T, float scale) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 4; ++j) t->e[i][j] = (float)T[i * 4 + j];
    t->fx = (float)K[0];
    t->fy = (float)K[4];
    t->cx = (float)K[2];
    t->cy = (float)K[5];
    t->scale = scale;
}

static void ti_rigid(const tindexer* t, float x, float y, float z, float* xo, float* yo, float* zo) {
    x *= t->scale;
    y *= t->scale;
    z *= t->scale;
    *xo = x * t->e[0][0] + y * t->e[0][1] + z * t->e[0][2] + t->e[0][3];
    *yo = x * t->e[1][0] + y * t->e[1][1] + z * t->e[1][2] + t->e[1][3];
    *zo = x * t->e[2][0] + y * t->e[2][1] + z * t->e[2][2] + t->e[2][3];
}

/* Rigid inverse in float64 (upstream t::geometry::InverseTransformation). */
static void rigid_inverse(const double* T, double* P) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) P[i * 4 + j] = T[j * 4 + i];
    for (int i = 0; i < 3; ++i)
        P[i * 4 + 3] = -(P[i * 4 + 0] * T[0 * 4 + 3] + P[i * 4 + 1] * T[1 * 4 + 3] + P[i * 4 + 2] * T[2 * 4 + 3]);
    P[12] = 0;
    P[13] = 0;
    P[14] = 0;
    P[15] = 1;
}

/*
 * compute_unique_block_coordinates (o3d_utils.py:212-219 -> upstream DepthTouch, stride 4,
 * 4 samples along the ray through the truncation band).  Writes unique keys (first-occurrence
 * order of the sequential loop) into keys_out (capacity 4*(H/4)*(W/4) keys) and their count.
 * Returns 0, or 1 when no block is touched (upstream raises in that case).
 */
int orc_touch(const float* depth, int H, int W, const double* K, const double* T, float voxel_size, int R,
              float depth_scale, float depth_max, float trunc_mult, int32_t* keys_out, int64_t* n_out) {
    double P[16];
    rigid_inverse(T, P);
    tindexer ti;
    ti_init(&ti, K, P, 1.0f);
    const int stride = 4, step_size = 3;
    const float sdf_trunc = voxel_size * trunc_mult;
    const float block_size = voxel_size * R;
    int64_t rows = H / stride, cols = W / stride, n = rows * cols;
    /* per-call dedup set */
    int64_t scap = 1024;
    while (scap < 8 * n) scap *= 2;
    uint64_t* set = (uint64_t*)malloc(sizeof(uint64_t) * scap);
    memset(set, 0xff, sizeof(uint64_t) * scap);
    int64_t count = 0, total = 0;
    for (int64_t w = 0; w < n; ++w) {
        int64_t y = (w / cols) * stride, x = (w % cols) * stride;
        float d = depth[y * W + x] / depth_scale;
        if (!(d > 0 && d < depth_max)) continue;
        float xc = ((float)x - ti.cx) * 1.0f / ti.fx;
        float yc = ((float)y - ti.cy) * 1.0f / ti.fy;
        float zc = 1.0f;
        float xg, yg, zg;
        ti_rigid(&ti, xc, yc, zc, &xg, &yg, &zg);
        float xo = ti.e[0][3], yo = ti.e[1][3], zo = ti.e[2][3];
        float xd = xg - xo, yd = yg - yo, zd = zg - zo;
        float t_min = fmaxf(d - sdf_trunc, 0.0f);
        float t_max = fminf(d + sdf_trunc, depth_max);
        float t_step = (t_max - t_min) / step_size;
        float t = t_min;
        for (int s = 0; s <= step_size; ++s) {
            int32_t xb = (int32_t)floorf((xo + t * xd) / block_size);
            int32_t yb = (int32_t)floorf((yo + t * yd) / block_size);
            int32_t zb = (int32_t)floorf((zo + t * zd) / block_size);
            ++total;
            uint64_t k = pack_key(xb, yb, zb), m = (uint64_t)scap - 1, h = mix64(k) & m;
            int fresh = 1;
            while (set[h] != ORC_EMPTY) {
                if (set[h] == k) {
                    fresh = 0;
                    break;
                }
                h = (h + 1) & m;
            }
            if (fresh) {
                set[h] = k;
                keys_out[3 * count + 0] = xb;
                keys_out[3 * count + 1] = yb;
                keys_out[3 * count + 2] = zb;
                ++count;
            }
            t += t_step;
        }
    }
    free(set);
    *n_out = count;
    return total == 0 ? 1 : 0;
}

/* vbg.integrate(block_coords, depth, K, T_wc, depth_scale, depth_max, trunc_mult) (o3d_utils.py:221-229). */
int orc_integrate(orc_vbg* v, const int32_t* keys, int64_t n, const float* depth, int H, int W, const double* K,
                  const double* T, float depth_scale, float depth_max, float trunc_mult) {
    int64_t* idx = (int64_t*)malloc(sizeof(int64_t) * (n > 0 ? n : 1));
    uint8_t* fresh = (uint8_t*)malloc(n > 0 ? n : 1);
    for (int64_t b = 0; b < n; ++b) {
        int created = 0;
        idx[b] = activate(v, keys[3 * b], keys[3 * b + 1], keys[3 * b + 2], &created);
        fresh[b] = (uint8_t)created;
        if (idx[b] < 0) {
            free(idx);
            free(fresh);
            return 2;
        }
    }
    tindexer ti;
    ti_init(&ti, K, T, v->voxel_size);
    const int R = v->R;
    const int64_t R3 = v->R3;
    const float sdf_trunc = v->voxel_size * trunc_mult;
    const float hm1 = (float)H - 1.0f, wm1 = (float)W - 1.0f;
    /* Duplicate keys in one call would update a block twice; the reference passes unique keys.
     * Voxel loops nested z, y, x (linear index (z R + y) R + x): the per-voxel arithmetic is the
     * upstream kernel's, evaluated in the same order; only the index decode is hoisted. */
#pragma omp parallel for schedule(dynamic, 8)
    for (int64_t b = 0; b < n; ++b) {
        int64_t bi = idx[b];
        int32_t xb = keys[3 * b], yb = keys[3 * b + 1], zb = keys[3 * b + 2];
        float* tsdf = v->tsdf + bi * R3;
        float* wgt = v->weight + bi * R3;
        if (fresh[b]) { /* new blocks start at zero (App. A.1) */
            memset(tsdf, 0, sizeof(float) * R3);
            memset(wgt, 0, sizeof(float) * R3);
        }
        int64_t vi = 0;
        for (int zv = 0; zv < R; ++zv)
            for (int yv = 0; yv < R; ++yv)
                for (int xv = 0; xv < R; ++xv, ++vi) {
                    int32_t x = xb * R + xv, y = yb * R + yv, z = zb * R + zv;
                    float xc, yc, zc;
                    ti_rigid(&ti, (float)x, (float)y, (float)z, &xc, &yc, &zc);
                    float inv_z = 1.0f / zc;
                    float u = ti.fx * xc * inv_z + ti.cx;
                    float vv = ti.fy * yc * inv_z + ti.cy;
                    if (!(vv >= 0 && u >= 0 && vv <= hm1 && u <= wm1)) continue;
                    int ui = (int)u, vi2 = (int)vv;
                    float d = depth[(int64_t)vi2 * W + ui] / depth_scale;
                    float sdf = d - zc;
                    if (d <= 0 || d > depth_max || zc <= 0 || sdf < -sdf_trunc) continue;
                    sdf = sdf < sdf_trunc ? sdf : sdf_trunc;
                    sdf /= sdf_trunc;
                    float inv_wsum = 1.0f / (wgt[vi] + 1);
                    float w = wgt[vi];
                    tsdf[vi] = (w * tsdf[vi] + sdf) * inv_wsum;
                    wgt[vi] = w + 1;
                }
    }
    free(idx);
    free(fresh);
    return 0;
}

int orc_export(const orc_vbg* v, int32_t* keys, float* tsdf, float* weight) {
    if (keys) memcpy(keys, v->keys, sizeof(int32_t) * 3 * v->n);
    if (tsdf) memcpy(tsdf, v->tsdf, sizeof(float) * v->n * v->R3);
    if (weight) memcpy(weight, v->weight, sizeof(float) * v->n * v->R3);
    return 0;
}

int orc_import(orc_vbg* v, const int32_t* keys, const float* tsdf, const float* weight, int64_t n) {
    for (int64_t b = 0; b < n; ++b) {
        int64_t bi = activate(v, keys[3 * b], keys[3 * b + 1], keys[3 * b + 2], NULL);
        if (bi < 0) return 2;
        memcpy(v->tsdf + bi * v->R3, tsdf + b * v->R3, sizeof(float) * v->R3);
        memcpy(v->weight + bi * v->R3, weight + b * v->R3, sizeof(float) * v->R3);
    }
    return 0;
}

/* ---------------- extraction (upstream ExtractPointCloud / ExtractTriangleMesh) ---------------- */

/* 27-neighbour block table for the active blocks: nb[b*27 + k] = buffer index or -1. */
static int64_t* build_nb(const orc_vbg* v) {
    int64_t* nb = (int64_t*)malloc(sizeof(int64_t) * 27 * (v->n > 0 ? v->n : 1));
#pragma omp parallel for schedule(static)
    for (int64_t b = 0; b < v->n; ++b)
        for (int k = 0; k < 27; ++k) {
            int dx = k % 3 - 1, dy = (k % 9) / 3 - 1, dz = k / 9 - 1;
            nb[b * 27 + k] = h_find(v, pack_key(v->keys[3 * b] + dx, v->keys[3 * b + 1] + dy, v->keys[3 * b + 2] + dz));
        }
    return nb;
}

/* DeviceGetLinearIdx: voxel (xo,yo,zo) relative to block b, possibly one outside it. */
static int64_t lin_idx(const orc_vbg* v, const int64_t* nb, int64_t b, int xo, int yo, int zo) {
    const int R = v->R;
    int xn = (xo + R) % R, yn = (yo + R) % R, zn = (zo + R) % R;
    int dxb = (xo - xn) < 0 ? -1 : ((xo - xn) > 0 ? 1 : 0);
    int dyb = (yo - yn) < 0 ? -1 : ((yo - yn) > 0 ? 1 : 0);
    int dzb = (zo - zn) < 0 ? -1 : ((zo - zn) > 0 ? 1 : 0);
    int k = (dxb + 1) + (dyb + 1) * 3 + (dzb + 1) * 9;
    int64_t bi = nb[b * 27 + k];
    if (bi < 0) return -1;
    return ((bi * R + zn) * R + yn) * R + xn;
}

/* DeviceGetNormal: central differences, components left untouched when a side is missing. */
static void get_normal(const orc_vbg* v, const int64_t* nb, int64_t b, int xo, int yo, int zo, float* n) {
    int64_t vxp = lin_idx(v, nb, b, xo + 1, yo, zo), vxn = lin_idx(v, nb, b, xo - 1, yo, zo);
    int64_t vyp = lin_idx(v, nb, b, xo, yo + 1, zo), vyn = lin_idx(v, nb, b, xo, yo - 1, zo);
    int64_t vzp = lin_idx(v, nb, b, xo, yo, zo + 1), vzn = lin_idx(v, nb, b, xo, yo, zo - 1);
    if (vxp >= 0 && vxn >= 0) n[0] = v->tsdf[vxp] - v->tsdf[vxn];
    if (vyp >= 0 && vyn >= 0) n[1] = v->tsdf[vyp] - v->tsdf[vyn];
    if (vzp >= 0 && vzn >= 0) n[2] = v->tsdf[vzp] - v->tsdf[vzn];
}

static void normalize_into(float nx, float ny, float nz, float* out) {
    float norm = (float)((double)sqrtf(nx * nx + ny * ny + nz * nz) + 1e-5);
    out[0] = nx / norm;
    out[1] = ny / norm;
    out[2] = nz / norm;
}

/* Exclusive prefix sum of per-block counts (in place); returns the total. */
static int64_t excl_scan(int64_t* c, int64_t n) {
    int64_t acc = 0;
    for (int64_t b = 0; b < n; ++b) {
        int64_t t = c[b];
        c[b] = acc;
        acc += t;
    }
    return acc;
}

/* Points of block b (upstream ExtractPointCloud, per voxel, axes x, y, z).  With pos == NULL only
 * counts.  Output order = block order, voxel order, axis: the sequential loop's order; the
 * parallel extraction counts per block, scans, then fills. */
static int64_t points_of_block(const orc_vbg* v, const int64_t* nb, int64_t b, float thr, float* pos, float* nrm) {
    const int R = v->R;
    const int64_t R3 = v->R3;
    int64_t cnt = 0;
    int32_t xb = v->keys[3 * b], yb = v->keys[3 * b + 1], zb = v->keys[3 * b + 2];
    for (int64_t vi = 0; vi < R3; ++vi) {
        int xv = (int)(vi % R), yv = (int)((vi / R) % R), zv = (int)(vi / (R * R));
        int64_t li = b * R3 + vi;
        float tsdf_o = v->tsdf[li], weight_o = v->weight[li];
        if (weight_o <= thr) continue;
        int32_t x = xb * R + xv, y = yb * R + yv, z = zb * R + zv;
        float no[3] = {0, 0, 0}, ni[3] = {0, 0, 0};
        int have_no = 0;
        for (int i = 0; i < 3; ++i) {
            int64_t lii = lin_idx(v, nb, b, xv + (i == 0), yv + (i == 1), zv + (i == 2));
            if (lii < 0) continue;
            float tsdf_i = v->tsdf[lii], weight_i = v->weight[lii];
            if (weight_i > thr && tsdf_i * tsdf_o < 0) {
                if (pos) {
                    if (!have_no) {
                        get_normal(v, nb, b, xv, yv, zv, no);
                        have_no = 1;
                    }
                    float ratio = (0 - tsdf_o) / (tsdf_i - tsdf_o);
                    pos[3 * cnt + 0] = v->voxel_size * (x + ratio * (int)(i == 0));
                    pos[3 * cnt + 1] = v->voxel_size * (y + ratio * (int)(i == 1));
                    pos[3 * cnt + 2] = v->voxel_size * (z + ratio * (int)(i == 2));
                    get_normal(v, nb, b, xv + (i == 0), yv + (i == 1), zv + (i == 2), ni);
                    float nx = (1 - ratio) * no[0] + ratio * ni[0];
                    float ny = (1 - ratio) * no[1] + ratio * ni[1];
                    float nz = (1 - ratio) * no[2] + ratio * ni[2];
                    normalize_into(nx, ny, nz, nrm + 3 * cnt);
                }
                ++cnt;
            }
        }
    }
    return cnt;
}

int64_t orc_extract_points(const orc_vbg* v, float thr, float** pos_out, float** nrm_out) {
    int64_t* nb = build_nb(v);
    const int64_t nblk = v->n;
    int64_t* off = (int64_t*)malloc(sizeof(int64_t) * (nblk > 0 ? nblk : 1));
#pragma omp parallel for schedule(dynamic, 16)
    for (int64_t b = 0; b < nblk; ++b) off[b] = points_of_block(v, nb, b, thr, NULL, NULL);
    const int64_t cnt = excl_scan(off, nblk);
    float* pos = (float*)malloc(sizeof(float) * 3 * (cnt > 0 ? cnt : 1));
    float* nrm = (float*)malloc(sizeof(float) * 3 * (cnt > 0 ? cnt : 1));
#pragma omp parallel for schedule(dynamic, 16)
    for (int64_t b = 0; b < nblk; ++b) points_of_block(v, nb, b, thr, pos + 3 * off[b], nrm + 3 * off[b]);
    free(off);
    free(nb);
    *pos_out = pos;
    *nrm_out = nrm;
    return cnt;
}

int64_t orc_extract_mesh(const orc_vbg* v, float thr, float** vtx_out, float** nrm_out, int32_t** tri_out,
                         int64_t* ntri_out) {
    int64_t* nb = build_nb(v);
    const int R = v->R;
    const int64_t R3 = v->R3, nblk = v->n;
    /* mesh structure: per voxel {vertex idx on +x, +y, +z edge, table index} */
    int32_t* ms = (int32_t*)calloc((size_t)(nblk > 0 ? nblk : 1) * R3 * 4, sizeof(int32_t));
    /* pass 0: cube classification and edge marking (an edge may belong to a neighbour block's
     * voxel: every writer stores the same -1) */
#pragma omp parallel for schedule(dynamic, 16)
    for (int64_t b = 0; b < nblk; ++b)
        for (int64_t vi = 0; vi < R3; ++vi) {
            int xv = (int)(vi % R), yv = (int)((vi / R) % R), zv = (int)(vi / (R * R));
            int table_idx = 0, ok = 1;
            for (int i = 0; i < 8; ++i) {
                int64_t li = lin_idx(v, nb, b, xv + mqr_vtx_shifts[i][0], yv + mqr_vtx_shifts[i][1],
                                     zv + mqr_vtx_shifts[i][2]);
                if (li < 0) {
                    ok = 0;
                    break;
                }
                if (v->weight[li] <= thr) {
                    ok = 0;
                    break;
                }
                table_idx |= (v->tsdf[li] < 0) ? (1 << i) : 0;
            }
            if (!ok) continue;
            ms[(b * R3 + vi) * 4 + 3] = table_idx;
            if (table_idx == 0 || table_idx == 255) continue;
            int edges = mqr_edge_table[table_idx];
            for (int i = 0; i < 12; ++i) {
                if (!(edges & (1 << i))) continue;
                int xi = xv + mqr_edge_shifts[i][0], yi = yv + mqr_edge_shifts[i][1], zi = zv + mqr_edge_shifts[i][2];
                int dxb = xi / R, dyb = yi / R, dzb = zi / R;
                int k = (dxb + 1) + (dyb + 1) * 3 + (dzb + 1) * 9;
                int64_t bi = nb[b * 27 + k];
                /* inverse index == buffer index here (blocks are enumerated in buffer order) */
                int64_t vi2 = ((int64_t)(zi - dzb * R) * R + (yi - dyb * R)) * R + (xi - dxb * R);
#pragma omp atomic write
                ms[(bi * R3 + vi2) * 4 + mqr_edge_shifts[i][3]] = -1;
            }
        }
    /* pass 1+2: vertices, numbered in block / voxel / edge order (count, scan, fill) */
    int64_t* off = (int64_t*)malloc(sizeof(int64_t) * (nblk > 0 ? nblk : 1));
#pragma omp parallel for schedule(static)
    for (int64_t b = 0; b < nblk; ++b) {
        int64_t c = 0;
        for (int64_t vi = 0; vi < R3; ++vi) {
            const int32_t* m = ms + (b * R3 + vi) * 4;
            c += (m[0] == -1) + (m[1] == -1) + (m[2] == -1);
        }
        off[b] = c;
    }
    const int64_t vcnt = excl_scan(off, nblk);
    float* vtx = (float*)malloc(sizeof(float) * 3 * (vcnt > 0 ? vcnt : 1));
    float* nrm = (float*)malloc(sizeof(float) * 3 * (vcnt > 0 ? vcnt : 1));
#pragma omp parallel for schedule(dynamic, 16)
    for (int64_t b = 0; b < nblk; ++b) {
        int64_t vc = off[b];
        int32_t xb = v->keys[3 * b], yb = v->keys[3 * b + 1], zb = v->keys[3 * b + 2];
        for (int64_t vi = 0; vi < R3; ++vi) {
            int32_t* m = ms + (b * R3 + vi) * 4;
            if (m[0] != -1 && m[1] != -1 && m[2] != -1) continue;
            int xv = (int)(vi % R), yv = (int)((vi / R) % R), zv = (int)(vi / (R * R));
            int32_t x = xb * R + xv, y = yb * R + yv, z = zb * R + zv;
            float tsdf_o = v->tsdf[b * R3 + vi];
            float no[3] = {0, 0, 0}, ne[3] = {0, 0, 0};
            get_normal(v, nb, b, xv, yv, zv, no);
            for (int e = 0; e < 3; ++e) {
                if (m[e] != -1) continue;
                int64_t lie = lin_idx(v, nb, b, xv + (e == 0), yv + (e == 1), zv + (e == 2));
                float tsdf_e = v->tsdf[lie];
                float ratio = (0 - tsdf_o) / (tsdf_e - tsdf_o);
                m[e] = (int32_t)vc;
                float rx = ratio * (int)(e == 0), ry = ratio * (int)(e == 1), rz = ratio * (int)(e == 2);
                vtx[3 * vc + 0] = v->voxel_size * (x + rx);
                vtx[3 * vc + 1] = v->voxel_size * (y + ry);
                vtx[3 * vc + 2] = v->voxel_size * (z + rz);
                get_normal(v, nb, b, xv + (e == 0), yv + (e == 1), zv + (e == 2), ne);
                float nx = (1 - ratio) * no[0] + ratio * ne[0];
                float ny = (1 - ratio) * no[1] + ratio * ne[1];
                float nz = (1 - ratio) * no[2] + ratio * ne[2];
                normalize_into(nx, ny, nz, nrm + 3 * vc);
                ++vc;
            }
        }
    }
    /* pass 3: triangles (vertex order reversed, tri[2 - k]), block / voxel order */
#pragma omp parallel for schedule(static)
    for (int64_t b = 0; b < nblk; ++b) {
        int64_t c = 0;
        for (int64_t vi = 0; vi < R3; ++vi) c += mqr_tri_count[ms[(b * R3 + vi) * 4 + 3]];
        off[b] = c;
    }
    const int64_t tcnt = excl_scan(off, nblk);
    int32_t* tri = (int32_t*)malloc(sizeof(int32_t) * 3 * (tcnt > 0 ? tcnt : 1));
#pragma omp parallel for schedule(dynamic, 16)
    for (int64_t b = 0; b < nblk; ++b) {
        int64_t tc = off[b];
        for (int64_t vi = 0; vi < R3; ++vi) {
            int table_idx = ms[(b * R3 + vi) * 4 + 3];
            if (mqr_tri_count[table_idx] == 0) continue;
            int xv = (int)(vi % R), yv = (int)((vi / R) % R), zv = (int)(vi / (R * R));
            for (int t = 0; t < 16; t += 3) {
                if (mqr_tri_table[table_idx][t] == -1) break;
                for (int k = 0; k < 3; ++k) {
                    int edge = mqr_tri_table[table_idx][t + k];
                    int xi = xv + mqr_edge_shifts[edge][0], yi = yv + mqr_edge_shifts[edge][1],
                        zi = zv + mqr_edge_shifts[edge][2];
                    int dxb = xi / R, dyb = yi / R, dzb = zi / R;
                    int kk = (dxb + 1) + (dyb + 1) * 3 + (dzb + 1) * 9;
                    int64_t bi = nb[b * 27 + kk];
                    int64_t vi2 = ((int64_t)(zi - dzb * R) * R + (yi - dyb * R)) * R + (xi - dxb * R);
                    tri[3 * tc + (2 - k)] = ms[(bi * R3 + vi2) * 4 + mqr_edge_shifts[edge][3]];
                }
                ++tc;
            }
        }
    }
    free(off);
    free(ms);
    free(nb);
    *vtx_out = vtx;
    *nrm_out = nrm;
    *tri_out = tri;
    *ntri_out = tcnt;
    return vcnt;
}

void orc_free(void* p) { free(p); }

/* ---------------- depth confidence (numpy restatement, float64) ---------------- */

/* One (ref pixel, target frame) evaluation of compute_pixel_error_map.py:120-220.
 * Returns 1 and writes the float32 error when the pixel gets a finite error, else 0 (NaN). */
static int pixel_error(const float* tgt_depth, int H, int W, const float* Kr, const float* Kt, const float* Tr,
                       const float* Tti, const float* Tt, double depth_max, int u, int v, float dref, float* err) {
    const float dmf = (float)depth_max;
    if (!(dref > 0 && dref <= dmf)) return 0;
    /* depth_to_pointcloud_numpy (:95-117): int64 - float32 -> float64 */
    double z = (double)dref;
    double x = (((double)u - (double)Kr[2]) * z) / (double)Kr[0];
    double y = (((double)v - (double)Kr[5]) * z) / (double)Kr[4];
    double pw[3];
    for (int i = 0; i < 3; ++i)
        pw[i] = (double)Tr[i * 4 + 0] * x + (double)Tr[i * 4 + 1] * y + (double)Tr[i * 4 + 2] * z + (double)Tr[i * 4 + 3] * 1.0;
    /* world -> target camera (:141-143) */
    double pt[3];
    for (int i = 0; i < 3; ++i)
        pt[i] = (double)Tti[i * 4 + 0] * pw[0] + (double)Tti[i * 4 + 1] * pw[1] + (double)Tti[i * 4 + 2] * pw[2] +
                (double)Tti[i * 4 + 3] * 1.0;
    double X = pt[0], Y = pt[1], Z = pt[2];
    if (!(Z > 0 && isfinite(Z) && Z <= depth_max && isfinite(X) && isfinite(Y))) return 0;
    double fx = (double)Kt[0], fy = (double)Kt[4], cx = (double)Kt[2], cy = (double)Kt[5];
    double uu = ((X * fx) / Z) + cx;
    double vv = ((Y * fy) / Z) + cy;
    if (!(isfinite(uu) && isfinite(vv))) return 0;
    /* bilinear_interpolate_depth (:4-92) */
    double max_coord = (double)((W > H ? W : H) * 10);
    if (!(uu >= -max_coord && uu < max_coord && vv >= -max_coord && vv < max_coord)) return 0;
    double uf = floor(uu), vf = floor(vv);
    int u0 = (int)uf, v0 = (int)vf, u1 = u0 + 1, v1 = v0 + 1;
    if (!(u0 >= 0 && u1 < W && v0 >= 0 && v1 < H)) return 0;
    float Ia = tgt_depth[(int64_t)v0 * W + u0], Ib = tgt_depth[(int64_t)v0 * W + u1];
    float Ic = tgt_depth[(int64_t)v1 * W + u0], Id = tgt_depth[(int64_t)v1 * W + u1];
    if (!(Ib > 0 && Ib <= dmf && Ia > 0 && Ia <= dmf && Ic > 0 && Ic <= dmf && Id > 0 && Id <= dmf)) return 0;
    double wa = ((double)u1 - uu) * ((double)v1 - vv);
    double wb = (uu - (double)u0) * ((double)v1 - vv);
    double wc = ((double)u1 - uu) * (vv - (double)v0);
    double wd = (uu - (double)u0) * (vv - (double)v0);
    float zt = (float)(wa * Ia + wb * Ib + wc * Ic + wd * Id);
    if (!(zt > 0 && isfinite(zt))) return 0;
    /* back-project the target pixel (:184-193) */
    double ztd = (double)zt;
    double xt = ((uu - cx) * ztd) / fx;
    double yt = ((vv - cy) * ztd) / fy;
    double pw2[3];
    for (int i = 0; i < 3; ++i)
        pw2[i] = (double)Tt[i * 4 + 0] * xt + (double)Tt[i * 4 + 1] * yt + (double)Tt[i * 4 + 2] * ztd +
                 (double)Tt[i * 4 + 3] * 1.0;
    double dx = pw[0] - pw2[0], dy = pw[1] - pw2[1], dz = pw[2] - pw2[2];
    *err = (float)sqrt(dx * dx + dy * dy + dz * dz);
    return 1;
}

/* compute_pixel_error_map for one (ref, tgt) pair; err_out H*W float32, NaN where invalid. */
int orc_pixel_error_map(const float* ref_depth, const float* tgt_depth, int H, int W, const float* Kr, const float* Kt,
                        const float* Tr, const float* Tti, const float* Tt, double depth_max, float* err_out) {
#pragma omp parallel for schedule(static)
    for (int64_t p = 0; p < (int64_t)H * W; ++p) {
        float e;
        int u = (int)(p % W), v = (int)(p / W);
        err_out[p] = pixel_error(tgt_depth, H, W, Kr, Kt, Tr, Tti, Tt, depth_max, u, v, ref_depth[p], &e) ? e : NAN;
    }
    return 0;
}

/*
 * build_confidence_map (estimate_depth_confidences.py:15-79) for reference frame `ref` of an
 * N-frame sequence.  depths: N*H*W metric float32; frame_valid[i]==0 marks frames whose load
 * failed (skipped as neighbours).  K: N*9, Tcw: N*16 (camera->world), Tcw_inv: N*16 (float32,
 * np.linalg.inv of Tcw).  conf: float64 H*W, valid: int32 H*W.
 */
int orc_confidence(const float* depths, const uint8_t* frame_valid, const float* K, const float* Tcw,
                   const float* Tcw_inv, int N, int H, int W, int ref, int r, double depth_max, double err_thr,
                   double* conf, int32_t* valid) {
    const int64_t HW = (int64_t)H * W;
    const float thr = (float)err_thr;
    int lo = ref - r > 0 ? ref - r : 0, hi = ref + r + 1 < N ? ref + r + 1 : N;
    const float* refd = depths + (int64_t)ref * HW;
#pragma omp parallel for schedule(static)
    for (int64_t p = 0; p < HW; ++p) {
        int u = (int)(p % W), v = (int)(p / W);
        int32_t nv = 0, nc = 0;
        for (int t = lo; t < hi; ++t) {
            if (t == ref || (frame_valid && !frame_valid[t])) continue;
            float e;
            if (pixel_error(depths + (int64_t)t * HW, H, W, K + 9 * ref, K + 9 * t, Tcw + 16 * ref, Tcw_inv + 16 * t,
                            Tcw + 16 * t, depth_max, u, v, refd[p], &e) &&
                !isnan(e)) {  /* valid_count += ~isnan(error_map) (estimate_depth_confidences.py:66) */
                ++nv;
                if (e <= thr) ++nc;
            }
        }
        valid[p] = nv;
        conf[p] = nv == 0 ? 0.0 : (double)nc / (double)nv;
    }
    return 0;
}

/* ------------------------------------------------------------------ ray casting (row f1)
 * Restates what the reference reads from Open3D's RaycastingScene (o3d_utils.py:324-341):
 * closest hit t in (0, inf) of each ray (origin, direction) against every triangle, inf on a
 * miss, with the primitive index.  Brute force, Moeller-Trumbore in float64 (the exact geometric
 * answer up to float64 rounding), OpenMP over rays.  Parity against Embree itself is unpinned
 * (Open3D is not installed); the GPU kernel is checked against this to a tolerance. */
int orc_raycast(const float* V, int64_t nv, const int32_t* T, int64_t nt, const float* rays, int64_t nrays,
                float* t_hit, int32_t* prim) {
    (void)nv;
#pragma omp parallel for schedule(dynamic, 64)
    for (int64_t r = 0; r < nrays; ++r) {
        const double o[3] = {rays[6 * r], rays[6 * r + 1], rays[6 * r + 2]};
        const double d[3] = {rays[6 * r + 3], rays[6 * r + 4], rays[6 * r + 5]};
        double best = INFINITY;
        int32_t bp = -1;
        for (int64_t i = 0; i < nt; ++i) {
            const float* a = V + 3 * (int64_t)T[3 * i];
            const float* b = V + 3 * (int64_t)T[3 * i + 1];
            const float* c = V + 3 * (int64_t)T[3 * i + 2];
            const double e1[3] = {(double)b[0] - a[0], (double)b[1] - a[1], (double)b[2] - a[2]};
            const double e2[3] = {(double)c[0] - a[0], (double)c[1] - a[1], (double)c[2] - a[2]};
            const double p[3] = {d[1] * e2[2] - d[2] * e2[1], d[2] * e2[0] - d[0] * e2[2], d[0] * e2[1] - d[1] * e2[0]};
            const double det = e1[0] * p[0] + e1[1] * p[1] + e1[2] * p[2];
            if (det == 0.0) continue;
            const double inv = 1.0 / det;
            const double tv[3] = {o[0] - a[0], o[1] - a[1], o[2] - a[2]};
            const double u = (tv[0] * p[0] + tv[1] * p[1] + tv[2] * p[2]) * inv;
            if (u < 0.0 || u > 1.0) continue;
            const double q[3] = {tv[1] * e1[2] - tv[2] * e1[1], tv[2] * e1[0] - tv[0] * e1[2],
                                 tv[0] * e1[1] - tv[1] * e1[0]};
            const double v = (d[0] * q[0] + d[1] * q[1] + d[2] * q[2]) * inv;
            if (v < 0.0 || u + v > 1.0) continue;
            const double t = (e2[0] * q[0] + e2[1] * q[1] + e2[2] * q[2]) * inv;
            if (t > 0.0 && t < best) {
                best = t;
                bp = (int32_t)i;
            }
        }
        t_hit[r] = (float)best;
        if (prim) prim[r] = bp;
    }
    return 0;
}

/* ------------------------------------------------------------------ per-vertex colour (row f1)
 * The colour averaging of Open3D's colour-map pipeline as the reference feeds it
 * (optimize_color_pose.py:24-73: extracted mesh + colour keyframes + ray-cast colour-aligned
 * depth -> run_rigid_optimizer); upstream ColorMapUtils.cpp CreateVertexAndImageVisibility +
 * SetGeometryColorAverage, recalled (Open3D is not installed here: parity unpinned, VERIFY).
 * Float64 projection Vt = T [X 1], u = float(Vt.x fx / Vt.z + cx), v likewise, d = float(Vt.z);
 * visible iff d >= 0, (round u, round v) in the image, depth there <= max_depth and
 * |d - depth| < thr; sampled iff also margin <= u < W - margin, margin <= v < H - margin;
 * colour = mean of (float)rgb / 255.0f over sampled keyframes (float64 sums in keyframe order), 0 if none.
 * The depth-discontinuity mask and the knn fill of unseen vertices are not restated. */
int orc_color_vertices(const float* V, int64_t nv, const uint8_t* images, const float* depths, int N, int H, int W,
                       const double* K, const double* T, double max_depth, double thr, int margin, float* out,
                       int32_t* counts) {
    const int64_t HW = (int64_t)H * W;
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < nv; ++i) {
        const double X = V[3 * i], Y = V[3 * i + 1], Z = V[3 * i + 2];
        double sr = 0.0, sg = 0.0, sb = 0.0;
        int cnt = 0;
        for (int c = 0; c < N; ++c) {
            const double* E = T + 16 * c;
            const double vx = E[0] * X + E[1] * Y + E[2] * Z + E[3];
            const double vy = E[4] * X + E[5] * Y + E[6] * Z + E[7];
            const double vz = E[8] * X + E[9] * Y + E[10] * Z + E[11];
            const float u = (float)((vx * K[9 * c]) / vz + K[9 * c + 2]);
            const float v = (float)((vy * K[9 * c + 4]) / vz + K[9 * c + 5]);
            const float d = (float)vz;
            const int ui = (int)roundf(u), vi = (int)roundf(v);
            if (d < 0.0f || ui < 0 || ui >= W || vi < 0 || vi >= H) continue;
            const int64_t px = (int64_t)c * HW + (int64_t)vi * W + ui;
            const float ds = depths[px];
            if (ds > max_depth) continue;
            if (!((double)fabsf(d - ds) < thr)) continue;
            if (!(u >= margin && u < W - margin && v >= margin && v < H - margin)) continue;
            const uint8_t* p = images + 3 * px;
            sr += (double)((float)p[0] / 255.0f);
            sg += (double)((float)p[1] / 255.0f);
            sb += (double)((float)p[2] / 255.0f);
            ++cnt;
        }
        out[3 * i] = cnt ? (float)(sr / cnt) : 0.f;
        out[3 * i + 1] = cnt ? (float)(sg / cnt) : 0.f;
        out[3 * i + 2] = cnt ? (float)(sb / cnt) : 0.f;
        if (counts) counts[i] = cnt;
    }
    return 0;
}

/* ------------------------------------------------------------------ colour map (row f1, complete)
 * What run_rigid_optimizer (optimize_color_pose.py:70-73) does to the vertex colours with the
 * keyframe poses as given (its pose refinement is OUT of scope, i.e. maximum_iteration = 0), from
 * upstream Open3D 0.19 ColorMapUtils.cpp / RigidOptimizer.cpp / Image.cpp as recalled (Open3D is not
 * installed here: parity unpinned, every rule VERIFY):
 *   RGBD depth: RGBDImage.create_from_color_and_depth(depth_scale = 1.0) -> d = t_hit / 1.0,
 *     d >= depth_trunc (3.0) -> 0 (misses, t_hit = inf, too);
 *   boundary mask (CreateDepthBoundaryMasks): dx = Filter(Sobel31 horizontal, Sobel32 vertical),
 *     dy = Filter(Sobel32, Sobel31) -- each pass per pixel temp (double) += (float)(d * (float)k)
 *     over the clamped 3-tap window, stored as float -- mask = sqrt(dx^2 + dy^2) > disc_thr (0.1),
 *     then Dilate(half = 3): 255 where any pixel of the (2 half + 1)^2 window inside the image is;
 *   visibility (CreateVertexAndImageVisibility): as orc_color_vertices plus mask(ui, vi) != 255;
 *   colour (SetGeometryColorAverage): the float64 mean over sampled keyframes of (float)rgb / 255.0f;
 *     a vertex no keyframe samples gets the float64 mean of the colours of its knn (3) nearest
 *     sampled vertices (KDTreeFlann over the sampled vertices; ties of the squared distance broken
 *     here by the lower vertex index -- VERIFY against nanoflann's visiting order).
 * Output colours float32 of the float64 values; counts = keyframes averaged (0 for filled ones). */

static void sobel_pass(const float* in, float* out, int H, int W, const float* k, int vertical) {
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            double temp = 0;
            for (int i = -1; i <= 1; ++i) {
                int xs = x, ys = y;
                if (vertical) {
                    ys = y + i;
                    if (ys < 0) ys = 0;
                    if (ys > H - 1) ys = H - 1;
                } else {
                    xs = x + i;
                    if (xs < 0) xs = 0;
                    if (xs > W - 1) xs = W - 1;
                }
                temp += (in[(int64_t)ys * W + xs] * k[i + 1]);
            }
            out[(int64_t)y * W + x] = (float)temp;
        }
}

int orc_depth_boundary_mask(const float* t_hit, int H, int W, double depth_trunc, double disc_thr, int half,
                            float* depth_out, uint8_t* mask_out) {
    const int64_t HW = (int64_t)H * W;
    static const float s31[3] = {-1.0f, 0.0f, 1.0f}, s32[3] = {1.0f, 2.0f, 1.0f};
    float* d = depth_out;
    float* a = (float*)malloc(sizeof(float) * HW);
    float* b = (float*)malloc(sizeof(float) * HW);
    float* gx = (float*)malloc(sizeof(float) * HW);
    uint8_t* m0 = (uint8_t*)malloc(HW);
    for (int64_t p = 0; p < HW; ++p) {
        float v = t_hit[p] / (float)1.0;
        d[p] = v >= depth_trunc ? 0.0f : v;
    }
    sobel_pass(d, a, H, W, s31, 0);  /* dx: Sobel31 along x, then Sobel32 along y */
    sobel_pass(a, gx, H, W, s32, 1);
    sobel_pass(d, a, H, W, s32, 0);  /* dy: Sobel32 along x, then Sobel31 along y */
    sobel_pass(a, b, H, W, s31, 1);
    for (int64_t p = 0; p < HW; ++p) {
        double dx = gx[p], dy = b[p];
        m0[p] = sqrt(dx * dx + dy * dy) > disc_thr ? 255 : 0;
    }
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            uint8_t o = 0;
            for (int yy = -half; yy <= half && !o; ++yy)
                for (int xx = -half; xx <= half; ++xx) {
                    int u = x + xx, v = y + yy;
                    if (u >= 0 && u < W && v >= 0 && v < H && m0[(int64_t)v * W + u] == 255) {
                        o = 255;
                        break;
                    }
                }
            mask_out[(int64_t)y * W + x] = o;
        }
    free(a);
    free(b);
    free(gx);
    free(m0);
    return 0;
}

/* ---- exact knn over the sampled vertices: implicit k-d tree (node = index range, split at the
 * middle element along the widest axis), best list ordered by (squared distance, vertex index) */
typedef struct {
    const double* P; /* 3 per point */
    int32_t* idx;    /* point ids, reordered */
    uint8_t* axis;   /* split axis of the node whose middle element is this position (unused by the search) */
    double* split;   /* its split value, recorded at build time (the children's builds reorder idx) */
    double* box;     /* 12 per node position: tight boxes (min xyz, max xyz) of [lo, mid) and [mid, hi) --
                      * the search prunes a child by its box distance: with the split plane alone a
                      * query far from a compact point set visits every node */
} kdtree;

static void kd_bounds(const kdtree* t, int64_t lo, int64_t hi, double* b) {
    b[0] = b[1] = b[2] = INFINITY;
    b[3] = b[4] = b[5] = -INFINITY;
    for (int64_t i = lo; i < hi; ++i)
        for (int a = 0; a < 3; ++a) {
            const double v = t->P[3 * t->idx[i] + a];
            if (v < b[a]) b[a] = v;
            if (v > b[3 + a]) b[3 + a] = v;
        }
}

/* squared distance from q to the box b (0 inside) */
static double box_d2(const double* q, const double* b) {
    double s = 0.0;
    for (int a = 0; a < 3; ++a) {
        const double d = q[a] < b[a] ? b[a] - q[a] : (q[a] > b[3 + a] ? q[a] - b[3 + a] : 0.0);
        s += d * d;
    }
    return s;
}

/* (value on axis, point id) order */
static int kd_less(const double* P, int32_t i, int32_t j, int ax) {
    const double x = P[3 * i + ax], y = P[3 * j + ax];
    return x < y || (x == y && i < j);
}

/* Quickselect: idx[mid] gets the element of rank mid - lo in [lo, hi), smaller ones before it,
 * larger after (O(n) expected per call; the tree build is O(n log n)). */
static void kd_select(const double* P, int32_t* idx, int64_t lo, int64_t hi, int64_t mid, int ax) {
    uint64_t seed = 0x9e3779b97f4a7c15ull ^ (uint64_t)lo ^ ((uint64_t)hi << 20);
    while (hi - lo > 1) {
        seed = seed * 6364136223846793005ull + 1442695040888963407ull;
        const int64_t pv = lo + (int64_t)((seed >> 33) % (uint64_t)(hi - lo));
        int32_t tmp = idx[pv];
        idx[pv] = idx[hi - 1];
        idx[hi - 1] = tmp;
        const int32_t piv = idx[hi - 1];
        int64_t st = lo;
        for (int64_t i = lo; i < hi - 1; ++i)
            if (kd_less(P, idx[i], piv, ax)) {
                tmp = idx[i];
                idx[i] = idx[st];
                idx[st] = tmp;
                ++st;
            }
        idx[hi - 1] = idx[st];
        idx[st] = piv;
        if (st == mid) return;
        if (st < mid) lo = st + 1;
        else hi = st;
    }
}

static void kd_build(kdtree* t, int64_t lo, int64_t hi) {
    if (hi - lo <= 8) return;
    double mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int64_t i = lo; i < hi; ++i)
        for (int a = 0; a < 3; ++a) {
            double v = t->P[3 * t->idx[i] + a];
            if (v < mn[a]) mn[a] = v;
            if (v > mx[a]) mx[a] = v;
        }
    int ax = 0;
    for (int a = 1; a < 3; ++a)
        if (mx[a] - mn[a] > mx[ax] - mn[ax]) ax = a;
    const int64_t mid = (lo + hi) / 2;
    kd_select(t->P, t->idx, lo, hi, mid, ax);
    t->axis[mid] = (uint8_t)ax;
    t->split[mid] = t->P[3 * t->idx[mid] + ax];
    kd_bounds(t, lo, mid, t->box + 12 * mid);
    kd_bounds(t, mid, hi, t->box + 12 * mid + 6);
    kd_build(t, lo, mid);
    kd_build(t, mid, hi);
}

typedef struct {
    double d2[8];
    int32_t id[8];
    int n, k;
} kbest;

static void kb_push(kbest* b, double d2, int32_t id) {
    if (b->n == b->k && !(d2 < b->d2[b->n - 1] || (d2 == b->d2[b->n - 1] && id < b->id[b->n - 1]))) return;
    int j = b->n < b->k ? b->n++ : b->n - 1;
    while (j > 0 && (d2 < b->d2[j - 1] || (d2 == b->d2[j - 1] && id < b->id[j - 1]))) {
        b->d2[j] = b->d2[j - 1];
        b->id[j] = b->id[j - 1];
        --j;
    }
    b->d2[j] = d2;
    b->id[j] = id;
}

static double sq3(const double* q, const double* p) {
    double dx = q[0] - p[0], dy = q[1] - p[1], dz = q[2] - p[2];
    return dx * dx + dy * dy + dz * dz;
}

static void kd_search(const kdtree* t, int64_t lo, int64_t hi, const double* q, kbest* b) {
    if (hi - lo <= 8) {
        for (int64_t i = lo; i < hi; ++i) kb_push(b, sq3(q, t->P + 3 * t->idx[i]), t->idx[i]);
        return;
    }
    const int64_t mid = (lo + hi) / 2;
    /* nearer child (by box distance) first; a child is visited while its box is not farther than the
     * current k-th distance (<=: equal distances still compete by vertex index) */
    const double dl = box_d2(q, t->box + 12 * mid), dr = box_d2(q, t->box + 12 * mid + 6);
    const int left_first = dl <= dr;
    for (int pass = 0; pass < 2; ++pass) {
        const int left = pass == 0 ? left_first : !left_first;
        const double dc = left ? dl : dr;
        if (b->n < b->k || dc <= b->d2[b->n - 1]) {
            if (left) kd_search(t, lo, mid, q, b);
            else kd_search(t, mid, hi, q, b);
        }
    }
}

int orc_color_map(const float* V, int64_t nv, const uint8_t* images, const float* t_hit, int N, int H, int W,
                  const double* K, const double* T, double max_depth, double thr, int margin, double disc_thr,
                  int half, double depth_trunc, int knn, float* out, int32_t* counts) {
    const int64_t HW = (int64_t)H * W;
    float* depth = (float*)malloc(sizeof(float) * HW * (N > 0 ? N : 1));
    uint8_t* mask = (uint8_t*)malloc(HW * (N > 0 ? N : 1));
    for (int c = 0; c < N; ++c)
        orc_depth_boundary_mask(t_hit + c * HW, H, W, depth_trunc, disc_thr, half, depth + c * HW, mask + c * HW);
    double* avg = (double*)malloc(sizeof(double) * 3 * (nv > 0 ? nv : 1));
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < nv; ++i) {
        const double X = V[3 * i], Y = V[3 * i + 1], Z = V[3 * i + 2];
        double sr = 0.0, sg = 0.0, sb = 0.0;
        int cnt = 0;
        for (int c = 0; c < N; ++c) {
            const double* E = T + 16 * c;
            const double vx = E[0] * X + E[1] * Y + E[2] * Z + E[3];
            const double vy = E[4] * X + E[5] * Y + E[6] * Z + E[7];
            const double vz = E[8] * X + E[9] * Y + E[10] * Z + E[11];
            const float u = (float)((vx * K[9 * c]) / vz + K[9 * c + 2]);
            const float v = (float)((vy * K[9 * c + 4]) / vz + K[9 * c + 5]);
            const float d = (float)vz;
            const int ui = (int)roundf(u), vi = (int)roundf(v);
            if (d < 0.0f || ui < 0 || ui >= W || vi < 0 || vi >= H) continue;
            const int64_t px = (int64_t)c * HW + (int64_t)vi * W + ui;
            const float ds = depth[px];
            if (ds > max_depth) continue;
            if (mask[px] == 255) continue;
            if (!((double)fabsf(d - ds) < thr)) continue;
            if (!(u >= margin && u < W - margin && v >= margin && v < H - margin)) continue;
            const uint8_t* p = images + 3 * px;
            sr += (double)((float)p[0] / 255.0f);
            sg += (double)((float)p[1] / 255.0f);
            sb += (double)((float)p[2] / 255.0f);
            ++cnt;
        }
        avg[3 * i] = cnt ? sr / cnt : 0.0;
        avg[3 * i + 1] = cnt ? sg / cnt : 0.0;
        avg[3 * i + 2] = cnt ? sb / cnt : 0.0;
        counts[i] = cnt;
    }
    int64_t nvalid = 0;
    for (int64_t i = 0; i < nv; ++i) nvalid += counts[i] > 0;
    double* P = (double*)malloc(sizeof(double) * 3 * (nv > 0 ? nv : 1));
    for (int64_t i = 0; i < 3 * nv; ++i) P[i] = V[i];
    kdtree t = {P, (int32_t*)malloc(sizeof(int32_t) * (nvalid > 0 ? nvalid : 1)), (uint8_t*)calloc(nvalid + 1, 1),
                (double*)calloc(nvalid + 1, sizeof(double)), (double*)calloc(12 * (nvalid + 1), sizeof(double))};
    int64_t j = 0;
    for (int64_t i = 0; i < nv; ++i)
        if (counts[i] > 0) t.idx[j++] = (int32_t)i;
    kd_build(&t, 0, nvalid);
    if (knn > 8) knn = 8;
#pragma omp parallel for schedule(dynamic, 256)
    for (int64_t i = 0; i < nv; ++i) {
        double c[3] = {avg[3 * i], avg[3 * i + 1], avg[3 * i + 2]};
        if (counts[i] == 0 && knn > 0 && nvalid > 0) {
            kbest b;
            b.n = 0;
            b.k = knn;
            kd_search(&t, 0, nvalid, P + 3 * i, &b);
            c[0] = c[1] = c[2] = 0.0;
            for (int q = 0; q < b.n; ++q)
                for (int a = 0; a < 3; ++a) c[a] += avg[3 * b.id[q] + a];
            for (int a = 0; a < 3; ++a) c[a] /= (double)b.n;
        }
        for (int a = 0; a < 3; ++a) out[3 * i + a] = (float)c[a];
    }
    free(t.idx);
    free(t.axis);
    free(t.split);
    free(t.box);
    free(P);
    free(avg);
    free(depth);
    free(mask);
    return 0;
}

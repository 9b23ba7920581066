// raycast.hip -- triangle-mesh ray casting for colour-aligned depth.
//
// Replaces Open3D's RaycastingScene as the reference uses it:
//   scene = o3d.t.geometry.RaycastingScene(); scene.add_triangles(mesh)   reconstruct_scene.py:197-198
//   rays = scene.create_rays_pinhole(K, T_wc, width_px, height_px)        o3d_utils.py:324-341
//   t_hit = scene.cast_rays(rays)['t_hit']                                (colour-aligned depth maps)
//
// MI355X design: the mesh (V vertices, T triangles, HBM-resident) gets a linear BVH built on the
// device (Karras 2012): 63-bit Morton codes of triangle centroids -> hipcub radix sort -> binary
// radix tree in one pass -> bottom-up box refit with per-node arrival counters.  Every internal
// node stores both children's boxes (one 64-byte node fetch per traversal step tests both
// children).  Leaves are single triangles stored in sort order as (v0, e1, e2) float4 triples.
// Queries: one thread per ray, short stack, nearest-first descent, Moeller-Trumbore hit test,
// closest hit with 0 < t < inf (Embree's tnear = 0, tfar = inf; no back-face culling).  Pinhole
// rays are generated on the device from (K, T_wc) exactly like CreateRaysPinhole -- origin
// C = -R^T t (float64, stored float32), direction = float32(R^T K^-1) * (x + 0.5, y + 0.5, 1) -- so
// t_hit is the camera-frame z depth of the hit.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <vector>

#include "mqr_common.hpp"
#include "device_block.hpp"

struct mqr_scene {
    int device = 0;
    hipStream_t stream = nullptr;
    struct Geom {
        float* v = nullptr;     // device, 3 * nv
        int32_t* t = nullptr;   // device, 3 * nt
        int64_t nv = 0, nt = 0;
    };
    std::vector<Geom> geoms;
    bool built = false;
    int64_t ntri = 0;
    float4* leaf = nullptr;     // [ntri][3]: (v0, prim id bits), (e1, geom id bits), (e2, 0)
    float4* node = nullptr;     // [ntri-1][4]: lo0, hi0, lo1, hi1 (w of lo0/lo1 = child index bits)
    void* bvh_blk = nullptr;    // leaf and node: one block of the device-block cache (geom_block_alloc)
    size_t bvh_cap = 0;
};

namespace mqr {

constexpr uint32_t kInvalidId = 0xffffffffu;

// ------------------------------------------------------------------ build
__device__ inline uint32_t f2ord(float f) {  // order-preserving float -> uint32
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ inline float ord2f(uint32_t u) { return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u); }

struct BuildTri {
    float v[9];
};

// Gather every geometry's triangles into one array (prim id / geom id kept) and accumulate the
// centroid bounds (ordered-int atomics).
// Centroid bounds: a wave-wide min / max, then a workgroup-wide one (block_bounds_atomic).
__device__ inline uint32_t wave_min_u32(uint32_t x) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) x = min(x, (uint32_t)__shfl_xor((int)x, o, 64));
    return x;
}
__device__ inline uint32_t wave_max_u32(uint32_t x) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) x = max(x, (uint32_t)__shfl_xor((int)x, o, 64));
    return x;
}

// Min / max of a workgroup's per-thread bounds (256 threads) into out[0..2] / out[3..5] by one atomic per
// word and workgroup.
__device__ inline void block_bounds_atomic(uint32_t (&lo)[3], uint32_t (&hi)[3], uint32_t* out) {
    __shared__ uint32_t part[4][6];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const uint32_t wl = wave_min_u32(lo[a]), wh = wave_max_u32(hi[a]);
        if (lane == 0) {
            part[wave][a] = wl;
            part[wave][3 + a] = wh;
        }
    }
    __syncthreads();
    if (threadIdx.x < 6) {
        const int c = threadIdx.x;
        uint32_t r = part[0][c];
        for (int w = 1; w < 4; ++w) r = c < 3 ? min(r, part[w][c]) : max(r, part[w][c]);
        if (c < 3) atomicMin(&out[c], r);
        else atomicMax(&out[c], r);
    }
}

// Grid-stride over the triangles (a capped grid: one atomic per bound word and WORKGROUP -- per-wave
// atomics on the same six words serialised this kernel to 44 ms for C5's 41 M triangles,
// profiles/r05_c5_kernel_stats.csv).  256 threads per workgroup.
constexpr unsigned kGatherGrid = 4096;
__global__ __launch_bounds__(256) void k_gather_tris(const float* __restrict__ v, const int32_t* __restrict__ t,
                                                     int64_t nt, int64_t nv, int64_t base, uint32_t geom, BuildTri* tris,
                                                     uint32_t* prim, uint32_t* gid,
                                                     uint32_t* cbounds /* 6: min xyz, max xyz (ordered) */, int* bad) {
    uint32_t lo[3] = {0xffffffffu, 0xffffffffu, 0xffffffffu}, hi[3] = {0u, 0u, 0u};
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nt; i += (int64_t)gridDim.x * blockDim.x) {
        BuildTri b;
        float c[3] = {0.f, 0.f, 0.f};
        for (int k = 0; k < 3; ++k) {
            int32_t vi = t[3 * i + k];
            if (vi < 0 || vi >= nv) {
                atomicOr(bad, 1);
                vi = 0;
            }
            for (int a = 0; a < 3; ++a) {
                b.v[3 * k + a] = v[3 * (int64_t)vi + a];
                c[a] += b.v[3 * k + a];
            }
        }
        tris[base + i] = b;
        prim[base + i] = (uint32_t)i;
        gid[base + i] = geom;
        for (int a = 0; a < 3; ++a) {
            const uint32_t o = f2ord(c[a] * (1.0f / 3.0f));
            lo[a] = min(lo[a], o);
            hi[a] = max(hi[a], o);
        }
    }
    block_bounds_atomic(lo, hi, cbounds);
}

__device__ inline uint64_t spread21(uint32_t x) {
    uint64_t v = x & 0x1fffff;
    v = (v | v << 32) & 0x1f00000000ffffull;
    v = (v | v << 16) & 0x1f0000ff0000ffull;
    v = (v | v << 8) & 0x100f00f00f00f00full;
    v = (v | v << 4) & 0x10c30c30c30c30c3ull;
    v = (v | v << 2) & 0x1249249249249249ull;
    return v;
}

__global__ void k_morton(const BuildTri* __restrict__ tris, int64_t n, const uint32_t* __restrict__ cb, uint64_t* keys,
                         uint32_t* idx) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t q[3];
    for (int a = 0; a < 3; ++a) {
        const float lo = ord2f(cb[a]), hi = ord2f(cb[3 + a]);
        const float c = (tris[i].v[a] + tris[i].v[3 + a] + tris[i].v[6 + a]) * (1.0f / 3.0f);
        const float ext = hi - lo;
        float s = ext > 0 ? (c - lo) / ext : 0.f;
        s = fminf(fmaxf(s, 0.f), 1.f);
        q[a] = (uint32_t)fminf(s * 2097152.0f, 2097151.0f);
    }
    keys[i] = spread21(q[0]) << 2 | spread21(q[1]) << 1 | spread21(q[2]);
    idx[i] = (uint32_t)i;
}

// Karras 2012: internal node i covers a key range [first, last] and splits at the highest
// differing bit; duplicate keys are disambiguated by the index (64 + clz(i ^ j)).
__device__ inline int delta(const uint64_t* k, int64_t n, int64_t i, int64_t j) {
    if (j < 0 || j >= n) return -1;
    const uint64_t a = k[i], b = k[j];
    if (a == b) return 64 + __clzll((unsigned long long)(i ^ j));
    return __clzll((unsigned long long)(a ^ b));
}

// child encoding: >= 0 internal node, < 0 leaf ~index
__global__ void k_radix_tree(const uint64_t* __restrict__ keys, int64_t n, int32_t* child /* 2(n-1) */,
                             int32_t* parent /* (n-1) internal + n leaves */) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n - 1) return;
    const int d = delta(keys, n, i, i + 1) - delta(keys, n, i, i - 1) >= 0 ? 1 : -1;
    const int dmin = delta(keys, n, i, i - d);
    int64_t lmax = 2;
    while (delta(keys, n, i, i + lmax * d) > dmin) lmax <<= 1;
    int64_t l = 0;
    for (int64_t t = lmax >> 1; t >= 1; t >>= 1)
        if (delta(keys, n, i, i + (l + t) * d) > dmin) l += t;
    const int64_t j = i + l * d;
    const int dnode = delta(keys, n, i, j);
    int64_t s = 0;
    for (int64_t t = (l + 1) >> 1;; t = (t + 1) >> 1) {
        if (delta(keys, n, i, i + (s + t) * d) > dnode) s += t;
        if (t == 1) break;
    }
    const int64_t gamma = i + s * d + min(d, 0);
    const int64_t lo = min(i, j), hi = max(i, j);
    const int32_t c0 = lo == gamma ? ~(int32_t)gamma : (int32_t)gamma;
    const int32_t c1 = hi == gamma + 1 ? ~(int32_t)(gamma + 1) : (int32_t)(gamma + 1);
    child[2 * i] = c0;
    child[2 * i + 1] = c1;
    parent[c0 >= 0 ? c0 : (n - 1) + ~c0] = (int32_t)i;
    parent[c1 >= 0 ? c1 : (n - 1) + ~c1] = (int32_t)i;
}

// Sorted leaves: v0 + primitive id, e1 + geometry id, e2.
__global__ void k_leaves(const BuildTri* __restrict__ tris, const uint32_t* __restrict__ prim,
                         const uint32_t* __restrict__ gid, const uint32_t* __restrict__ order, int64_t n, float4* leaf) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t o = order[i];
    const BuildTri b = tris[o];
    const float e1[3] = {b.v[3] - b.v[0], b.v[4] - b.v[1], b.v[5] - b.v[2]};
    const float e2[3] = {b.v[6] - b.v[0], b.v[7] - b.v[1], b.v[8] - b.v[2]};
    leaf[3 * i + 0] = make_float4(b.v[0], b.v[1], b.v[2], __uint_as_float(prim[o]));
    leaf[3 * i + 1] = make_float4(e1[0], e1[1], e1[2], __uint_as_float(gid[o]));
    leaf[3 * i + 2] = make_float4(e2[0], e2[1], e2[2], 0.f);
}

// Depth of every internal node (root 0), for the level-by-level refit.  The bottom-up refit with
// per-node arrival counters needs a device-scope fence per level so that a sibling on another XCD
// (whose L2 is not coherent with this one) sees the child box: on gfx950 every such fence writes
// back L2, which made that single kernel ~15 ms for 2 M triangles.  Kernel boundaries order the
// levels here instead (<= 96 levels: 63 key bits + 32 index bits + 1).
__global__ void k_node_depth(const int32_t* __restrict__ parent, int64_t m, uint32_t* depth, uint32_t* ids,
                             int* bad) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    uint32_t d = 0;
    for (int32_t x = parent[i]; x >= 0; x = parent[x]) ++d;
    if (d >= 256) atomicOr(bad, 2);
    depth[i] = d;
    ids[i] = (uint32_t)i;
}

__global__ void k_level_bounds(const uint32_t* __restrict__ ds, int64_t m, int* start, int* end) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const uint32_t d = ds[i] & 0xffu;
    if (i == 0 || (ds[i - 1] & 0xffu) != d) start[d] = (int)i;
    if (i == m - 1 || (ds[i + 1] & 0xffu) != d) end[d] = (int)(i + 1);
}

// Boxes of the nodes of one level (their children are leaves or deeper, already written).
__global__ void k_refit_level(const BuildTri* __restrict__ tris, const uint32_t* __restrict__ order,
                              const int32_t* __restrict__ child, const uint32_t* __restrict__ ids, int64_t cnt,
                              float4* node) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= cnt) return;
    const int32_t p = (int32_t)ids[k];
    {
        float lo[2][3], hi[2][3];
        for (int c = 0; c < 2; ++c) {
            const int32_t ch = child[2 * p + c];
            if (ch < 0) {
                const BuildTri t = tris[order[~ch]];
                for (int a = 0; a < 3; ++a) {
                    lo[c][a] = fminf(fminf(t.v[a], t.v[3 + a]), t.v[6 + a]);
                    hi[c][a] = fmaxf(fmaxf(t.v[a], t.v[3 + a]), t.v[6 + a]);
                }
            } else {
                const float4* cn = node + 4 * (int64_t)ch;  // written by an earlier level's launch
                const float4 l0 = cn[0], h0 = cn[1], l1 = cn[2], h1 = cn[3];
                lo[c][0] = fminf(l0.x, l1.x), lo[c][1] = fminf(l0.y, l1.y), lo[c][2] = fminf(l0.z, l1.z);
                hi[c][0] = fmaxf(h0.x, h1.x), hi[c][1] = fmaxf(h0.y, h1.y), hi[c][2] = fmaxf(h0.z, h1.z);
            }
        }
        float4* nd = node + 4 * (int64_t)p;
        nd[0] = make_float4(lo[0][0], lo[0][1], lo[0][2], __int_as_float(child[2 * p]));
        nd[1] = make_float4(hi[0][0], hi[0][1], hi[0][2], 0.f);
        nd[2] = make_float4(lo[1][0], lo[1][1], lo[1][2], __int_as_float(child[2 * p + 1]));
        nd[3] = make_float4(hi[1][0], hi[1][1], hi[1][2], 0.f);
    }
}

// ------------------------------------------------------------------ queries
struct Hit {
    float t, u, v;
    int32_t leaf;
};

__device__ inline bool slab(const float3 lo, const float3 hi, const float3 o, const float3 inv, float tmax,
                            float& tenter) {
    const float tx0 = (lo.x - o.x) * inv.x, tx1 = (hi.x - o.x) * inv.x;
    const float ty0 = (lo.y - o.y) * inv.y, ty1 = (hi.y - o.y) * inv.y;
    const float tz0 = (lo.z - o.z) * inv.z, tz1 = (hi.z - o.z) * inv.z;
    const float tn = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fmaxf(fminf(tz0, tz1), 0.0f));
    const float tf = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fminf(fmaxf(tz0, tz1), tmax));
    tenter = tn;
    return tn <= tf * 1.00000024f;  // 2 ulp slack: conservative box test
}

__device__ inline void tri_test(const float4* __restrict__ leaf, int32_t li, const float3 o, const float3 d, Hit& h) {
    const float4 a = leaf[3 * li], b = leaf[3 * li + 1], c = leaf[3 * li + 2];
    const float3 e1 = make_float3(b.x, b.y, b.z), e2 = make_float3(c.x, c.y, c.z);
    const float px = d.y * e2.z - d.z * e2.y, py = d.z * e2.x - d.x * e2.z, pz = d.x * e2.y - d.y * e2.x;
    const float det = e1.x * px + e1.y * py + e1.z * pz;
    if (det == 0.0f) return;
    const float inv = 1.0f / det;
    const float tx = o.x - a.x, ty = o.y - a.y, tz = o.z - a.z;
    const float u = (tx * px + ty * py + tz * pz) * inv;
    if (u < 0.0f || u > 1.0f) return;
    const float qx = ty * e1.z - tz * e1.y, qy = tz * e1.x - tx * e1.z, qz = tx * e1.y - ty * e1.x;
    const float v = (d.x * qx + d.y * qy + d.z * qz) * inv;
    if (v < 0.0f || u + v > 1.0f) return;
    const float t = (e2.x * qx + e2.y * qy + e2.z * qz) * inv;
    if (t > 0.0f && t < h.t) {
        h.t = t;
        h.u = u;
        h.v = v;
        h.leaf = li;
    }
}

__device__ Hit trace(const float4* __restrict__ node, const float4* __restrict__ leaf, int64_t n, float3 o, float3 d) {
    Hit h{INFINITY, 0.f, 0.f, -1};
    if (n == 1) {
        tri_test(leaf, 0, o, d, h);
        return h;
    }
    const float3 inv = make_float3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    int32_t stack[64];
    int sp = 0;
    int32_t cur = 0;
    while (true) {
        const float4* nd = node + 4 * (int64_t)cur;
        const float4 l0 = nd[0], h0 = nd[1], l1 = nd[2], h1 = nd[3];
        float t0, t1;
        const bool b0 = slab(make_float3(l0.x, l0.y, l0.z), make_float3(h0.x, h0.y, h0.z), o, inv, h.t, t0);
        const bool b1 = slab(make_float3(l1.x, l1.y, l1.z), make_float3(h1.x, h1.y, h1.z), o, inv, h.t, t1);
        int32_t c0 = __float_as_int(l0.w), c1 = __float_as_int(l1.w);
        if (b0 && c0 < 0) tri_test(leaf, ~c0, o, d, h);
        if (b1 && c1 < 0) tri_test(leaf, ~c1, o, d, h);
        const bool go0 = b0 && c0 >= 0 && t0 <= h.t, go1 = b1 && c1 >= 0 && t1 <= h.t;
        if (go0 && go1) {
            if (t1 < t0) {
                const int32_t tmp = c0;
                c0 = c1;
                c1 = tmp;
            }
            if (sp < 64) stack[sp++] = c1;
            cur = c0;
        } else if (go0) {
            cur = c0;
        } else if (go1) {
            cur = c1;
        } else {
            if (sp == 0) break;
            cur = stack[--sp];
        }
    }
    return h;
}

struct PinholeFrame {
    float m[9];  // float32(R^T K^-1), row-major
    float c[3];  // camera centre -R^T t (float64 -> float32)
};

__device__ inline void store_hit(const Hit& h, const float4* __restrict__ leaf, const float3 d, int64_t o,
                                 float* t_hit, uint32_t* geom_ids, uint32_t* prim_ids, float* uvs, float* normals) {
    t_hit[o] = h.t;
    if (geom_ids || prim_ids || uvs || normals) {
        uint32_t g = kInvalidId, p = kInvalidId;
        float u = 0.f, v = 0.f, nx = 0.f, ny = 0.f, nz = 0.f;
        if (h.leaf >= 0) {
            const float4 a = leaf[3 * h.leaf], b = leaf[3 * h.leaf + 1], c = leaf[3 * h.leaf + 2];
            p = __float_as_uint(a.w);
            g = __float_as_uint(b.w);
            u = h.u;
            v = h.v;
            nx = b.y * c.z - b.z * c.y, ny = b.z * c.x - b.x * c.z, nz = b.x * c.y - b.y * c.x;
            const float len = sqrtf(nx * nx + ny * ny + nz * nz);
            if (len > 0) nx /= len, ny /= len, nz /= len;
        }
        if (geom_ids) geom_ids[o] = g;
        if (prim_ids) prim_ids[o] = p;
        if (uvs) uvs[2 * o] = u, uvs[2 * o + 1] = v;
        if (normals) normals[3 * o] = nx, normals[3 * o + 1] = ny, normals[3 * o + 2] = nz;
    }
}

__global__ __launch_bounds__(256) void k_cast_pinhole(const float4* __restrict__ node, const float4* __restrict__ leaf,
                                                      int64_t n, const PinholeFrame* __restrict__ frames, int H,
                                                      int W, float* t_hit, uint32_t* geom_ids, uint32_t* prim_ids,
                                                      float* uvs, float* normals) {
    const int f = blockIdx.y;
    const int64_t HW = (int64_t)H * W;
    // (XCD bands -- workgroup bx remapped so that XCD bx mod 8 casts one eighth of the image -- ran
    // 15.0-16.1 vs 13.2-13.4 ms for 64 C2 frames, identical hits: the bands' traversal costs differ,
    // tools/raycast_workload.py, profiles/r04_ab_raycast_xcd.json)
    const unsigned bx = blockIdx.x;
    // 8x8 pixel tiles per wave keep a wave's rays coherent (same BVH paths)
    const int64_t tile = (int64_t)bx * 4 + (threadIdx.x >> 6);
    const int tiles_x = (W + 7) / 8;
    const int tx = (int)(tile % tiles_x), ty = (int)(tile / tiles_x);
    const int x = tx * 8 + (threadIdx.x & 7), y = ty * 8 + ((threadIdx.x >> 3) & 7);
    if (y >= H || x >= W) return;
    const PinholeFrame fr = frames[f];
    const float px = (float)x + 0.5f, py = (float)y + 0.5f;
    const float3 d = make_float3((fr.m[0] * px + fr.m[1] * py) + fr.m[2], (fr.m[3] * px + fr.m[4] * py) + fr.m[5],
                                 (fr.m[6] * px + fr.m[7] * py) + fr.m[8]);
    const float3 o = make_float3(fr.c[0], fr.c[1], fr.c[2]);
    const Hit h = trace(node, leaf, n, o, d);
    const int64_t oi = (int64_t)f * HW + (int64_t)y * W + x;
    store_hit(h, leaf, d, oi, t_hit, geom_ids, prim_ids, uvs, normals);
}

__global__ __launch_bounds__(256) void k_cast_rays(const float4* __restrict__ node, const float4* __restrict__ leaf,
                                                   int64_t n, const float* __restrict__ rays, int64_t nrays,
                                                   float* t_hit, uint32_t* geom_ids, uint32_t* prim_ids, float* uvs,
                                                   float* normals) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nrays) return;
    const float* r = rays + 6 * i;
    const float3 o = make_float3(r[0], r[1], r[2]), d = make_float3(r[3], r[4], r[5]);
    const Hit h = trace(node, leaf, n, o, d);
    store_hit(h, leaf, d, i, t_hit, geom_ids, prim_ids, uvs, normals);
}

// ------------------------------------------------------------------ host
static void free_built(mqr_scene* s) {
    geom_block_release(s->device, s->bvh_blk, s->bvh_cap);
    s->bvh_blk = nullptr;
    s->bvh_cap = 0;
    s->leaf = nullptr;
    s->node = nullptr;
    s->built = false;
}

static size_t al256(size_t x) { return (x + 255) & ~size_t(255); }


static int build(mqr_scene* s) {
    if (s->built) return 0;
    free_built(s);
    int64_t n = 0;
    for (auto& g : s->geoms) n += g.nt;
    MQR_REQUIRE(n > 0, "raycasting scene has no triangles");
    MQR_REQUIRE(n < (int64_t)1 << 30, "raycasting scene too large (>= 2^30 triangles)");
    hipStream_t st = s->stream;
    int rc = 0;
    // Every temporary of the build carved from one block of the process's device-block cache
    // (geom_block_alloc), and the scene's leaf / node arrays from another: a rebuild or the next scene's
    // build reuses them instead of 15 hipMalloc / hipFree pairs: 2.93 -> 1.01 ms per build of a 2.1 M-triangle
    // mesh, the kernels' own 1.06 ms (tools/bvh_build_probe.py, profiles/r05_bvh_build_probe.json).
    const int64_t m1 = std::max<int64_t>(n - 1, 1);
    size_t sort_bytes = 0, depth_sort_bytes = 0;
    MQR_CHECK_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, sort_bytes, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                                     (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)n, 0, 63, st));
    MQR_CHECK_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, depth_sort_bytes, (const uint32_t*)nullptr,
                                                     (uint32_t*)nullptr, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                                     (int)m1, 0, 8, st));
    const size_t tmp_bytes = std::max(sort_bytes, depth_sort_bytes) + 16;
    const size_t sizes[] = {al256(sizeof(BuildTri) * n), al256(4 * n), al256(4 * n), al256(4 * 6), al256(4 * n),
                            al256(4 * n), al256(8 * n), al256(8 * n), al256(8 * m1), al256(8 * n),
                            al256(4 * std::max<int64_t>(m1, 512)), al256(4), al256(tmp_bytes)};
    size_t total = 0;
    for (size_t z : sizes) total += z;
    size_t blk_cap = 0;
    void* blk = geom_block_alloc(s->device, total, &blk_cap);
    MQR_REQUIRE(blk, "raycasting scene: device allocation failed");
    char* q = static_cast<char*>(blk);
    auto carve = [&](int i) {
        char* r = q;
        q += sizes[i];
        return r;
    };
    BuildTri* tris = reinterpret_cast<BuildTri*>(carve(0));
    uint32_t* prim = reinterpret_cast<uint32_t*>(carve(1));
    uint32_t* gid = reinterpret_cast<uint32_t*>(carve(2));
    uint32_t* cb = reinterpret_cast<uint32_t*>(carve(3));
    uint32_t* idx = reinterpret_cast<uint32_t*>(carve(4));
    uint32_t* idx_sorted = reinterpret_cast<uint32_t*>(carve(5));
    uint64_t* keys = reinterpret_cast<uint64_t*>(carve(6));
    uint64_t* keys_sorted = reinterpret_cast<uint64_t*>(carve(7));
    int32_t* child = reinterpret_cast<int32_t*>(carve(8));
    int32_t* parent = reinterpret_cast<int32_t*>(carve(9));
    int* arrivals = reinterpret_cast<int*>(carve(10));
    int* bad = reinterpret_cast<int*>(carve(11));
    void* tmp = carve(12);
    auto cleanup = [&]() {
        (void)hipStreamSynchronize(st);  // (the block goes back to the cache: no kernel of this build may still use it)
        geom_block_release(s->device, blk, blk_cap);
    };
#define RC_HIP(expr)                                                           \
    do {                                                                       \
        hipError_t _e = (expr);                                                \
        if (_e != hipSuccess) {                                                \
            set_error(std::string(#expr) + ": " + hipGetErrorString(_e));      \
            cleanup();                                                         \
            return 1;                                                          \
        }                                                                      \
    } while (0)
    const uint32_t init[6] = {0xffffffffu, 0xffffffffu, 0xffffffffu, 0u, 0u, 0u};
    RC_HIP(hipMemcpyAsync(cb, init, sizeof(init), hipMemcpyHostToDevice, st));
    RC_HIP(hipMemsetAsync(bad, 0, sizeof(int), st));
    RC_HIP(hipMemsetAsync(arrivals, 0, sizeof(int) * std::max<int64_t>(n - 1, 1), st));
    RC_HIP(hipMemsetAsync(parent, 0xff, sizeof(int32_t) * 2 * n, st));
    int64_t base = 0;
    for (size_t g = 0; g < s->geoms.size(); ++g) {
        const auto& G = s->geoms[g];
        if (G.nt == 0) continue;
        hipLaunchKernelGGL(k_gather_tris, dim3((unsigned)std::min<int64_t>((G.nt + 255) / 256, kGatherGrid)), dim3(256), 0,
                           st, G.v, G.t, G.nt,
                           G.nv, base, (uint32_t)g, tris, prim, gid, cb, bad);
        RC_HIP(hipGetLastError());
        base += G.nt;
    }
    const unsigned gb = (unsigned)((n + 255) / 256);
    hipLaunchKernelGGL(k_morton, dim3(gb), dim3(256), 0, st, tris, n, cb, keys, idx);
    RC_HIP(hipGetLastError());
    size_t sb = sort_bytes;
    RC_HIP(hipcub::DeviceRadixSort::SortPairs(tmp, sb, keys, keys_sorted, idx, idx_sorted, (int)n, 0, 63, st));
    {
        const size_t sl = al256(sizeof(float4) * 3 * n);
        s->bvh_blk = geom_block_alloc(s->device, sl + sizeof(float4) * 4 * m1, &s->bvh_cap);
        if (!s->bvh_blk) {
            set_error("raycasting scene: device allocation failed");
            cleanup();
            return 1;
        }
        s->leaf = static_cast<float4*>(s->bvh_blk);
        s->node = reinterpret_cast<float4*>(static_cast<char*>(s->bvh_blk) + sl);
    }
    if (n > 1) {
        hipLaunchKernelGGL(k_radix_tree, dim3((unsigned)((n - 1 + 255) / 256)), dim3(256), 0, st, keys_sorted, n,
                           child, parent);
        RC_HIP(hipGetLastError());
    }
    hipLaunchKernelGGL(k_leaves, dim3(gb), dim3(256), 0, st, tris, prim, gid, idx_sorted, n, s->leaf);
    RC_HIP(hipGetLastError());
    int h_bad = 0;
    if (n > 1) {
        // level-by-level refit: internal node depths -> sort ids by depth -> one launch per level
        const int64_t m = n - 1;
        uint32_t* depth = reinterpret_cast<uint32_t*>(keys);  // 2 x uint32 per former 64-bit key slot
        uint32_t* depth_s = depth + m;
        uint32_t* ids = reinterpret_cast<uint32_t*>(keys_sorted);
        uint32_t* ids_s = ids + m;
        int* lvl = arrivals;  // 512 ints: start[256], end[256] (arrivals has max(n - 1, 512) slots)
        RC_HIP(hipMemsetAsync(lvl, 0, sizeof(int) * 512, st));
        const unsigned gm = (unsigned)((m + 255) / 256);
        hipLaunchKernelGGL(k_node_depth, dim3(gm), dim3(256), 0, st, parent, m, depth, ids, bad);
        RC_HIP(hipGetLastError());
        sb = depth_sort_bytes;
        RC_HIP(hipcub::DeviceRadixSort::SortPairs(tmp, sb, depth, depth_s, ids, ids_s, (int)m, 0, 8, st));
        hipLaunchKernelGGL(k_level_bounds, dim3(gm), dim3(256), 0, st, depth_s, m, lvl, lvl + 256);
        RC_HIP(hipGetLastError());
        int h_lvl[512];
        RC_HIP(hipMemcpyAsync(h_lvl, lvl, sizeof(h_lvl), hipMemcpyDeviceToHost, st));
        RC_HIP(hipMemcpyAsync(&h_bad, bad, sizeof(int), hipMemcpyDeviceToHost, st));
        RC_HIP(hipStreamSynchronize(st));
        if (h_bad & 2) {
            set_error("internal: BVH deeper than 255 levels");
            cleanup();
            free_built(s);
            return 1;
        }
        for (int d = 255; d >= 0; --d) {
            const int64_t cnt = (int64_t)h_lvl[256 + d] - h_lvl[d];
            if (cnt <= 0) continue;
            hipLaunchKernelGGL(k_refit_level, dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0, st, tris, idx_sorted,
                               child, ids_s + h_lvl[d], cnt, s->node);
            RC_HIP(hipGetLastError());
        }
    }
    RC_HIP(hipMemcpyAsync(&h_bad, bad, sizeof(int), hipMemcpyDeviceToHost, st));
    RC_HIP(hipStreamSynchronize(st));
#undef RC_HIP
    cleanup();
    if (h_bad) {
        free_built(s);
        set_error("triangle index out of range of the vertex array");
        return 1;
    }
    s->ntri = n;
    s->built = true;
    return rc;
}

// CreateRaysPinhole's camera: invK = K^-1 in float64 (Eigen partial-pivot LU on the pinhole K,
// i.e. back substitution: 1/fx, -cx/fx, 1/fy, -cy/fy for K = [[fx,0,cx],[0,fy,cy],[0,0,1]]; general
// K falls back to the adjugate), RT_invK = float32(R^T invK), C = float32(-R^T t).
static PinholeFrame pinhole(const double* K, const double* T) {
    double inv[9];
    if (K[1] == 0 && K[3] == 0 && K[6] == 0 && K[7] == 0 && K[8] == 1) {
        inv[0] = 1.0 / K[0], inv[1] = 0.0, inv[2] = -K[2] / K[0];
        inv[3] = 0.0, inv[4] = 1.0 / K[4], inv[5] = -K[5] / K[4];
        inv[6] = 0.0, inv[7] = 0.0, inv[8] = 1.0;
    } else {
        const double a = K[0], b = K[1], c = K[2], d = K[3], e = K[4], f = K[5], g = K[6], h = K[7], i = K[8];
        const double A = e * i - f * h, B = -(d * i - f * g), C = d * h - e * g;
        const double det = a * A + b * B + c * C;
        const double adj[9] = {A, -(b * i - c * h), b * f - c * e, B, a * i - c * g, -(a * f - c * d),
                               C, -(a * h - b * g), a * e - b * d};
        for (int k = 0; k < 9; ++k) inv[k] = adj[k] / det;
    }
    PinholeFrame fr;
    for (int r = 0; r < 3; ++r)
        for (int k = 0; k < 3; ++k) {
            double acc = T[0 * 4 + r] * inv[0 * 3 + k];  // (R^T)[r][m] = R[m][r]
            acc += T[1 * 4 + r] * inv[1 * 3 + k];
            acc += T[2 * 4 + r] * inv[2 * 3 + k];
            fr.m[r * 3 + k] = (float)acc;
        }
    for (int r = 0; r < 3; ++r) {
        double acc = T[0 * 4 + r] * T[0 * 4 + 3];
        acc += T[1 * 4 + r] * T[1 * 4 + 3];
        acc += T[2 * 4 + r] * T[2 * 4 + 3];
        fr.c[r] = (float)(-acc);
    }
    return fr;
}

}  // namespace mqr

using namespace mqr;

extern "C" {

int mqr_scene_create(int device, mqr_scene** out) {
    MQR_REQUIRE(out, "null argument");
    MQR_CHECK_HIP(hipSetDevice(device));
    mqr_scene* s = new mqr_scene();
    s->device = device;
    if (hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) != hipSuccess) {
        delete s;
        set_error("hipStreamCreate failed");
        return 1;
    }
    *out = s;
    return 0;
}

int mqr_scene_destroy(mqr_scene* s) {
    if (!s) return 0;
    (void)hipSetDevice(s->device);
    (void)hipStreamSynchronize(s->stream);
    free_built(s);
    for (auto& g : s->geoms) {
        if (g.v) (void)hipFree(g.v);
        if (g.t) (void)hipFree(g.t);
    }
    (void)hipStreamDestroy(s->stream);
    delete s;
    return 0;
}

int mqr_scene_add_triangles(mqr_scene* s, const float* vertices, int64_t nv, const int32_t* triangles, int64_t nt,
                            int loc, uint32_t* geom_id) {
    MQR_REQUIRE(s && (nv == 0 || vertices) && (nt == 0 || triangles), "null argument");
    MQR_REQUIRE(nv >= 0 && nt >= 0, "negative size");
    MQR_CHECK_HIP(hipSetDevice(s->device));
    mqr_scene::Geom g;
    g.nv = nv;
    g.nt = nt;
    const hipMemcpyKind k = loc == MQR_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
    if (loc == MQR_DEVICE && order_after_caller(s->device, s->stream)) return 2;
    MQR_CHECK_HIP(hipMalloc(&g.v, sizeof(float) * 3 * std::max<int64_t>(nv, 1)));
    MQR_CHECK_HIP(hipMalloc(&g.t, sizeof(int32_t) * 3 * std::max<int64_t>(nt, 1)));
    if (loc == MQR_DEVICE) {
        if (nv) MQR_CHECK_HIP(hipMemcpyAsync(g.v, vertices, sizeof(float) * 3 * nv, k, s->stream));
        if (nt) MQR_CHECK_HIP(hipMemcpyAsync(g.t, triangles, sizeof(int32_t) * 3 * nt, k, s->stream));
        MQR_CHECK_HIP(hipStreamSynchronize(s->stream));
    } else if (copy_to_device(s->device, g.v, vertices, sizeof(float) * 3 * nv, s->stream) ||
               copy_to_device(s->device, g.t, triangles, sizeof(int32_t) * 3 * nt, s->stream)) {
        (void)hipFree(g.v);
        (void)hipFree(g.t);
        return 1;
    }
    if (geom_id) *geom_id = (uint32_t)s->geoms.size();
    s->geoms.push_back(g);
    s->built = false;
    return 0;
}

int mqr_scene_build(mqr_scene* s) {
    MQR_REQUIRE(s, "null scene");
    MQR_CHECK_HIP(hipSetDevice(s->device));
    return build(s);
}

int mqr_scene_cast_pinhole(mqr_scene* s, const double* K, const double* T_wc, int n_frames, int H, int W,
                           float* t_hit, uint32_t* geom_ids, uint32_t* prim_ids, float* uvs, float* normals,
                           int out_loc) {
    MQR_REQUIRE(s && K && T_wc && t_hit, "null argument");
    MQR_REQUIRE(n_frames > 0 && H > 0 && W > 0, "bad image shape");
    MQR_CHECK_HIP(hipSetDevice(s->device));
    if (build(s)) return 1;
    const int64_t HW = (int64_t)H * W, total = HW * n_frames;
    if (out_loc == MQR_DEVICE && order_after_caller(s->device, s->stream)) return 2;
    std::vector<PinholeFrame> hf(n_frames);
    for (int f = 0; f < n_frames; ++f) hf[f] = pinhole(K + 9 * f, T_wc + 16 * f);
    float *d_t = t_hit, *d_uv = uvs, *d_n = normals;
    uint32_t *d_g = geom_ids, *d_p = prim_ids;
    const bool host_out = out_loc != MQR_DEVICE;
    const size_t per_px = host_out ? 4 + (geom_ids ? 4 : 0) + (prim_ids ? 4 : 0) + (uvs ? 8 : 0) +
                                         (normals ? 12 : 0)
                                   : 0;
    CachedBlock blk(s->device, al256(sizeof(PinholeFrame) * n_frames) + per_px * total + 5 * 256);
    bool ok = blk.p != nullptr;
    PinholeFrame* d_fr = ok ? (PinholeFrame*)blk.take(sizeof(PinholeFrame) * n_frames) : nullptr;
    if (ok && host_out) {
        d_t = (float*)blk.take(sizeof(float) * total);
        if (geom_ids) d_g = (uint32_t*)blk.take(sizeof(uint32_t) * total);
        if (prim_ids) d_p = (uint32_t*)blk.take(sizeof(uint32_t) * total);
        if (uvs) d_uv = (float*)blk.take(sizeof(float) * 2 * total);
        if (normals) d_n = (float*)blk.take(sizeof(float) * 3 * total);
    }
    int rc = 0;
    if (!ok) {
        set_error("cast_pinhole: device allocation failed");
        rc = 1;
    }
    if (!rc && hipMemcpyAsync(d_fr, hf.data(), sizeof(PinholeFrame) * n_frames, hipMemcpyHostToDevice, s->stream)) {
        set_error("cast_pinhole: upload failed");
        rc = 1;
    }
    if (!rc) {
        const int64_t tiles = (int64_t)((W + 7) / 8) * ((H + 7) / 8);
        hipLaunchKernelGGL(k_cast_pinhole, dim3((unsigned)((tiles + 3) / 4), (unsigned)n_frames), dim3(256), 0,
                           s->stream, s->node, s->leaf, s->ntri, d_fr, H, W, d_t, d_g, d_p, d_uv, d_n);
        if (hipGetLastError() != hipSuccess) {
            set_error("cast_pinhole: launch failed");
            rc = 1;
        }
    }
    if (!rc && out_loc != MQR_DEVICE) {
        const int dv = s->device;
        if (copy_to_host(dv, t_hit, d_t, sizeof(float) * total, s->stream) ||
            (geom_ids && copy_to_host(dv, geom_ids, d_g, sizeof(uint32_t) * total, s->stream)) ||
            (prim_ids && copy_to_host(dv, prim_ids, d_p, sizeof(uint32_t) * total, s->stream)) ||
            (uvs && copy_to_host(dv, uvs, d_uv, sizeof(float) * 2 * total, s->stream)) ||
            (normals && copy_to_host(dv, normals, d_n, sizeof(float) * 3 * total, s->stream))) {
            set_error("cast_pinhole: copy back failed");
            rc = 1;
        }
    }
    if (hipStreamSynchronize(s->stream) != hipSuccess && !rc) {
        set_error("cast_pinhole: kernel failed");
        rc = 1;
    }
    return rc;
}

int mqr_scene_cast_rays(mqr_scene* s, const float* rays, int64_t nrays, int rays_loc, float* t_hit,
                        uint32_t* geom_ids, uint32_t* prim_ids, float* uvs, float* normals, int out_loc) {
    MQR_REQUIRE(s && rays && t_hit, "null argument");
    MQR_REQUIRE(nrays >= 0, "negative ray count");
    MQR_CHECK_HIP(hipSetDevice(s->device));
    if (build(s)) return 1;
    if (nrays == 0) return 0;
    if ((rays_loc == MQR_DEVICE || out_loc == MQR_DEVICE) && order_after_caller(s->device, s->stream)) return 2;
    const float* d_r = rays;
    float *d_t = t_hit, *d_uv = uvs, *d_n = normals;
    uint32_t *d_g = geom_ids, *d_p = prim_ids;
    const bool host_in = rays_loc != MQR_DEVICE, host_out = out_loc != MQR_DEVICE;
    const size_t per_ray = (host_in ? 24 : 0) + (host_out ? 4 + (geom_ids ? 4 : 0) + (prim_ids ? 4 : 0) +
                                                             (uvs ? 8 : 0) + (normals ? 12 : 0)
                                                       : 0);
    CachedBlock blk(s->device, per_ray * (size_t)nrays + 6 * 256);
    bool ok = blk.p != nullptr;
    if (ok && host_in) {
        float* p = (float*)blk.take(sizeof(float) * 6 * nrays);
        ok = copy_to_device(s->device, p, rays, sizeof(float) * 6 * nrays, s->stream) == 0;
        d_r = p;
    }
    if (ok && host_out) {
        d_t = (float*)blk.take(sizeof(float) * nrays);
        if (geom_ids) d_g = (uint32_t*)blk.take(sizeof(uint32_t) * nrays);
        if (prim_ids) d_p = (uint32_t*)blk.take(sizeof(uint32_t) * nrays);
        if (uvs) d_uv = (float*)blk.take(sizeof(float) * 2 * nrays);
        if (normals) d_n = (float*)blk.take(sizeof(float) * 3 * nrays);
    }
    int rc = 0;
    if (!ok) {
        set_error("cast_rays: device allocation / upload failed");
        rc = 1;
    }
    if (!rc) {
        hipLaunchKernelGGL(k_cast_rays, dim3((unsigned)((nrays + 255) / 256)), dim3(256), 0, s->stream, s->node,
                           s->leaf, s->ntri, d_r, nrays, d_t, d_g, d_p, d_uv, d_n);
        if (hipGetLastError() != hipSuccess) {
            set_error("cast_rays: launch failed");
            rc = 1;
        }
    }
    if (!rc && out_loc != MQR_DEVICE) {
        const int dv = s->device;
        if (copy_to_host(dv, t_hit, d_t, sizeof(float) * nrays, s->stream) ||
            (geom_ids && copy_to_host(dv, geom_ids, d_g, sizeof(uint32_t) * nrays, s->stream)) ||
            (prim_ids && copy_to_host(dv, prim_ids, d_p, sizeof(uint32_t) * nrays, s->stream)) ||
            (uvs && copy_to_host(dv, uvs, d_uv, sizeof(float) * 2 * nrays, s->stream)) ||
            (normals && copy_to_host(dv, normals, d_n, sizeof(float) * 3 * nrays, s->stream))) {
            set_error("cast_rays: copy back failed");
            rc = 1;
        }
    }
    if (hipStreamSynchronize(s->stream) != hipSuccess && !rc) {
        set_error("cast_rays: kernel failed");
        rc = 1;
    }
    return rc;
}

int mqr_scene_triangle_count(mqr_scene* s, int64_t* n) {
    MQR_REQUIRE(s && n, "null argument");
    int64_t t = 0;
    for (auto& g : s->geoms) t += g.nt;
    *n = t;
    return 0;
}

}  // extern "C"

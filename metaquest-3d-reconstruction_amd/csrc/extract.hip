// extract.hip -- surface extraction from the HBM-resident volume.
//
//   vbg.extract_point_cloud(weight_threshold=3.0)   reconstruct_scene.py:90, refine_fragment_poses.py:39
//   vbg.extract_triangle_mesh(weight_threshold=1.5) reconstruct_scene.py:105-108, 186-189
//
// Semantics = upstream Open3D 0.19 ExtractPointCloud / ExtractTriangleMesh:
// cube valid iff all 8 corners exist with weight > thr, bit i set iff tsdf_i < 0, one vertex per
// marked owned edge, Bourke tri-table with reversed vertex order, normals from central TSDF
// differences (component left unchanged when a side's block is missing, carried across edges
// exactly like upstream's per-voxel normal scratch).
//
// GPU structure (no atomics on the output, deterministic order = (block, voxel, edge)):
//   k_nb        27-neighbour buffer table per active block (hash lookups)
//   k_*_count   one 256-thread workgroup per block: stage the (R+3)^3 tile [-1, R+1]^3 of
//               (tsdf, flags) in LDS from up to 27 blocks, classify cubes, count vertices /
//               triangles / points, block-local prefix by wave64 scan; the mesh pass also
//               publishes the local vertex ids of the block's three low faces
//   hipcub      exclusive scans of the per-block counts
//   k_*_emit    re-stage the tile, write vertices + normals + triangles at their global offsets
#include <hipcub/hipcub.hpp>

#include <algorithm>

#include "mqr_common.hpp"
#include "mqr_mc_tables.h"

namespace mqr {

constexpr int kMaxR = 16;
constexpr int kThreads = 512;  // 8 waves per workgroup: two LDS-resident blocks per CU keep 16 waves busy

__device__ inline int64_t dev_find(const Table t, uint64_t k) {
    const uint64_t m = (uint64_t)t.cap - 1;
    uint64_t h = mix64(k) & m;
    for (int64_t p = 0; p < t.cap; ++p) {
        const uint64_t cur = t.keys[h];
        if (cur == k) return (int64_t)h;
        if (cur == kEmpty) return -1;
        h = (h + 1) & m;
    }
    return -1;
}

__global__ void k_nb(const uint64_t* __restrict__ bkeys, int64_t n, const Table t, int32_t* nb) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n * 27) return;
    const int64_t b = i / 27;
    const int k = (int)(i % 27);
    int x, y, z;
    unpack_key(bkeys[b], x, y, z);
    x += k % 3 - 1;
    y += (k % 9) / 3 - 1;
    z += k / 9 - 1;
    int32_t r = -1;
    if (key_in_range(x, y, z)) {
        const int64_t s = dev_find(t, pack_key(x, y, z));
        if (s >= 0) r = t.vals[s];
    }
    nb[i] = r;
}

// Kernels are templated on the block resolution RT (16 / 8 at compile time; 0 = runtime R <= 16)
// so that every index split below is a shift, and LDS arrays are sized for RM = RT or kMaxR.
template <int RT>
struct Dims {
    static constexpr int RM = RT > 0 ? RT : kMaxR;
    static constexpr int SM = RM + 3;      // tile side [-1, R+1]
    static constexpr int CM = RM + 1;      // cube origins [-1, R-1]
    int R, S, C;
    __device__ explicit Dims(int r) : R(RT > 0 ? RT : r), S((RT > 0 ? RT : r) + 3), C((RT > 0 ? RT : r) + 1) {}
    __device__ int tidx(int x, int y, int z) const { return ((z + 1) * S + (y + 1)) * S + (x + 1); }
    __device__ int cidx(int x, int y, int z) const { return ((z + 1) * C + (y + 1)) * C + (x + 1); }
};

// flags: bit0 block present, bit1 weight > thr, bit2 tsdf < 0
template <int RT>
struct FlagTile {
    uint8_t flag[Dims<RT>::SM * Dims<RT>::SM * Dims<RT>::SM];
};
template <int RT>
struct Tile {
    float tsdf[Dims<RT>::SM * Dims<RT>::SM * Dims<RT>::SM];
    uint8_t flag[Dims<RT>::SM * Dims<RT>::SM * Dims<RT>::SM];
};

// Stage the (R+3)^3 tile [-1, R+1]^3 from the block and its 26 neighbours (nbrow: buffer or -1).
template <int RT, bool TSDF>
__device__ void load_tile(uint8_t* __restrict__ flag, float* __restrict__ tsdf, const int32_t* __restrict__ nbrow,
                          const float2* __restrict__ pool, const Dims<RT>& d, float thr) {
    const int R = d.R, S = d.S;
    const int S3 = S * S * S;
    const int R3 = R * R * R;
    for (int i = threadIdx.x; i < S3; i += blockDim.x) {
        const int lx = i % S - 1, ly = (i / S) % S - 1, lz = i / (S * S) - 1;
        const int dx = lx < 0 ? -1 : (lx >= R ? 1 : 0);
        const int dy = ly < 0 ? -1 : (ly >= R ? 1 : 0);
        const int dz = lz < 0 ? -1 : (lz >= R ? 1 : 0);
        const int nbuf = nbrow[(dx + 1) + 3 * (dy + 1) + 9 * (dz + 1)];
        uint8_t f = 0;
        float ts = 0.f;
        if (nbuf >= 0) {
            const float2 tw =
                pool[(int64_t)nbuf * R3 + ((lz - dz * R) * R + (ly - dy * R)) * R + (lx - dx * R)];
            ts = tw.x;
            f = 1 | (tw.y > thr ? 2 : 0) | (tw.x < 0 ? 4 : 0);
        }
        flag[i] = f;
        if (TSDF) tsdf[i] = ts;
    }
}

// Block-wide exclusive scan of one int per thread (blockDim / 64 waves of 64, <= 16).
__device__ inline int block_exclusive_scan(int v, int* scratch /* >= blockDim / 64 ints */, int& total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int incl = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int o = __shfl_up(incl, d, 64);
        if (lane >= d) incl += o;
    }
    if (lane == 63) scratch[wave] = incl;
    __syncthreads();
    int off = 0;
    total = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) {
        if (w < wave) off += scratch[w];
        total += scratch[w];
    }
    __syncthreads();
    return off + incl - v;
}

// Per-block mesh classification shared by the count and emit passes.  Thread t owns the
// contiguous voxel chunk [t * chunk, (t + 1) * chunk) in both passes (triangle ids run over it).
template <int RT>
struct MeshLocal {
    static constexpr int R3M = Dims<RT>::RM * Dims<RT>::RM * Dims<RT>::RM;
    uint16_t cube[Dims<RT>::CM * Dims<RT>::CM * Dims<RT>::CM];  // origins [-1, R-1]^3: bit8 valid | index
    uint8_t emask[R3M];                                          // owned edges with a vertex (bits x,y,z)
    uint16_t vbase[R3M];                                         // local vertex id of the voxel's first vertex
    int scratch[16];
};

template <int RT>
__device__ void classify_mesh(const uint8_t* __restrict__ flag, MeshLocal<RT>& ml, const Dims<RT>& d, int& nverts,
                              int& ntris, int& tstart) {
    const int R = d.R, C = d.C;
    for (int i = threadIdx.x; i < C * C * C; i += blockDim.x) {
        const int cx = i % C - 1, cy = (i / C) % C - 1, cz = i / (C * C) - 1;
        int ci = 0;
        bool ok = true;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint8_t f = flag[d.tidx(cx + mqr_vtx_shifts[k][0], cy + mqr_vtx_shifts[k][1],
                                          cz + mqr_vtx_shifts[k][2])];
            ok = ok && (f & 2);
            ci |= (f & 4) ? (1 << k) : 0;
        }
        ml.cube[i] = ok ? (uint16_t)(0x100 | ci) : (uint16_t)0;
    }
    __syncthreads();
    const int R3 = R * R * R;
    const int chunk = (R3 + blockDim.x - 1) / blockDim.x;
    const int p0 = threadIdx.x * chunk, p1 = min(p0 + chunk, R3);
    int vsum = 0, tsum = 0;
    for (int p = p0; p < p1; ++p) {
        const int x = p % R, y = (p / R) % R, z = p / (R * R);
        const bool s0 = flag[d.tidx(x, y, z)] & 4;
        int m = 0;
        // x edge: cubes at v, v-y, v-z, v-y-z
        if (((flag[d.tidx(x + 1, y, z)] & 4) != 0) != s0 &&
            ((ml.cube[d.cidx(x, y, z)] | ml.cube[d.cidx(x, y - 1, z)] | ml.cube[d.cidx(x, y, z - 1)] |
              ml.cube[d.cidx(x, y - 1, z - 1)]) & 0x100))
            m |= 1;
        if (((flag[d.tidx(x, y + 1, z)] & 4) != 0) != s0 &&
            ((ml.cube[d.cidx(x, y, z)] | ml.cube[d.cidx(x - 1, y, z)] | ml.cube[d.cidx(x, y, z - 1)] |
              ml.cube[d.cidx(x - 1, y, z - 1)]) & 0x100))
            m |= 2;
        if (((flag[d.tidx(x, y, z + 1)] & 4) != 0) != s0 &&
            ((ml.cube[d.cidx(x, y, z)] | ml.cube[d.cidx(x - 1, y, z)] | ml.cube[d.cidx(x, y - 1, z)] |
              ml.cube[d.cidx(x - 1, y - 1, z)]) & 0x100))
            m |= 4;
        ml.emask[p] = (uint8_t)m;
        vsum += __popc(m);
        const uint16_t c = ml.cube[d.cidx(x, y, z)];
        if (c & 0x100) tsum += mqr_tri_count[c & 0xff];
    }
    int vtot, ttot;
    int voff = block_exclusive_scan(vsum, ml.scratch, vtot);
    tstart = block_exclusive_scan(tsum, ml.scratch + 8, ttot);
    for (int p = p0; p < p1; ++p) {
        ml.vbase[p] = (uint16_t)voff;
        voff += __popc(ml.emask[p]);
    }
    __syncthreads();
    nverts = vtot;
    ntris = ttot;
}

// face table entry: bits 0..15 local vertex base, bits 16..18 edge mask
template <int RT>
__device__ inline uint32_t face_entry(const MeshLocal<RT>& ml, int p) {
    return (uint32_t)ml.vbase[p] | ((uint32_t)ml.emask[p] << 16);
}

template <int RT>
__global__ __launch_bounds__(kThreads) void k_mesh_count(const int32_t* __restrict__ nb, int64_t n,
                                                         const float2* __restrict__ pool, int Rrt, float thr,
                                                         int32_t* vcount, int32_t* tcount, uint32_t* faces) {
    __shared__ FlagTile<RT> tl;
    __shared__ MeshLocal<RT> ml;
    __shared__ int32_t nbrow[27];
    const Dims<RT> d(Rrt);
    const int R = d.R;
    const int64_t b = blockIdx.x;
    if (threadIdx.x < 27) nbrow[threadIdx.x] = nb[b * 27 + threadIdx.x];
    __syncthreads();
    load_tile<RT, false>(tl.flag, nullptr, nbrow, pool, d, thr);
    __syncthreads();
    int nv, nt, ts;
    classify_mesh<RT>(tl.flag, ml, d, nv, nt, ts);
    if (threadIdx.x == 0) {
        vcount[b] = nv;
        tcount[b] = nt;
    }
    // low faces: x == 0 (index z*R+y), y == 0 (z*R+x), z == 0 (y*R+x)
    const int RR = R * R;
    uint32_t* fb = faces + b * 3 * RR;
    for (int i = threadIdx.x; i < RR; i += blockDim.x) {
        const int a = i / R, c = i % R;
        fb[i] = face_entry(ml, (a * R + c) * R + 0);           // x = 0: z = a, y = c
        fb[RR + i] = face_entry(ml, (a * R + 0) * R + c);      // y = 0: z = a, x = c
        fb[2 * RR + i] = face_entry(ml, (0 * R + a) * R + c);  // z = 0: y = a, x = c
    }
}

// normal at tile point (x,y,z) in [0, R]: central differences over present voxels, components
// of `n` untouched when a side is absent (upstream DeviceGetNormal).
template <int RT>
__device__ inline void tile_normal(const Tile<RT>& tl, const Dims<RT>& d, int x, int y, int z, float* n) {
    const int xp = d.tidx(x + 1, y, z), xn = d.tidx(x - 1, y, z);
    const int yp = d.tidx(x, y + 1, z), yn = d.tidx(x, y - 1, z);
    const int zp = d.tidx(x, y, z + 1), zn = d.tidx(x, y, z - 1);
    if ((tl.flag[xp] & 1) && (tl.flag[xn] & 1)) n[0] = tl.tsdf[xp] - tl.tsdf[xn];
    if ((tl.flag[yp] & 1) && (tl.flag[yn] & 1)) n[1] = tl.tsdf[yp] - tl.tsdf[yn];
    if ((tl.flag[zp] & 1) && (tl.flag[zn] & 1)) n[2] = tl.tsdf[zp] - tl.tsdf[zn];
}

__device__ inline void write_normal(float nx, float ny, float nz, float* out) {
    const float norm = (float)((double)sqrtf(nx * nx + ny * ny + nz * nz) + 1e-5);
    out[0] = nx / norm;
    out[1] = ny / norm;
    out[2] = nz / norm;
}

template <int RT>
__global__ __launch_bounds__(kThreads) void k_mesh_emit(const int32_t* __restrict__ nb, int64_t n,
                                                        const uint64_t* __restrict__ bkeys,
                                                        const float2* __restrict__ pool, int Rrt, float voxel_size,
                                                        float thr, const int32_t* __restrict__ vcount,
                                                        const int32_t* __restrict__ tcount,
                                                        const int32_t* __restrict__ voff,
                                                        const int32_t* __restrict__ toff,
                                                        const uint32_t* __restrict__ faces, float* pos, float* nrm,
                                                        int32_t* tri) {
    __shared__ Tile<RT> tl;
    __shared__ MeshLocal<RT> ml;
    __shared__ int32_t nbrow[27];
    __shared__ int32_t nbvoff[27];
    const int64_t b = blockIdx.x;
    if (vcount[b] == 0 && tcount[b] == 0) return;  // block-uniform: nothing to write
    const Dims<RT> d(Rrt);
    const int R = d.R;
    if (threadIdx.x < 27) {
        const int32_t q = nb[b * 27 + threadIdx.x];
        nbrow[threadIdx.x] = q;
        nbvoff[threadIdx.x] = q >= 0 ? voff[q] : 0;
    }
    __syncthreads();
    load_tile<RT, true>(tl.flag, tl.tsdf, nbrow, pool, d, thr);
    __syncthreads();
    int nv, nt, tstart;
    classify_mesh<RT>(tl.flag, ml, d, nv, nt, tstart);
    const int R3 = R * R * R;
    const int RR = R * R;
    int xb, yb, zb;
    unpack_key(bkeys[b], xb, yb, zb);
    const int32_t vb = voff[b];
    int t = toff[b] + tstart;
    const int chunk = (R3 + blockDim.x - 1) / blockDim.x;
    const int p0 = threadIdx.x * chunk, p1 = min(p0 + chunk, R3);
    for (int p = p0; p < p1; ++p) {
        const int x = p % R, y = (p / R) % R, z = p / (R * R);
        const int m = ml.emask[p];
        if (m) {
            const float tsdf_o = tl.tsdf[d.tidx(x, y, z)];
            float no[3] = {0.f, 0.f, 0.f}, ne[3] = {0.f, 0.f, 0.f};
            tile_normal(tl, d, x, y, z, no);
            int id = vb + ml.vbase[p];
            const int gx = xb * R + x, gy = yb * R + y, gz = zb * R + z;
            for (int e = 0; e < 3; ++e) {
                if (!(m & (1 << e))) continue;
                const int ex = x + (e == 0), ey = y + (e == 1), ez = z + (e == 2);
                const float tsdf_e = tl.tsdf[d.tidx(ex, ey, ez)];
                const float ratio = (0 - tsdf_o) / (tsdf_e - tsdf_o);
                const float rx = ratio * (int)(e == 0), ry = ratio * (int)(e == 1), rz = ratio * (int)(e == 2);
                pos[3 * (int64_t)id + 0] = voxel_size * (gx + rx);
                pos[3 * (int64_t)id + 1] = voxel_size * (gy + ry);
                pos[3 * (int64_t)id + 2] = voxel_size * (gz + rz);
                tile_normal(tl, d, ex, ey, ez, ne);
                const float nx = (1 - ratio) * no[0] + ratio * ne[0];
                const float ny = (1 - ratio) * no[1] + ratio * ne[1];
                const float nz = (1 - ratio) * no[2] + ratio * ne[2];
                write_normal(nx, ny, nz, nrm + 3 * (int64_t)id);
                ++id;
            }
        }
        const uint16_t c = ml.cube[d.cidx(x, y, z)];
        if (!(c & 0x100)) continue;
        const int ci = c & 0xff;
        for (int r = 0; r < 16; r += 3) {
            if (mqr_tri_table[ci][r] == -1) break;
            for (int k = 0; k < 3; ++k) {
                const int edge = mqr_tri_table[ci][r + k];
                const int ox = x + mqr_edge_shifts[edge][0], oy = y + mqr_edge_shifts[edge][1],
                          oz = z + mqr_edge_shifts[edge][2];
                const int axis = mqr_edge_shifts[edge][3];
                int32_t vid;
                if (ox < R && oy < R && oz < R) {
                    const int q = (oz * R + oy) * R + ox;
                    vid = vb + ml.vbase[q] + __popc(ml.emask[q] & ((1 << axis) - 1));
                } else {
                    const int dx = ox >= R, dy = oy >= R, dz = oz >= R;
                    const int k27 = (dx + 1) + 3 * (dy + 1) + 9 * (dz + 1);
                    const int32_t nbuf = nbrow[k27];
                    if (nbuf < 0) {  // cannot happen for a valid cube (all corners exist); stay in bounds
                        tri[3 * (int64_t)t + (2 - k)] = -1;
                        continue;
                    }
                    const int lx = ox - dx * R, ly = oy - dy * R, lz = oz - dz * R;
                    uint32_t fe;
                    if (lx == 0)
                        fe = faces[(int64_t)nbuf * 3 * RR + lz * R + ly];
                    else if (ly == 0)
                        fe = faces[(int64_t)nbuf * 3 * RR + RR + lz * R + lx];
                    else
                        fe = faces[(int64_t)nbuf * 3 * RR + 2 * RR + ly * R + lx];
                    vid = nbvoff[k27] + (int32_t)(fe & 0xffff) + __popc((fe >> 16) & ((1u << axis) - 1));
                }
                tri[3 * (int64_t)t + (2 - k)] = vid;
            }
            ++t;
        }
    }
}

// ---------------------------------------------------------------- point cloud
template <int RT>
__device__ inline int point_mask(const Tile<RT>& tl, const Dims<RT>& d, int x, int y, int z) {
    const int o = d.tidx(x, y, z);
    if (!(tl.flag[o] & 2)) return 0;
    const float t_o = tl.tsdf[o];
    int m = 0;
    for (int i = 0; i < 3; ++i) {
        const int q = d.tidx(x + (i == 0), y + (i == 1), z + (i == 2));
        if ((tl.flag[q] & 2) && tl.tsdf[q] * t_o < 0) m |= 1 << i;
    }
    return m;
}

template <int RT>
__global__ __launch_bounds__(kThreads) void k_points(const int32_t* __restrict__ nb, int64_t n,
                                                     const uint64_t* __restrict__ bkeys,
                                                     const float2* __restrict__ pool, int Rrt, float voxel_size,
                                                     float thr, int32_t* counts, const int32_t* __restrict__ offs,
                                                     float* pos, float* nrm) {
    __shared__ Tile<RT> tl;
    __shared__ int32_t nbrow[27];
    __shared__ int scratch[8];
    const int64_t b = blockIdx.x;
    if (offs && counts[b] == 0) return;  // emit pass: block-uniform skip
    const Dims<RT> d(Rrt);
    const int R = d.R;
    if (threadIdx.x < 27) nbrow[threadIdx.x] = nb[b * 27 + threadIdx.x];
    __syncthreads();
    load_tile<RT, true>(tl.flag, tl.tsdf, nbrow, pool, d, thr);
    __syncthreads();
    const int R3 = R * R * R;
    const int chunk = (R3 + blockDim.x - 1) / blockDim.x;
    const int p0 = threadIdx.x * chunk, p1 = min(p0 + chunk, R3);
    int cnt = 0;
    for (int p = p0; p < p1; ++p) cnt += __popc(point_mask(tl, d, p % R, (p / R) % R, p / (R * R)));
    int total;
    int id = block_exclusive_scan(cnt, scratch, total);
    if (!offs) {
        if (threadIdx.x == 0) counts[b] = total;
        return;
    }
    id += offs[b];
    int xb, yb, zb;
    unpack_key(bkeys[b], xb, yb, zb);
    for (int p = p0; p < p1; ++p) {
        const int x = p % R, y = (p / R) % R, z = p / (R * R);
        const int m = point_mask(tl, d, x, y, z);
        if (!m) continue;
        const float t_o = tl.tsdf[d.tidx(x, y, z)];
        float no[3] = {0.f, 0.f, 0.f}, ni[3] = {0.f, 0.f, 0.f};
        tile_normal(tl, d, x, y, z, no);
        const int gx = xb * R + x, gy = yb * R + y, gz = zb * R + z;
        for (int i = 0; i < 3; ++i) {
            if (!(m & (1 << i))) continue;
            const int qx = x + (i == 0), qy = y + (i == 1), qz = z + (i == 2);
            const float t_i = tl.tsdf[d.tidx(qx, qy, qz)];
            const float ratio = (0 - t_o) / (t_i - t_o);
            pos[3 * (int64_t)id + 0] = voxel_size * (gx + ratio * (int)(i == 0));
            pos[3 * (int64_t)id + 1] = voxel_size * (gy + ratio * (int)(i == 1));
            pos[3 * (int64_t)id + 2] = voxel_size * (gz + ratio * (int)(i == 2));
            tile_normal(tl, d, qx, qy, qz, ni);
            const float nx = (1 - ratio) * no[0] + ratio * ni[0];
            const float ny = (1 - ratio) * no[1] + ratio * ni[1];
            const float nz = (1 - ratio) * no[2] + ratio * ni[2];
            write_normal(nx, ny, nz, nrm + 3 * (int64_t)id);
            ++id;
        }
    }
}

// ---------------------------------------------------------------- host side
static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// Carve the grow-only per-volume scratch: nb[27n], 4 count/offset arrays of n, faces[3R^2 n], scan temp.
struct ExScratch {
    int32_t *nb, *c0, *c1, *o0, *o1;
    uint32_t* faces;
    void* tmp;
    size_t tmp_bytes;
};

static int ex_scratch(mqr_vbg* v, int64_t n, bool mesh, ExScratch& e) {
    size_t tmp_bytes = 0;
    MQR_CHECK_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, (const int32_t*)nullptr, (int32_t*)nullptr,
                                                   (int)n, v->stream));
    const size_t sz_nb = align256(sizeof(int32_t) * 27 * n), sz_c = align256(sizeof(int32_t) * n);
    const size_t sz_f = mesh ? align256(sizeof(uint32_t) * 3 * v->R * v->R * n) : 0;
    const size_t need = sz_nb + 4 * sz_c + sz_f + align256(tmp_bytes);
    if (v->ex_scratch_bytes < need) {
        MQR_CHECK_HIP(hipStreamSynchronize(v->stream));
        if (v->ex_scratch) MQR_CHECK_HIP(hipFree(v->ex_scratch));
        v->ex_scratch = nullptr;
        v->ex_scratch_bytes = 0;
        const size_t cap = need + need / 4;
        MQR_CHECK_HIP(hipMalloc(&v->ex_scratch, cap));
        v->ex_scratch_bytes = cap;
    }
    if (!v->h_ex) MQR_CHECK_HIP(hipHostMalloc(&v->h_ex, 4 * sizeof(int64_t), hipHostMallocDefault));
    char* p = static_cast<char*>(v->ex_scratch);
    e.nb = reinterpret_cast<int32_t*>(p);
    p += sz_nb;
    e.c0 = reinterpret_cast<int32_t*>(p);
    e.c1 = reinterpret_cast<int32_t*>(p + sz_c);
    e.o0 = reinterpret_cast<int32_t*>(p + 2 * sz_c);
    e.o1 = reinterpret_cast<int32_t*>(p + 3 * sz_c);
    p += 4 * sz_c;
    e.faces = reinterpret_cast<uint32_t*>(p);
    p += sz_f;
    e.tmp = p;
    e.tmp_bytes = tmp_bytes;
    return 0;
}

// Exclusive scans of up to two per-block count arrays; totals = last count + last offset (one sync).
static int scan_totals(mqr_vbg* v, const ExScratch& e, int64_t n, int arrays, int64_t* tot0, int64_t* tot1) {
    int32_t* h = reinterpret_cast<int32_t*>(v->h_ex);
    size_t tb = e.tmp_bytes;
    MQR_CHECK_HIP(hipcub::DeviceScan::ExclusiveSum(e.tmp, tb, e.c0, e.o0, (int)n, v->stream));
    MQR_CHECK_HIP(hipMemcpyAsync(h + 0, e.c0 + n - 1, sizeof(int32_t), hipMemcpyDeviceToHost, v->stream));
    MQR_CHECK_HIP(hipMemcpyAsync(h + 1, e.o0 + n - 1, sizeof(int32_t), hipMemcpyDeviceToHost, v->stream));
    if (arrays > 1) {
        tb = e.tmp_bytes;
        MQR_CHECK_HIP(hipcub::DeviceScan::ExclusiveSum(e.tmp, tb, e.c1, e.o1, (int)n, v->stream));
        MQR_CHECK_HIP(hipMemcpyAsync(h + 2, e.c1 + n - 1, sizeof(int32_t), hipMemcpyDeviceToHost, v->stream));
        MQR_CHECK_HIP(hipMemcpyAsync(h + 3, e.o1 + n - 1, sizeof(int32_t), hipMemcpyDeviceToHost, v->stream));
    }
    MQR_CHECK_HIP(hipStreamSynchronize(v->stream));
    *tot0 = (int64_t)h[0] + h[1];
    if (arrays > 1) *tot1 = (int64_t)h[2] + h[3];
    return 0;
}

static int build_nb(mqr_vbg* v, int32_t* nb) {
    const int64_t n = v->pool_count;
    hipLaunchKernelGGL(k_nb, dim3((unsigned)((n * 27 + 255) / 256)), dim3(256), 0, v->stream, v->bkeys, n, v->tab, nb);
    MQR_CHECK_HIP(hipGetLastError());
    return 0;
}

template <int RT>
static int mesh_passes(mqr_vbg* v, float thr, const ExScratch& e, mqr_geom* g) {
    const int64_t n = v->pool_count;
    hipLaunchKernelGGL(k_mesh_count<RT>, dim3((unsigned)n), dim3(kThreads), 0, v->stream, e.nb, n, v->pool, v->R,
                       thr, e.c0, e.c1, e.faces);
    MQR_CHECK_HIP(hipGetLastError());
    int64_t nv = 0, nt = 0;
    if (scan_totals(v, e, n, 2, &nv, &nt)) return 1;
    MQR_REQUIRE(nv < (int64_t)1 << 31 && nt < (int64_t)1 << 31, "mesh exceeds int32 vertex / triangle ids");
    g->nv = nv;
    g->nt = nt;
    MQR_CHECK_HIP(hipMalloc(&g->pos, sizeof(float) * 3 * std::max<int64_t>(nv, 1)));
    MQR_CHECK_HIP(hipMalloc(&g->nrm, sizeof(float) * 3 * std::max<int64_t>(nv, 1)));
    MQR_CHECK_HIP(hipMalloc(&g->tri, sizeof(int32_t) * 3 * std::max<int64_t>(nt, 1)));
    hipLaunchKernelGGL(k_mesh_emit<RT>, dim3((unsigned)n), dim3(kThreads), 0, v->stream, e.nb, n, v->bkeys, v->pool,
                       v->R, v->voxel_size, thr, e.c0, e.c1, e.o0, e.o1, e.faces, g->pos, g->nrm, g->tri);
    MQR_CHECK_HIP(hipGetLastError());
    MQR_CHECK_HIP(hipStreamSynchronize(v->stream));
    return 0;
}

template <int RT>
static int point_passes(mqr_vbg* v, float thr, const ExScratch& e, mqr_geom* g) {
    const int64_t n = v->pool_count;
    hipLaunchKernelGGL(k_points<RT>, dim3((unsigned)n), dim3(kThreads), 0, v->stream, e.nb, n, v->bkeys, v->pool,
                       v->R, v->voxel_size, thr, e.c0, (const int32_t*)nullptr, (float*)nullptr, (float*)nullptr);
    MQR_CHECK_HIP(hipGetLastError());
    int64_t np = 0;
    if (scan_totals(v, e, n, 1, &np, nullptr)) return 1;
    g->nv = np;
    MQR_CHECK_HIP(hipMalloc(&g->pos, sizeof(float) * 3 * std::max<int64_t>(np, 1)));
    MQR_CHECK_HIP(hipMalloc(&g->nrm, sizeof(float) * 3 * std::max<int64_t>(np, 1)));
    hipLaunchKernelGGL(k_points<RT>, dim3((unsigned)n), dim3(kThreads), 0, v->stream, e.nb, n, v->bkeys, v->pool,
                       v->R, v->voxel_size, thr, e.c0, e.o0, g->pos, g->nrm);
    MQR_CHECK_HIP(hipGetLastError());
    MQR_CHECK_HIP(hipStreamSynchronize(v->stream));
    return 0;
}

}  // namespace mqr

using namespace mqr;

extern "C" {

int mqr_extract_mesh(mqr_vbg* v, float thr, mqr_geom** out) {
    MQR_REQUIRE(v && out, "null argument");
    MQR_REQUIRE(v->R <= kMaxR, "extract_triangle_mesh supports block_resolution <= 16");
    MQR_CHECK_HIP(hipSetDevice(v->device));
    if (sync_all(v)) return 1;  // an integrate may still be running on the second stream
    const int64_t n = v->pool_count;
    mqr_geom* g = new mqr_geom();
    g->device = v->device;
    *out = g;
    if (n == 0) return 0;
    ExScratch e{};
    if (ex_scratch(v, n, true, e) || build_nb(v, e.nb)) return 1;
    if (v->R == 16) return mesh_passes<16>(v, thr, e, g);
    if (v->R == 8) return mesh_passes<8>(v, thr, e, g);
    return mesh_passes<0>(v, thr, e, g);
}

int mqr_extract_points(mqr_vbg* v, float thr, mqr_geom** out) {
    MQR_REQUIRE(v && out, "null argument");
    MQR_REQUIRE(v->R <= kMaxR, "extract_point_cloud supports block_resolution <= 16");
    MQR_CHECK_HIP(hipSetDevice(v->device));
    if (sync_all(v)) return 1;
    const int64_t n = v->pool_count;
    mqr_geom* g = new mqr_geom();
    g->device = v->device;
    *out = g;
    if (n == 0) return 0;
    ExScratch e{};
    if (ex_scratch(v, n, false, e) || build_nb(v, e.nb)) return 1;
    if (v->R == 16) return point_passes<16>(v, thr, e, g);
    if (v->R == 8) return point_passes<8>(v, thr, e, g);
    return point_passes<0>(v, thr, e, g);
}

int mqr_geom_counts(mqr_geom* g, int64_t* nv, int64_t* nt) {
    MQR_REQUIRE(g, "null geometry");
    if (nv) *nv = g->nv;
    if (nt) *nt = g->nt;
    return 0;
}

int mqr_geom_copy(mqr_geom* g, float* positions, float* normals, int32_t* triangles, int loc) {
    MQR_REQUIRE(g, "null geometry");
    MQR_CHECK_HIP(hipSetDevice(g->device));
    const hipMemcpyKind k = loc == MQR_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
    if (positions && g->nv) MQR_CHECK_HIP(hipMemcpy(positions, g->pos, sizeof(float) * 3 * g->nv, k));
    if (normals && g->nv) MQR_CHECK_HIP(hipMemcpy(normals, g->nrm, sizeof(float) * 3 * g->nv, k));
    if (triangles && g->nt) MQR_CHECK_HIP(hipMemcpy(triangles, g->tri, sizeof(int32_t) * 3 * g->nt, k));
    return 0;
}

int mqr_geom_free(mqr_geom* g) {
    if (!g) return 0;
    (void)hipSetDevice(g->device);
    if (g->pos) (void)hipFree(g->pos);
    if (g->nrm) (void)hipFree(g->nrm);
    if (g->tri) (void)hipFree(g->tri);
    delete g;
    return 0;
}

}  // extern "C"

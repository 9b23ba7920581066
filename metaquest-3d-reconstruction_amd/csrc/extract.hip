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
//   R = 8 / 16 (k_mc_*):
//   k_mc_bits   the volume read once, coalesced: per block three bit planes (weight > thr,
//               tsdf < 0, tsdf > 0) of R^2 rows
//   k_mc_count  one workgroup per block: halo rows [-1, R]^3 rebuilt from the block's and its
//               neighbours' bit planes, cube classification, vertex / triangle counts, per-row
//               records (bases, owned edges / cubes) and sign rows for the emission pass
//               and, by decoupled look-back in the same pass, the blocks' output offsets
//   k_mc_emit   blocks with output only: vertices with tsdf values gathered from the pool,
//               triangles at their global offsets (latency: ~4 dependent load phases per block)
//   other R: the byte-tile kernels (k_mesh_count / k_mesh_emit) stage (tsdf, flags) tiles.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdlib>

#include <atomic>
#include <cstring>
#include <mutex>
#include <thread>
#include <tuple>
#include <vector>

#include "mqr_common.hpp"
#include "mqr_mc_tables.h"

namespace mqr {

constexpr int kMaxR = 16;
constexpr int kThreads = 512;  // 8 waves per workgroup: two LDS-resident blocks per CU keep 16 waves busy
// The bit-row kernels (R = 8 / 16) are latency-bound chains of small dependent loads per block:
// 256-thread workgroups (one per voxel row at R = 16) double the blocks in flight per CU.
constexpr int kMcThreads = 256;
constexpr uint32_t kAll27 = (1u << 27) - 1;  // presence mask of a block whose 26 neighbours all exist

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
// Compile-time R: every thread first issues all of its ceil(S^3 / kThreads) pool loads into
// registers and only then writes LDS, so a workgroup has ~14 loads per lane in flight instead of
// one latency-serialised load per loop trip.
template <int RT, bool TSDF>
__device__ void load_tile(uint8_t* __restrict__ flag, float* __restrict__ tsdf, const int32_t* __restrict__ nbrow,
                          const float2* __restrict__ pool, const Dims<RT>& d, float thr) {
    if constexpr (RT > 0) {
        constexpr int R = RT, S = RT + 3, S3 = S * S * S, R3 = R * R * R;
        constexpr int NIT = (S3 + kThreads - 1) / kThreads;
        float2 v[NIT];
        uint32_t present = 0;
#pragma unroll
        for (int k = 0; k < NIT; ++k) {
            const int i = threadIdx.x + k * kThreads;
            v[k] = make_float2(0.f, 0.f);
            if (i < S3) {
                const int lx = i % S - 1, ly = (i / S) % S - 1, lz = i / (S * S) - 1;
                const int dx = lx < 0 ? -1 : (lx >= R ? 1 : 0);
                const int dy = ly < 0 ? -1 : (ly >= R ? 1 : 0);
                const int dz = lz < 0 ? -1 : (lz >= R ? 1 : 0);
                const int nbuf = nbrow[(dx + 1) + 3 * (dy + 1) + 9 * (dz + 1)];
                if (nbuf >= 0) {
                    v[k] = pool[(int64_t)nbuf * R3 + ((lz - dz * R) * R + (ly - dy * R)) * R + (lx - dx * R)];
                    present |= 1u << k;
                }
            }
        }
#pragma unroll
        for (int k = 0; k < NIT; ++k) {
            const int i = threadIdx.x + k * kThreads;
            if (i < S3) {
                const bool p = (present >> k) & 1u;
                flag[i] = p ? (uint8_t)(1 | (v[k].y > thr ? 2 : 0) | (v[k].x < 0 ? 4 : 0)) : (uint8_t)0;
                if (TSDF) tsdf[i] = v[k].x;
            }
        }
        (void)d;
    } else {
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
}

// Marching-cubes tables staged in LDS: the lookups below are lane-divergent (one cube index per
// lane), which from __constant__ memory become serialised vector loads.
struct McLds {
    int8_t tri[256 * 16];
    uint8_t count[256];
};

__device__ inline void load_mc_tables(McLds& mc, bool tri) {
    for (int i = threadIdx.x; i < 256; i += blockDim.x) {
        mc.count[i] = (uint8_t)mqr_tri_count[i];
        if (tri) {
#pragma unroll
            for (int r = 0; r < 16; ++r) mc.tri[i * 16 + r] = mqr_tri_table[i][r];
        }
    }
}

// Edge e's owning-voxel shift (dx, dy, dz) and axis packed 5 bits per edge (mqr_edge_shifts).
__host__ __device__ constexpr uint64_t pack_edge_shifts() {
    constexpr int es[12][4] = {{0, 0, 0, 0}, {1, 0, 0, 1}, {0, 1, 0, 0}, {0, 0, 0, 1}, {0, 0, 1, 0}, {1, 0, 1, 1},
                               {0, 1, 1, 0}, {0, 0, 1, 1}, {0, 0, 0, 2}, {1, 0, 0, 2}, {1, 1, 0, 2}, {0, 1, 0, 2}};
    uint64_t r = 0;
    for (int e = 0; e < 12; ++e)
        r |= (uint64_t)(es[e][0] | es[e][1] << 1 | es[e][2] << 2 | es[e][3] << 3) << (5 * e);
    return r;
}
constexpr uint64_t kEdgeShifts = pack_edge_shifts();

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
__device__ void classify_mesh(const uint8_t* __restrict__ flag, MeshLocal<RT>& ml, const McLds& mc, const Dims<RT>& d,
                              int& nverts, int& ntris, int& tstart) {
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
        if (c & 0x100) tsum += mc.count[c & 0xff];
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
    __shared__ McLds mc;
    __shared__ int32_t nbrow[27];
    const Dims<RT> d(Rrt);
    const int R = d.R;
    const int64_t b = blockIdx.x;
    if (threadIdx.x < 27) nbrow[threadIdx.x] = nb[b * 27 + threadIdx.x];
    load_mc_tables(mc, false);
    __syncthreads();
    load_tile<RT, false>(tl.flag, nullptr, nbrow, pool, d, thr);
    __syncthreads();
    int nv, nt, ts;
    classify_mesh<RT>(tl.flag, ml, mc, d, nv, nt, ts);
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
    __shared__ McLds mc;
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
    load_mc_tables(mc, true);
    __syncthreads();
    load_tile<RT, true>(tl.flag, tl.tsdf, nbrow, pool, d, thr);
    __syncthreads();
    int nv, nt, tstart;
    classify_mesh<RT>(tl.flag, ml, mc, d, nv, nt, tstart);
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
        const int8_t* trow = mc.tri + ci * 16;
        for (int r = 0; r < 16; r += 3) {
            if (trow[r] == -1) break;
            for (int k = 0; k < 3; ++k) {
                const int edge = trow[r + k];
                const uint32_t es = (uint32_t)(kEdgeShifts >> (5 * edge));
                const int ox = x + (int)(es & 1u), oy = y + (int)((es >> 1) & 1u), oz = z + (int)((es >> 2) & 1u);
                const int axis = (int)((es >> 3) & 3u);
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

// ================================================================ bit-row marching cubes (R = 8 / 16)
// The tile's per-voxel predicates are kept as bit rows: for tile row q = (z + 1) * S + (y + 1),
// bit (x + 1) of rowV[q] / rowN[q] is "weight > thr" / "tsdf < 0" of voxel x in [-1, R + 1]
// (absent voxels: 0, 0).  Cube validity (AND of the four corner rows and of adjacent bits), the cube
// index and the owned crossing edges of a whole x-row then take a few word operations instead of
// per-voxel byte lookups in LDS (which the byte-granular bank conflicts made the bottleneck of the
// per-voxel kernels above: SQ_LDS_IDX_ACTIVE ~ 80 % of k_mesh_count's time).  Vertices and
// triangles are emitted by a balanced thread-per-output loop (binary search over the per-row
// prefix), in the same (block, voxel, edge) / (block, cube, triangle) order as the kernels above.
// HI = 1: tile [-1, R]^3 (classification; both passes -- the emit pass reads its tsdf values from the pool).
template <int R, int HI>
struct Mc {
    static constexpr int S = R + 1 + HI, S2 = S * S, C = R + 1, C2 = C * C, R2 = R * R, R3 = R * R * R;
    static constexpr int NH = 1 + HI;                  // halo columns x = -1 and x = R .. R + HI - 1
    static constexpr int RPW = 64 / R;                 // tile rows per wave-wide ballot
    static constexpr int NG = (S2 + RPW - 1) / RPW;    // ballot groups
    static constexpr uint32_t RMASK = (1u << R) - 1;
    static constexpr uint32_t CMASK = (1u << C) - 1;
    static_assert(R == 8 || R == 16, "bit-row kernels: R = 8 or 16");
    static_assert(HI == 1 || HI == 2, "tile upper halo: 1 or 2");
    static_assert(R2 <= kMcThreads, "one thread per voxel row");
    __device__ static int q(int y, int z) { return (z + 1) * S + (y + 1); }
    __device__ static int c(int y, int z) { return (z + 1) * C + (y + 1); }
    __device__ static int t(int x, int y, int z) { return q(y, z) * S + (x + 1); }
    __device__ static int blk(int v) { return v < 0 ? -1 : (v >= R ? 1 : 0); }
    __device__ static int k27(int x, int y, int z) { return (blk(x) + 1) + 3 * (blk(y) + 1) + 9 * (blk(z) + 1); }
};

// ---- bits pass: every voxel read once, fully coalesced -------------------------------------------
// Per block three bit planes of R^2 rows of R bits (u16, row = z R + y, bit = x): weight > thr
// (V), tsdf < 0 (N), tsdf > 0 (P).  NaN sets neither N nor P, like the upstream comparisons.  The
// classification and emission passes rebuild their halo rows from these (~3 KB per block instead
// of re-reading the (R+2)^3 neighbourhood of float2 voxels, 2.6x the volume over two passes).
// The same launch also fills the block's row of the 27-neighbour table (hash lookups, k_nb).
template <int R>
__global__ __launch_bounds__(kMcThreads) void k_mc_bits(const float2* __restrict__ pool, float thr,
                                                        uint16_t* __restrict__ bits, const uint64_t* __restrict__ bkeys,
                                                        const Table t, int32_t* __restrict__ nb) {
    constexpr int R2 = R * R, R3 = R2 * R, NIT = (R3 + kMcThreads - 1) / kMcThreads, RPB = 64 / R;
    constexpr uint64_t RM = (1ull << R) - 1;
    const int64_t b = blockIdx.x;
    const float2* __restrict__ src = pool + b * R3;
    const int tid = threadIdx.x, lane = tid & 63;
    float2 v[NIT];
#pragma unroll
    for (int it = 0; it < NIT; ++it) {  // all loads in flight before the ballots
        const int i = it * kMcThreads + tid;
        v[it] = i < R3 ? src[i] : make_float2(0.f, 0.f);
    }
    if (tid < 27) {
        int x, y, z;
        unpack_key(bkeys[b], x, y, z);
        x += tid % 3 - 1;
        y += (tid % 9) / 3 - 1;
        z += tid / 9 - 1;
        int32_t r = -1;
        if (key_in_range(x, y, z)) {
            const int64_t sl = dev_find(t, pack_key(x, y, z));
            if (sl >= 0) r = t.vals[sl];
        }
        nb[b * 27 + tid] = r;
    }
    uint16_t* __restrict__ out = bits + b * 3 * R2;
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
        const int i = it * kMcThreads + tid;
        const bool in = i < R3;
        const uint64_t mv = __ballot(in && v[it].y > thr);
        const uint64_t mn = __ballot(in && v[it].x < 0.f);
        const uint64_t mp = __ballot(in && v[it].x > 0.f);
        const int i0 = i - lane;  // the wave's first voxel
        if (lane < RPB && i0 + lane * R < R3) {
            const int row = i0 / R + lane;
            out[row] = (uint16_t)((mv >> (lane * R)) & RM);
            out[R2 + row] = (uint16_t)((mn >> (lane * R)) & RM);
            out[2 * R2 + row] = (uint16_t)((mp >> (lane * R)) & RM);
        }
    }
}

// Tile rows of the block's [-1, R + HI - 1] neighbourhood from the bit planes: bit (x + 1) of
// rowV[q] / rowN[q] (/ rowP[q]) for tile row q = (z + 1) S + (y + 1); absent blocks give 0 bits.
template <class M>
__device__ void mc_stage_bits(const int32_t* __restrict__ nbrow, const uint16_t* __restrict__ bits, uint32_t* rowV,
                              uint32_t* rowN, uint32_t* rowP) {
    constexpr int R = M::C - 1, R2 = R * R;
    for (int q = threadIdx.x; q < M::S2; q += blockDim.x) {
        const int ty = q % M::S - 1, tz = q / M::S - 1;
        const int dy = M::blk(ty), dz = M::blk(tz);
        const int row = (tz - dz * R) * R + (ty - dy * R);
        const int k0 = 3 * (dy + 1) + 9 * (dz + 1);
        const int32_t bm = nbrow[k0], bc = nbrow[k0 + 1], bp = nbrow[k0 + 2];
        uint32_t w[3];
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            if (a == 2 && !rowP) break;
            uint32_t x = 0;
            if (bc >= 0) x = (uint32_t)bits[((int64_t)bc * 3 + a) * R2 + row] << 1;
            if (bm >= 0) x |= ((uint32_t)bits[((int64_t)bm * 3 + a) * R2 + row] >> (R - 1)) & 1u;
            if (bp >= 0) {
                const uint32_t pb = bits[((int64_t)bp * 3 + a) * R2 + row];
#pragma unroll
                for (int h = 0; h < M::NH - 1; ++h) x |= ((pb >> h) & 1u) << (R + 1 + h);
            }
            w[a] = x;
        }
        rowV[q] = w[0];
        rowN[q] = w[1];
        if (rowP) rowP[q] = w[2];
    }
    __syncthreads();
}

// Surface cubes per cube row (origins y, z in [-1, R-1]): bit (x + 1) set iff the cube at origin x
// has all 8 corners with weight > thr and an index other than 0 / 255.  (An edge with a sign change
// next to a valid cube makes that cube mixed, so edge ownership can test these bits.)
template <class M>
__device__ void mc_cubes(const uint32_t* rowV, const uint32_t* rowN, uint32_t* cs) {
    for (int i = threadIdx.x; i < M::C2; i += blockDim.x) {
        const int cy = i % M::C - 1, cz = i / M::C - 1;
        const int q00 = M::q(cy, cz), q10 = M::q(cy + 1, cz), q01 = M::q(cy, cz + 1), q11 = M::q(cy + 1, cz + 1);
        const uint32_t v4 = rowV[q00] & rowV[q10] & rowV[q01] & rowV[q11];
        const uint32_t no = rowN[q00] | rowN[q10] | rowN[q01] | rowN[q11];
        const uint32_t na = rowN[q00] & rowN[q10] & rowN[q01] & rowN[q11];
        cs[i] = (v4 & (v4 >> 1)) & (no | (no >> 1)) & ~(na & (na >> 1)) & M::CMASK;
    }
}

// Owned crossing edges (bit x = voxel x of row (y, z) owns a vertex on its +x / +y / +z edge) and
// owned surface cubes (oc) of one voxel row.
struct RowEdges {
    uint32_t ex, ey, ez, oc;
};

template <class M>
__device__ inline RowEdges mc_row(const uint32_t* rowN, const uint32_t* cs, int y, int z) {
    const uint32_t n0 = rowN[M::q(y, z)];
    const uint32_t c00 = cs[M::c(y, z)], cym = cs[M::c(y - 1, z)], czm = cs[M::c(y, z - 1)];
    const uint32_t cyzm = cs[M::c(y - 1, z - 1)];
    RowEdges e;
    e.ex = (((n0 ^ (n0 >> 1)) & (c00 | cym | czm | cyzm)) >> 1) & M::RMASK;  // cubes (x,y,z) (x,y-1,z) (x,y,z-1) (x,y-1,z-1)
    const uint32_t a = c00 | czm;                                             // + the same at x - 1
    e.ey = (((n0 ^ rowN[M::q(y + 1, z)]) & (a | (a << 1))) >> 1) & M::RMASK;
    const uint32_t b = c00 | cym;
    e.ez = (((n0 ^ rowN[M::q(y, z + 1)]) & (b | (b << 1))) >> 1) & M::RMASK;
    e.oc = (c00 >> 1) & M::RMASK;
    return e;
}

// Cube index of the cube at origin x from the four corner rows shifted right by x + 1.
__device__ inline int mc_index(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    return (int)((a & 1) | (a & 2) | ((b & 2) << 1) | ((b & 1) << 3) | ((c & 1) << 4) | ((c & 2) << 4) |
                 ((d & 2) << 5) | ((d & 1) << 7));
}
__device__ inline int mc_tri_count(int ci) { return (int)((mqr_tri_count_packed[ci >> 3] >> ((ci & 7) * 4)) & 0xFu); }

// (nib: the per-cube counts as 4-bit fields, field x = the cube at origin x, for the emission pass)
template <class M>
__device__ inline int mc_row_tris(const uint32_t* rowN, uint32_t oc, int y, int z, uint64_t* nib = nullptr) {
    const uint32_t a = rowN[M::q(y, z)], b = rowN[M::q(y + 1, z)], c = rowN[M::q(y, z + 1)];
    const uint32_t d = rowN[M::q(y + 1, z + 1)];
    int n = 0;
    uint64_t w = 0;
    while (oc) {
        const int x = __builtin_ctz(oc);
        oc &= oc - 1;
        const int k = mc_tri_count(mc_index(a >> (x + 1), b >> (x + 1), c >> (x + 1), d >> (x + 1)));
        n += k;
        w |= (uint64_t)k << (4 * x);
    }
    if (nib) *nib = w;
    return n;
}

// Per-block counts and, per voxel row, the record the emission pass works from:
//   rows4[b][row] = {vertex base in the block, triangle base in the block, ex | ey << 16, ez | oc << 16}
// (owned crossing edges and owned surface cubes of the row) and the sign rows rowNt[b][q] of the
// block's [-1, R]^3 tile (cube indices).  Emission of this block and of its -x / -y / -z
// neighbours (triangles referencing vertices this block owns) read these instead of rebuilding them.
// NIB: also the rows' per-cube triangle counts (rowsT[b][row], mc_row_tris) for the emission pass.
template <int R, bool NIB = false>
__global__ __launch_bounds__(kMcThreads) void k_mc_count(const int32_t* __restrict__ nb, const uint16_t* __restrict__ bits,
                                                         int64_t tri_blocks, int32_t* vcount, int32_t* tcount,
                                                         uint4* __restrict__ rows4, uint32_t* __restrict__ rowNt,
                                                         uint64_t* __restrict__ rowsT = nullptr) {
    using M = Mc<R, 1>;
    __shared__ uint32_t rowV[M::S2], rowN[M::S2], cs[M::C2];
    __shared__ int32_t nbrow[27];
    __shared__ int scratch[16];
    const int64_t b = blockIdx.x;
    if (threadIdx.x < 27) nbrow[threadIdx.x] = nb[b * 27 + threadIdx.x];
    __syncthreads();
    mc_stage_bits<M>(nbrow, bits, rowV, rowN, nullptr);
    mc_cubes<M>(rowV, rowN, cs);
    __syncthreads();
    const int r = threadIdx.x;
    RowEdges e{0, 0, 0, 0};
    int nv = 0, nt = 0;
    uint64_t tw = 0;
    if (r < M::R2) {
        e = mc_row<M>(rowN, cs, r % R, r / R);
        if (b >= tri_blocks) e.oc = 0;  // halo block of a shard: its vertices, none of its cubes
        nv = __popc(e.ex) + __popc(e.ey) + __popc(e.ez);
        nt = mc_row_tris<M>(rowN, e.oc, r % R, r / R, NIB ? &tw : nullptr);
        if constexpr (NIB) rowsT[b * M::R2 + r] = tw;
    }
    int vtot, ttot;
    const int vb = block_exclusive_scan(nv, scratch, vtot);
    const int tb = block_exclusive_scan(nt, scratch + 8, ttot);
    if (r < M::R2) rows4[b * M::R2 + r] = make_uint4((uint32_t)vb, (uint32_t)tb, e.ex | (e.ey << 16), e.ez | (e.oc << 16));
    for (int q = threadIdx.x; q < M::S2; q += blockDim.x) rowNt[b * M::S2 + q] = rowN[q];
    if (threadIdx.x == 0) {
        vcount[b] = vtot;
        tcount[b] = ttot;
    }
}

// tsdf of tile point (x, y, z) in [-1, R + 1]^3 (its block present), read from the pool.
template <class M>
__device__ inline float mc_tsdf(const int32_t* __restrict__ nbrow, const float2* __restrict__ pool, int x, int y,
                                int z) {
    constexpr int R = M::C - 1;
    const int dx = M::blk(x), dy = M::blk(y), dz = M::blk(z);
    const int32_t nbuf = nbrow[(dx + 1) + 3 * (dy + 1) + 9 * (dz + 1)];
    return pool[(int64_t)nbuf * M::R3 + ((z - dz * R) * R + (y - dy * R)) * R + (x - dx * R)].x;
}

// Central-difference normal at tile point (x, y, z), components left untouched where a side's
// block is absent (upstream DeviceGetNormal; presence is per block: bit k27 of pres).
template <class M>
__device__ inline void mc_normal(const int32_t* __restrict__ nbrow, const float2* __restrict__ pool, uint32_t pres,
                                 int x, int y, int z, float* n) {
    auto present = [&](int a, int b, int c) { return (pres >> M::k27(a, b, c)) & 1u; };
    if (present(x + 1, y, z) && present(x - 1, y, z))
        n[0] = mc_tsdf<M>(nbrow, pool, x + 1, y, z) - mc_tsdf<M>(nbrow, pool, x - 1, y, z);
    if (present(x, y + 1, z) && present(x, y - 1, z))
        n[1] = mc_tsdf<M>(nbrow, pool, x, y + 1, z) - mc_tsdf<M>(nbrow, pool, x, y - 1, z);
    if (present(x, y, z + 1) && present(x, y, z - 1))
        n[2] = mc_tsdf<M>(nbrow, pool, x, y, z + 1) - mc_tsdf<M>(nbrow, pool, x, y, z - 1);
}

// Everything a vertex / point on the edge (o, o + axis) needs when all 27 blocks of the neighbourhood
// are present (then every normal component is written, so upstream's per-voxel normal scratch
// carries nothing across the voxel's edges and only this edge's normals matter): the 13 tsdf taps
// -- o, o +- x/y/z, e = o + axis, e +- x/y/z -- issued as one batch of loads.
template <class M>
__device__ inline void mc_edge_full(const int32_t* __restrict__ nbrow, const float2* __restrict__ pool, int x, int y,
                                    int z, int axis, float& t_o, float& t_e, float* no, float* ne) {
    const int ex = x + (axis == 0), ey = y + (axis == 1), ez = z + (axis == 2);
    const int px[13] = {x, x + 1, x - 1, x, x, x, x, ex + 1, ex - 1, ex, ex, ex, ex};
    const int py[13] = {y, y, y, y + 1, y - 1, y, y, ey, ey, ey + 1, ey - 1, ey, ey};
    const int pz[13] = {z, z, z, z, z, z + 1, z - 1, ez, ez, ez, ez, ez + 1, ez - 1};
    float v[13];
#pragma unroll
    for (int j = 0; j < 13; ++j) v[j] = mc_tsdf<M>(nbrow, pool, px[j], py[j], pz[j]);
    t_o = v[0];
    t_e = axis == 0 ? v[1] : axis == 1 ? v[3] : v[5];
    no[0] = v[1] - v[2];
    no[1] = v[3] - v[4];
    no[2] = v[5] - v[6];
    ne[0] = v[7] - v[8];
    ne[1] = v[9] - v[10];
    ne[2] = v[11] - v[12];
}

// mc_edge_full with a fast path for an edge whose 13 taps all lie inside the block (~60 % of the
// edges at R = 16): one base address and constant offsets instead of a 27-neighbour lookup and a
// 64-bit address per tap -- the same values, so the same results.
template <class M>
__device__ inline void mc_edge_taps(const int32_t* __restrict__ nbrow, const float2* __restrict__ pool, int x, int y,
                                    int z, int axis, float& t_o, float& t_e, float* no, float* ne) {
    constexpr int R = M::C - 1, DY = R, DZ = R * R;
    const int ex = x + (axis == 0), ey = y + (axis == 1), ez = z + (axis == 2);
    if (min(min(x, y), z) >= 1 && max(max(ex, ey), ez) <= R - 2) {
        const float2* c = pool + (int64_t)nbrow[13] * M::R3 + (z * R + y) * R + x;
        const float2* e = c + (axis == 0 ? 1 : axis == 1 ? DY : DZ);
        const float vxp = c[1].x, vxm = c[-1].x, vyp = c[DY].x, vym = c[-DY].x, vzp = c[DZ].x, vzm = c[-DZ].x;
        const float wxp = e[1].x, wxm = e[-1].x, wyp = e[DY].x, wym = e[-DY].x, wzp = e[DZ].x, wzm = e[-DZ].x;
        t_o = c[0].x;
        t_e = axis == 0 ? vxp : axis == 1 ? vyp : vzp;
        no[0] = vxp - vxm;
        no[1] = vyp - vym;
        no[2] = vzp - vzm;
        ne[0] = wxp - wxm;
        ne[1] = wyp - wym;
        ne[2] = wzp - wzm;
    } else {
        mc_edge_full<M>(nbrow, pool, x, y, z, axis, t_o, t_e, no, ne);
    }
}

// The k-th output of a row whose outputs are ordered by (x, axis) with per-axis bit rows ex / ey /
// ez: x = the largest x with (outputs below x) <= k, by binary search on prefix popcounts; k becomes
// the rank of the output among voxel x's axes.
template <int R>
__device__ __forceinline__ void row_select(uint32_t ex, uint32_t ey, uint32_t ez, int& k, int& x) {
    auto below = [&](int c) {
        const uint32_t low = (1u << c) - 1;
        return __popc(ex & low) + __popc(ey & low) + __popc(ez & low);
    };
    x = 0;
#pragma unroll
    for (int st = R / 2; st >= 1; st >>= 1)
        if (below(x + st) <= k) x += st;
    k -= below(x);
}

// Global vertex id of the edge owned by voxel (ox, oy, oz) (may lie in a +x/+y/+z neighbour) along axis.
__device__ inline int32_t mc_vid(uint32_t vbase, uint32_t ex, uint32_t ey, uint32_t ez, int x, int axis) {
    const uint32_t low = (1u << x) - 1;
    return (int32_t)(vbase + __popc(ex & low) + __popc(ey & low) + __popc(ez & low) +
                     (axis > 0 ? (ex >> x) & 1u : 0u) + (axis > 1 ? (ey >> x) & 1u : 0u));
}

// Vertex i of a block (emission pass): its row by binary search over the row vertex bases, its voxel
// and edge by row_select, position and normal from the tsdf taps of the pool.
// The last row whose vertex (F = 0) / triangle (F = 1) base is <= i, i.e. the (non-empty) row of output i.
template <int R2, int F>
__device__ __forceinline__ int row_search(const uint4* rows, int i) {
    int lo = 0, hi = R2 - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if ((int)(F == 0 ? rows[mid].x : rows[mid].y) <= i) lo = mid; else hi = mid - 1;
    }
    return lo;
}

template <class M>
__device__ __forceinline__ void mc_emit_vertex(int i, int lo, const uint4* rows, const int32_t* nbrow,
                                               const float2* __restrict__ pool, uint32_t pres, int xb, int yb, int zb,
                                               float voxel_size, int32_t vb0, float* pos, float* nrm) {
    constexpr int R = M::C - 1;
    const uint4 rw = rows[lo];
    const uint32_t ex = rw.z & 0xffffu, ey = rw.z >> 16, ez = rw.w & 0xffffu;
    int k = i - (int)rw.x, x;
    row_select<R>(ex, ey, ez, k, x);
    const uint32_t m3 = ((ex >> x) & 1u) | (((ey >> x) & 1u) << 1) | (((ez >> x) & 1u) << 2);
    const int y = lo % R, z = lo / R;
    float tsdf_o, tsdf_e;
    float no[3] = {0.f, 0.f, 0.f}, ne[3] = {0.f, 0.f, 0.f};
    int axis = 0;
    if (pres == kAll27) {  // block-uniform
        uint32_t mm = m3;
        for (int j = 0; j < k; ++j) mm &= mm - 1;
        axis = __builtin_ctz(mm);
        mc_edge_taps<M>(nbrow, pool, x, y, z, axis, tsdf_o, tsdf_e, no, ne);
    } else {
        tsdf_o = mc_tsdf<M>(nbrow, pool, x, y, z);
        mc_normal<M>(nbrow, pool, pres, x, y, z, no);
        // upstream keeps one per-voxel normal scratch across the voxel's edges: replay the earlier ones
        uint32_t mm = m3;
        for (int j = 0;; ++j) {
            axis = __builtin_ctz(mm);
            mc_normal<M>(nbrow, pool, pres, x + (axis == 0), y + (axis == 1), z + (axis == 2), ne);
            if (j == k) break;
            mm &= mm - 1;
        }
        tsdf_e = mc_tsdf<M>(nbrow, pool, x + (axis == 0), y + (axis == 1), z + (axis == 2));
    }
    const float ratio = (0 - tsdf_o) / (tsdf_e - tsdf_o);
    const float rx = ratio * (int)(axis == 0), ry = ratio * (int)(axis == 1), rz = ratio * (int)(axis == 2);
    const int gx = xb * R + x, gy = yb * R + y, gz = zb * R + z;
    const int64_t id = (int64_t)vb0 + i;
    pos[3 * id + 0] = voxel_size * (gx + rx);
    pos[3 * id + 1] = voxel_size * (gy + ry);
    pos[3 * id + 2] = voxel_size * (gz + rz);
    const float nx = (1 - ratio) * no[0] + ratio * ne[0];
    const float ny = (1 - ratio) * no[1] + ratio * ne[1];
    const float nz = (1 - ratio) * no[2] + ratio * ne[2];
    write_normal(nx, ny, nz, nrm + 3 * id);
}

// Triangle i of a block (emission pass): its cube by binary search over the row triangle bases and a
// walk over the row's owned cubes, its three vertex ids from the row records (this block's in LDS,
// a +x / +y / +z neighbour's from rows4).
// (tcs: the rows' per-cube triangle counts (NIB) -- the cube found by skipping 4-bit fields in
// registers instead of a walk with a table lookup per cube)
template <class M, bool NIB>
__device__ __forceinline__ void mc_emit_tri(int i, int lo, const uint4* rows, const uint64_t* tcs, const uint32_t* rowN,
                                            const uint32_t* triC, const uint64_t* triP, const int32_t* nbrow,
                                            const int32_t* __restrict__ voff, const uint4* __restrict__ rows4,
                                            int32_t vb0, int32_t tb0, int32_t* tri) {
    constexpr int R = M::C - 1;
    const uint4 rw = rows[lo];
    const int y = lo % R, z = lo / R;
    const uint32_t a = rowN[M::q(y, z)], bb = rowN[M::q(y + 1, z)], c = rowN[M::q(y, z + 1)];
    const uint32_t d = rowN[M::q(y + 1, z + 1)];
    int k = i - (int)rw.y, x = 0, ci = 0;
    if constexpr (NIB) {
        uint64_t w = tcs[lo];  // non-zero fields = the owned surface cubes; k < their sum
        for (;;) {
            const int s = __builtin_ctzll(w) & ~3;
            w >>= s;
            x += s >> 2;
            const int n = (int)(w & 0xFu);
            if (k < n) break;
            k -= n;
            w >>= 4;
            ++x;
        }
        ci = mc_index(a >> (x + 1), bb >> (x + 1), c >> (x + 1), d >> (x + 1));
    } else {
        uint32_t oc = rw.w >> 16;
        while (oc) {
            x = __builtin_ctz(oc);
            ci = mc_index(a >> (x + 1), bb >> (x + 1), c >> (x + 1), d >> (x + 1));
            const int n = (int)((triC[ci >> 3] >> ((ci & 7) * 4)) & 0xFu);
            if (k < n) break;
            k -= n;
            oc &= oc - 1;
        }
    }
    const uint64_t te = triP[ci] >> (12 * k);
    const int64_t t = (int64_t)tb0 + i;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const int edge = (int)((te >> (4 * j)) & 0xFu);
        const uint32_t es = (uint32_t)(kEdgeShifts >> (5 * edge));
        const int ox = x + (int)(es & 1u), oy = y + (int)((es >> 1) & 1u), oz = z + (int)((es >> 2) & 1u);
        const int axis = (int)((es >> 3) & 3u);
        int32_t vid;
        if (ox < R && oy < R && oz < R) {
            const uint4 ow = rows[oz * R + oy];
            vid = vb0 + mc_vid(ow.x, ow.z & 0xffffu, ow.z >> 16, ow.w & 0xffffu, ox, axis);
        } else {
            const int dx = ox >= R, dy = oy >= R, dz = oz >= R;
            const int k27 = (dx + 1) + 3 * (dy + 1) + 9 * (dz + 1);
            const int32_t nbuf = nbrow[k27];
            if (nbuf < 0) {
                vid = -1;  // cannot happen for a valid cube (all corners exist); stay in bounds
            } else {
                const int lx = ox - dx * R, ly = oy - dy * R, lz = oz - dz * R;
                const uint4 ow = rows4[(int64_t)nbuf * M::R2 + lz * R + ly];
                // (the neighbour's block offset read here, beside its row record, not in the prologue:
                // one dependent global round trip fewer before the block's first barrier)
                vid = voff[nbuf] + mc_vid(ow.x, ow.z & 0xffffu, ow.z >> 16, ow.w & 0xffffu, lx, axis);
            }
        }
        tri[3 * t + (2 - j)] = vid;
    }
}

// Emission of a block with vertices or triangles, from the count pass's row records: vertices
// (positions and normals from tsdf values gathered from the pool) and triangles at the offsets of
// the scan, in (block, voxel, edge) / (block, cube, triangle) order.  role 0: both (one workgroup per
// block, vertices then triangles); 1: vertices only; 2: triangles only (timing diagnostics).
// (A merged vertex / triangle item loop, 512-thread blocks and a vertex and a triangle workgroup per
// block were measured: no change or slower)
// MAP: blocks with at most kRowMap vertices / triangles find each output's row in an LDS byte map
// (filled by one pass over the rows) instead of by a binary search over the row bases.
constexpr int kRowMap = 2048;

template <int R, int NT, bool NIB = false, bool MAP = false>
__device__ __forceinline__ void mc_emit_block(int64_t b, int role, const int32_t* __restrict__ nb,
                                              const uint64_t* __restrict__ bkeys, const float2* __restrict__ pool,
                                              float voxel_size, const int32_t* __restrict__ vcount,
                                              const int32_t* __restrict__ tcount, const int32_t* __restrict__ voff,
                                              const int32_t* __restrict__ toff, const uint4* __restrict__ rows4,
                                              const uint32_t* __restrict__ rowNt, float* pos, float* nrm, int32_t* tri,
                                              int64_t cap_v, int64_t cap_t, const uint64_t* __restrict__ rowsT) {
    using M = Mc<R, 1>;
    static_assert(NT >= 256, "one thread per triangle-table row");
    static_assert(M::R2 <= 256, "row ids in bytes");
    __shared__ uint32_t rowN[M::S2];
    __shared__ uint4 rows[M::R2];  // vbase, tbase, ex | ey << 16, ez | oc << 16
    __shared__ int32_t nbrow[27];
    __shared__ uint64_t triP[256];  // the triangle tables: lane-divergent lookups in a dependent loop
    __shared__ uint32_t triC[32];
    __shared__ uint64_t tcs[NIB ? M::R2 : 1];
    __shared__ uint8_t vmap[MAP ? kRowMap : 1], tmap[MAP ? kRowMap : 1];
    const int nvb = role == 2 ? 0 : vcount[b], ntb = role == 1 ? 0 : tcount[b];
    if (nvb == 0 && ntb == 0) return;  // block-uniform: nothing to write
    const int32_t vb0 = voff[b], tb0 = toff[b];
    // outputs past the speculative capacity: the host re-runs this pass into exact buffers
    // (int32 offsets: a total past 2^31 wraps them negative -- the host then fails the call after
    // this speculative pass, which must not have written before the buffers' start)
    if (vb0 < 0 || tb0 < 0 || (int64_t)vb0 + vcount[b] > cap_v || (int64_t)tb0 + tcount[b] > cap_t) return;
    const int tid = threadIdx.x;
    if (ntb) {
        if (tid < 256) triP[tid] = mqr_tri_packed[tid];
        if (tid < 32) triC[tid] = mqr_tri_count_packed[tid];
    }
    if (tid < 27) nbrow[tid] = nb[b * 27 + tid];
    for (int r = tid; r < M::R2; r += NT) rows[r] = rows4[b * M::R2 + r];
    if (ntb) {
        for (int q = tid; q < M::S2; q += NT) rowN[q] = rowNt[b * M::S2 + q];
        if constexpr (NIB)
            for (int r = tid; r < M::R2; r += NT) tcs[r] = rowsT[b * M::R2 + r];
    }
    __syncthreads();
    const bool vm = MAP && nvb <= kRowMap, tm = MAP && ntb <= kRowMap;  // block-uniform
    if (vm || tm) {
        for (int r = tid; r < M::R2; r += NT) {
            const uint4 rw = rows[r];
            if (vm) {
                const int e = min(r + 1 < M::R2 ? (int)rows[r + 1].x : nvb, nvb);
                for (int j = (int)rw.x; j < e; ++j) vmap[j] = (uint8_t)r;
            }
            if (tm) {
                const int e = min(r + 1 < M::R2 ? (int)rows[r + 1].y : ntb, ntb);
                for (int j = (int)rw.y; j < e; ++j) tmap[j] = (uint8_t)r;
            }
        }
        __syncthreads();
    }
    if (nvb) {
        const int lane = tid & 63;
        const uint32_t pres = (uint32_t)__ballot(lane < 27 && nbrow[lane < 27 ? lane : 0] >= 0);
        int xb, yb, zb;
        unpack_key(bkeys[b], xb, yb, zb);
        for (int i = tid; i < nvb; i += NT) {
            const int lo = vm ? (int)vmap[i] : row_search<M::R2, 0>(rows, i);
            mc_emit_vertex<M>(i, lo, rows, nbrow, pool, pres, xb, yb, zb, voxel_size, vb0, pos, nrm);
        }
    }
    for (int i = tid; i < ntb; i += NT) {
        const int lo = tm ? (int)tmap[i] : row_search<M::R2, 1>(rows, i);
        mc_emit_tri<M, NIB>(i, lo, rows, tcs, rowN, triC, triP, nbrow, voff, rows4, vb0, tb0, tri);
    }
}

// diag (A/B library, MQR_EMIT_DIAG): 1 vertices only, 2 triangles only (timing of one half, wrong output)
template <int R, bool NIB = false, bool MAP = false, int NT = kMcThreads>
__global__ __launch_bounds__(NT) void k_mc_emit(const int32_t* __restrict__ nb, const uint64_t* __restrict__ bkeys,
                                                const float2* __restrict__ pool, float voxel_size,
                                                const int32_t* __restrict__ vcount, const int32_t* __restrict__ tcount,
                                                const int32_t* __restrict__ voff, const int32_t* __restrict__ toff,
                                                const uint4* __restrict__ rows4, const uint32_t* __restrict__ rowNt,
                                                float* pos, float* nrm, int32_t* tri, int64_t cap_v, int64_t cap_t,
                                                const uint64_t* __restrict__ rowsT, int diag = 0) {
#if !MQR_AB
    diag = 0;
#endif
    mc_emit_block<R, NT, NIB, MAP>(blockIdx.x, diag, nb, bkeys, pool, voxel_size, vcount, tcount, voff, toff, rows4,
                                   rowNt, pos, nrm, tri, cap_v, cap_t, rowsT);
}


// (A decoupled look-back inside the count pass, one word per step or 64 per step, made the C2 count
// pass 99 / 77 us against 31 + 5 here: each step is a cross-XCD round trip.)
// Exclusive scans of the two per-block count arrays (vertices, triangles) in one workgroup of
// kScanThreads; totals[0..1] = the sums.  (Two hipcub scans cost ~20 us of launches at these sizes.)
// Tiles of kScanTile counts: coalesced loads, all of a thread's in flight, staged in LDS; each
// thread scans kScanPer consecutive counts, wave and workgroup scans of the thread sums; results
// back through LDS to coalesced stores; a running carry between tiles.
constexpr int kScanThreads = 1024, kScanPer = 8, kScanTile = kScanThreads * kScanPer;
__global__ __launch_bounds__(kScanThreads) void k_scan_counts(const int32_t* __restrict__ c0,
                                                              const int32_t* __restrict__ c1, int64_t n,
                                                              int32_t* __restrict__ o0, int32_t* __restrict__ o1,
                                                              int64_t* __restrict__ totals) {
    __shared__ int32_t t0[kScanTile], t1[kScanTile];
    __shared__ int64_t ws0[kScanThreads / 64], ws1[kScanThreads / 64];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const bool two = c1 != nullptr;
    int64_t carry0 = 0, carry1 = 0;
    for (int64_t base = 0; base < n; base += kScanTile) {
        int32_t v0[kScanPer], v1[kScanPer];
#pragma unroll
        for (int k = 0; k < kScanPer; ++k) {
            const int64_t i = base + k * kScanThreads + tid;
            v0[k] = i < n ? c0[i] : 0;
            v1[k] = two && i < n ? c1[i] : 0;
        }
#pragma unroll
        for (int k = 0; k < kScanPer; ++k) {
            t0[k * kScanThreads + tid] = v0[k];
            t1[k * kScanThreads + tid] = v1[k];
        }
        __syncthreads();
        int64_t s0 = 0, s1 = 0;
#pragma unroll
        for (int k = 0; k < kScanPer; ++k) {
            s0 += t0[tid * kScanPer + k];
            s1 += t1[tid * kScanPer + k];
        }
        int64_t i0 = s0, i1 = s1;  // inclusive wave scans of the thread sums
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int64_t a = __shfl_up(i0, d, 64), b = __shfl_up(i1, d, 64);
            if (lane >= d) {
                i0 += a;
                i1 += b;
            }
        }
        if (lane == 63) {
            ws0[wave] = i0;
            ws1[wave] = i1;
        }
        __syncthreads();
        int64_t b0 = carry0, b1 = carry1, tot0 = 0, tot1 = 0;
        for (int w = 0; w < kScanThreads / 64; ++w) {
            if (w < wave) {
                b0 += ws0[w];
                b1 += ws1[w];
            }
            tot0 += ws0[w];
            tot1 += ws1[w];
        }
        int64_t r0 = b0 + i0 - s0, r1 = b1 + i1 - s1;  // exclusive prefix of this thread's counts
#pragma unroll
        for (int k = 0; k < kScanPer; ++k) {
            const int32_t a = t0[tid * kScanPer + k], b = t1[tid * kScanPer + k];
            t0[tid * kScanPer + k] = (int32_t)r0;
            t1[tid * kScanPer + k] = (int32_t)r1;
            r0 += a;
            r1 += b;
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < kScanPer; ++k) {
            const int64_t i = base + k * kScanThreads + tid;
            if (i < n) {
                o0[i] = t0[k * kScanThreads + tid];
                if (two) o1[i] = t1[k * kScanThreads + tid];
            }
        }
        carry0 += tot0;
        carry1 += tot1;
        __syncthreads();  // the tile buffers and wave sums are reused
    }
    if (tid == 0) {
        totals[0] = carry0;
        totals[1] = carry1;
    }
}

// ---------------------------------------------------------------- point cloud (R = 8 / 16)
// Candidates from the bit planes: voxel o (weight > thr) and its +x / +y / +z neighbour q (weight >
// thr, block present) with opposite strict signs; each candidate is then confirmed by upstream's own
// test tsdf_o * tsdf_q < 0 on the two tsdf values (a product that underflows to -0 is not a point),
// so the counts are exact.  Per row: {point base in the block, ex | ey << 16, ez}.
template <int R>
__global__ __launch_bounds__(kMcThreads) void k_pt_count(const int32_t* __restrict__ nb, const uint16_t* __restrict__ bits,
                                                         const float2* __restrict__ pool, int32_t* __restrict__ count,
                                                         uint4* __restrict__ rows4) {
    using M = Mc<R, 1>;
    __shared__ uint32_t rowV[M::S2], rowN[M::S2], rowP[M::S2];
    __shared__ int32_t nbrow[27];
    __shared__ int scratch[16];
    const int64_t b = blockIdx.x;
    if (threadIdx.x < 27) nbrow[threadIdx.x] = nb[b * 27 + threadIdx.x];
    __syncthreads();
    mc_stage_bits<M>(nbrow, bits, rowV, rowN, rowP);
    const int r = threadIdx.x;
    uint32_t m[3] = {0, 0, 0};
    if (r < M::R2) {
        const int y = r % R, z = r / R;
        const int q0 = M::q(y, z);
        const uint32_t v0 = rowV[q0], n0 = rowN[q0], p0 = rowP[q0];
        const int qn[3] = {q0, M::q(y + 1, z), M::q(y, z + 1)};
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            // neighbour bits aligned onto the voxel's bit (x + 1): +x is the same row shifted right
            const uint32_t va = a == 0 ? v0 >> 1 : rowV[qn[a]], na = a == 0 ? n0 >> 1 : rowN[qn[a]];
            const uint32_t pa = a == 0 ? p0 >> 1 : rowP[qn[a]];
            uint32_t c = ((v0 & va & ((n0 & pa) | (p0 & na))) >> 1) & M::RMASK;
            uint32_t ok = 0;
            while (c) {  // confirm with the product (few candidates per row)
                const int x = __builtin_ctz(c);
                c &= c - 1;
                const float t_o = mc_tsdf<M>(nbrow, pool, x, y, z);
                const float t_q = mc_tsdf<M>(nbrow, pool, x + (a == 0), y + (a == 1), z + (a == 2));
                if (t_q * t_o < 0) ok |= 1u << x;
            }
            m[a] = ok;
        }
    }
    const int np = __popc(m[0]) + __popc(m[1]) + __popc(m[2]);
    int tot;
    const int base = block_exclusive_scan(np, scratch, tot);
    if (r < M::R2) rows4[b * M::R2 + r] = make_uint4((uint32_t)base, m[0] | (m[1] << 16), m[2], 0u);
    if (threadIdx.x == 0) count[b] = tot;
}

// Points in (block, voxel, axis) order: position voxel_size (X + ratio e), normal interpolated
// between the central-difference normals at o and q (the q-normal scratch carried across the
// voxel's point axes, as upstream's per-voxel ni).
template <int R>
__global__ __launch_bounds__(kMcThreads) void k_pt_emit(const int32_t* __restrict__ nb, const uint64_t* __restrict__ bkeys,
                                                        const float2* __restrict__ pool, float voxel_size,
                                                        const int32_t* __restrict__ count,
                                                        const int32_t* __restrict__ off,
                                                        const uint4* __restrict__ rows4, float* pos, float* nrm,
                                                        int64_t cap) {
    using M = Mc<R, 1>;
    __shared__ uint4 rows[M::R2];
    __shared__ int32_t nbrow[27];
    const int64_t b = blockIdx.x;
    const int npb = count[b];
    if (npb == 0) return;  // block-uniform
    if (off[b] < 0 || (int64_t)off[b] + npb > cap) return;  // past the speculative capacity (or a wrapped int32
                                                           // offset): the host re-runs / fails the call
    const int tid = threadIdx.x;
    if (tid < 27) nbrow[tid] = nb[b * 27 + tid];
    for (int r = tid; r < M::R2; r += blockDim.x) rows[r] = rows4[b * M::R2 + r];
    __syncthreads();
    const int lane = tid & 63;
    const uint32_t pres = (uint32_t)__ballot(lane < 27 && nbrow[lane < 27 ? lane : 0] >= 0);
    int xb, yb, zb;
    unpack_key(bkeys[b], xb, yb, zb);
    const int64_t p0 = off[b];
    for (int i = tid; i < npb; i += blockDim.x) {
        int lo = 0, hi = M::R2 - 1;
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if ((int)rows[mid].x <= i) lo = mid; else hi = mid - 1;
        }
        const uint4 rw = rows[lo];
        const uint32_t ex = rw.y & 0xffffu, ey = rw.y >> 16, ez = rw.z;
        int k = i - (int)rw.x, x;
        row_select<R>(ex, ey, ez, k, x);
        const uint32_t m3 = ((ex >> x) & 1u) | (((ey >> x) & 1u) << 1) | (((ez >> x) & 1u) << 2);
        const int y = lo % R, z = lo / R;
        float t_o, t_i;
        float no[3] = {0.f, 0.f, 0.f}, ni[3] = {0.f, 0.f, 0.f};
        int axis = 0;
        if (pres == kAll27) {  // block-uniform
            uint32_t mm = m3;
            for (int j = 0; j < k; ++j) mm &= mm - 1;
            axis = __builtin_ctz(mm);
            mc_edge_taps<M>(nbrow, pool, x, y, z, axis, t_o, t_i, no, ni);
        } else {
            t_o = mc_tsdf<M>(nbrow, pool, x, y, z);
            mc_normal<M>(nbrow, pool, pres, x, y, z, no);
            uint32_t mm = m3;
            for (int j = 0;; ++j) {
                axis = __builtin_ctz(mm);
                mc_normal<M>(nbrow, pool, pres, x + (axis == 0), y + (axis == 1), z + (axis == 2), ni);
                if (j == k) break;
                mm &= mm - 1;
            }
            t_i = mc_tsdf<M>(nbrow, pool, x + (axis == 0), y + (axis == 1), z + (axis == 2));
        }
        const float ratio = (0 - t_o) / (t_i - t_o);
        const int gx = xb * R + x, gy = yb * R + y, gz = zb * R + z;
        const int64_t id = p0 + i;
        pos[3 * id + 0] = voxel_size * (gx + ratio * (int)(axis == 0));
        pos[3 * id + 1] = voxel_size * (gy + ratio * (int)(axis == 1));
        pos[3 * id + 2] = voxel_size * (gz + ratio * (int)(axis == 2));
        const float nx = (1 - ratio) * no[0] + ratio * ni[0];
        const float ny = (1 - ratio) * no[1] + ratio * ni[1];
        const float nz = (1 - ratio) * no[2] + ratio * ni[2];
        write_normal(nx, ny, nz, nrm + 3 * id);
    }
}

// ---------------------------------------------------------------- point cloud (other R: byte tiles)
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
    uint16_t* bits;  // k_mc_bits planes, 3 R^2 u16 per block (R = 8 / 16)
    void* tmp;
    size_t tmp_bytes;
};

static int ex_scratch(mqr_vbg* v, int64_t n, bool mesh, ExScratch& e) {
    size_t tmp_bytes = 0;
    MQR_CHECK_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, (const int32_t*)nullptr, (int32_t*)nullptr,
                                                   (int)n, v->stream));
    const size_t sz_nb = align256(sizeof(int32_t) * 27 * n), sz_c = align256(sizeof(int32_t) * n);
    // mesh: the byte-tile path's face tables (3 R^2 u32 per block), or the bit-row path's row records
    // (R^2 uint4), sign rows ((R + 2)^2 u32) and per-cube triangle counts (R^2 u64) per block,
    // whichever is larger
    const size_t sz_f = mesh ? align256(std::max(sizeof(uint32_t) * 3 * v->R * v->R,
                                                 sizeof(uint32_t) * (6 * v->R * v->R + (v->R + 2) * (v->R + 2))) *
                                        n)
                             : 0;
    const size_t sz_b = align256(sizeof(uint16_t) * 3 * v->R * v->R * n);
    tmp_bytes = std::max<size_t>(tmp_bytes, 2 * sizeof(int64_t));
    const size_t need = sz_nb + 4 * sz_c + sz_f + sz_b + align256(tmp_bytes);
    if (v->ex_scratch_bytes < need) {
        MQR_CHECK_HIP(hipStreamSynchronize(v->stream));
        if (v->ex_scratch) MQR_CHECK_HIP(hipFree(v->ex_scratch));
        v->ex_scratch = nullptr;
        v->ex_scratch_bytes = 0;
        const size_t cap = need + need / 4;
        MQR_CHECK_HIP(hipMalloc(&v->ex_scratch, cap));
        v->ex_scratch_bytes = cap;
    }
    // fine-grained (coherent) pinned memory: k_scan_counts writes the totals straight into it (ex_mode bit 2)
    if (!v->h_ex) MQR_CHECK_HIP(hipHostMalloc(&v->h_ex, 4 * sizeof(int64_t), hipHostMallocCoherent));
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
    e.bits = reinterpret_cast<uint16_t*>(p);
    p += sz_b;
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

static std::mutex g_geom_mu;
static std::vector<std::tuple<int, void*, size_t>> g_geom_cache;  // (device, block, capacity)
constexpr size_t kGeomCacheBlocks = 4;

void* geom_block_alloc(int device, size_t bytes, size_t* cap) {
    {
        std::lock_guard<std::mutex> lk(g_geom_mu);
        int best = -1;
        for (size_t i = 0; i < g_geom_cache.size(); ++i) {
            const auto& e = g_geom_cache[i];
            if (std::get<0>(e) == device && std::get<2>(e) >= bytes &&
                (best < 0 || std::get<2>(e) < std::get<2>(g_geom_cache[best])))
                best = (int)i;
        }
        if (best >= 0) {
            void* p = std::get<1>(g_geom_cache[best]);
            *cap = std::get<2>(g_geom_cache[best]);
            g_geom_cache.erase(g_geom_cache.begin() + best);
            return p;
        }
    }
    const size_t want = (bytes + (size_t(1) << 20) - 1) & ~((size_t(1) << 20) - 1);
    void* p = nullptr;
    if (hipMalloc(&p, want) != hipSuccess) return nullptr;
    *cap = want;
    return p;
}

void geom_block_release(int device, void* p, size_t cap) {
    if (!p) return;
    {
        std::lock_guard<std::mutex> lk(g_geom_mu);
        if (cap && g_geom_cache.size() < kGeomCacheBlocks) {
            g_geom_cache.emplace_back(device, p, cap);
            return;
        }
    }
    (void)hipFree(p);
}

// One allocation for positions, normals and triangles, recycled across results (geom_block_alloc).
static int alloc_geom(mqr_geom* g, int64_t nv, int64_t nt) {
    const size_t sv = align256(sizeof(float) * 3 * std::max<int64_t>(nv, 1));
    const size_t st = align256(sizeof(int32_t) * 3 * std::max<int64_t>(nt, 1));
    g->blk = geom_block_alloc(g->device, 2 * sv + st, &g->blk_cap);
    MQR_REQUIRE(g->blk, "geometry: device allocation failed");
    char* p = static_cast<char*>(g->blk);
    g->pos = reinterpret_cast<float*>(p);
    g->nrm = reinterpret_cast<float*>(p + sv);
    g->tri = reinterpret_cast<int32_t*>(p + 2 * sv);
    return 0;
}

static int build_nb(mqr_vbg* v, int32_t* nb) {
    const int64_t n = v->pool_count;
    hipLaunchKernelGGL(k_nb, dim3((unsigned)((n * 27 + 255) / 256)), dim3(256), 0, v->stream, v->bkeys, n, v->tab, nb);
    MQR_CHECK_HIP(hipGetLastError());
    return 0;
}

// Speculative output capacity from the volume's previous extraction (0 = none yet: the host waits
// for the totals before emitting).  The margin absorbs the growth between two extractions of a
// volume that is still being integrated.
static int64_t spec_cap(int64_t hint) { return hint > 0 ? hint + hint / 4 + 4096 : 0; }

// Extraction configuration: bit 0 = NIB (k_mc_count), bit 1 = MAP (k_mc_emit), bit 2 = the scan writes
// the totals straight into pinned host memory (without: a D2H copy enqueued between the scan and the
// emission pass, whose latency the emission waited behind); the A/B library takes it from
// mqr_vbg_set_extract_mode (below; tools/ab_extract.py; a negative mode = the library default).  (Also measured in round 4
// and removed, DESIGN.md §4.2: the emission over a compacted list of the blocks with output, by one
// workgroup per listed block or by a grid of 8 workgroups per CU walking the list; the block's tsdf
// staged in LDS for its interior vertices' taps; XCD bands of the pool in the count and emission
// passes; the triangles' neighbour row records prefetched into LDS during the vertex loop -- all
// neutral or slower.)
[[maybe_unused]] constexpr int kExMode = 7;  // NIB + MAP + direct totals (tools/ab_extract.py)
static int ex_mode(const mqr_vbg* v) {
#if MQR_AB
    return v->ex_mode < 0 ? kExMode : v->ex_mode;
#else
    (void)v;
    return kExMode;
#endif
}

template <int RT, bool NIB, bool MAP, class... A>
static void launch_mc_emit_t(const mqr_vbg* v, int64_t n, A... args) {
#if MQR_AB  // MQR_EMIT_DIAG=1: vertices only, 2: triangles only (timing diagnostics)
    static const int diag = getenv("MQR_EMIT_DIAG") ? atoi(getenv("MQR_EMIT_DIAG")) : 0;
#else
    constexpr int diag = 0;
#endif
    hipLaunchKernelGGL((k_mc_emit<RT, NIB, MAP>), dim3((unsigned)n), dim3(kMcThreads), 0, v->stream, args..., diag);
}

template <int RT, class... A>
static void launch_mc_emit(const mqr_vbg* v, int64_t n, A... args) {
    switch (ex_mode(v) & 3) {
        case 1: launch_mc_emit_t<RT, true, false>(v, n, args...); break;
        case 2: launch_mc_emit_t<RT, false, true>(v, n, args...); break;
        case 3: launch_mc_emit_t<RT, true, true>(v, n, args...); break;
        default: launch_mc_emit_t<RT, false, false>(v, n, args...); break;
    }
}

template <int RT>
static int mesh_passes(mqr_vbg* v, float thr, const ExScratch& e, mqr_geom* g, int64_t tri_blocks) {
    const int64_t n = v->pool_count;
    constexpr int RR = RT > 0 ? RT : 16;
    uint4* rows4 = reinterpret_cast<uint4*>(e.faces);
    uint32_t* rowNt = reinterpret_cast<uint32_t*>(rows4 + n * RR * RR);
    uint64_t* rowsT = reinterpret_cast<uint64_t*>(rowNt + n * (RR + 2) * (RR + 2));  // 8-byte aligned: (R + 2)^2 even
    int64_t nv = 0, nt = 0;
    if constexpr (RT > 0) {
        int64_t* tot = reinterpret_cast<int64_t*>(e.tmp);
        hipLaunchKernelGGL(k_mc_bits<RT>, dim3((unsigned)n), dim3(kMcThreads), 0, v->stream, v->pool, thr, e.bits,
                           v->bkeys, v->tab, e.nb);
        if (ex_mode(v) & 1)
            hipLaunchKernelGGL((k_mc_count<RT, true>), dim3((unsigned)n), dim3(kMcThreads), 0, v->stream, e.nb, e.bits,
                               tri_blocks, e.c0, e.c1, rows4, rowNt, rowsT);
        else
            hipLaunchKernelGGL((k_mc_count<RT, false>), dim3((unsigned)n), dim3(kMcThreads), 0, v->stream, e.nb, e.bits,
                               tri_blocks, e.c0, e.c1, rows4, rowNt, rowsT);
        const bool direct = ex_mode(v) & 4;
        hipLaunchKernelGGL(k_scan_counts, dim3(1), dim3(kScanThreads), 0, v->stream, e.c0, e.c1, n, e.o0, e.o1,
                           direct ? v->h_ex : tot);
        // With a previous extraction's counts, emit into buffers of that size (+ margin) without
        // waiting for this one's totals; blocks past the capacity write nothing and the pass is re-run
        // into exact buffers if the totals exceed it.  Without, wait for the totals first.
        int64_t cv = spec_cap(v->ex_hint[0]), ct = spec_cap(v->ex_hint[1]);
        const bool spec = cv > 0 && ct > 0;
        if (spec && alloc_geom(g, cv, ct)) return 1;
        MQR_CHECK_HIP(hipGetLastError());
        if (!direct) MQR_CHECK_HIP(hipMemcpyAsync(v->h_ex, tot, 2 * sizeof(int64_t), hipMemcpyDeviceToHost, v->stream));
        bool emitted = false;
        if (spec) {
            launch_mc_emit<RT>(v, n, (const int32_t*)e.nb, (const uint64_t*)v->bkeys, (const float2*)v->pool,
                               v->voxel_size, (const int32_t*)e.c0, (const int32_t*)e.c1, (const int32_t*)e.o0,
                               (const int32_t*)e.o1, (const uint4*)rows4, (const uint32_t*)rowNt, g->pos, g->nrm,
                               g->tri, cv, ct, (const uint64_t*)rowsT);
            MQR_CHECK_HIP(hipGetLastError());
            emitted = true;
        }
        MQR_CHECK_HIP(hipStreamSynchronize(v->stream));
        nv = v->h_ex[0];
        nt = v->h_ex[1];
        MQR_REQUIRE(nv < (int64_t)1 << 31 && nt < (int64_t)1 << 31, "mesh exceeds int32 vertex / triangle ids");
        v->ex_hint[0] = nv;
        v->ex_hint[1] = nt;
        g->nv = nv;
        g->nt = nt;
        if (emitted && nv <= cv && nt <= ct) return 0;
        if (g->blk) {
            geom_block_release(g->device, g->blk, g->blk_cap);
            g->blk = nullptr;
        }
        if (alloc_geom(g, nv, nt)) return 1;
        launch_mc_emit<RT>(v, n, (const int32_t*)e.nb, (const uint64_t*)v->bkeys, (const float2*)v->pool, v->voxel_size,
                           (const int32_t*)e.c0, (const int32_t*)e.c1, (const int32_t*)e.o0, (const int32_t*)e.o1,
                           (const uint4*)rows4, (const uint32_t*)rowNt, g->pos, g->nrm, g->tri, nv, nt,
                           (const uint64_t*)rowsT);
    } else {
        if (build_nb(v, e.nb)) return 1;
        hipLaunchKernelGGL(k_mesh_count<RT>, dim3((unsigned)n), dim3(kThreads), 0, v->stream, e.nb, n, v->pool, v->R,
                           thr, e.c0, e.c1, e.faces);
        MQR_CHECK_HIP(hipGetLastError());
        if (scan_totals(v, e, n, 2, &nv, &nt)) return 1;
        MQR_REQUIRE(nv < (int64_t)1 << 31 && nt < (int64_t)1 << 31, "mesh exceeds int32 vertex / triangle ids");
        g->nv = nv;
        g->nt = nt;
        if (alloc_geom(g, nv, nt)) return 1;
        hipLaunchKernelGGL(k_mesh_emit<RT>, dim3((unsigned)n), dim3(kThreads), 0, v->stream, e.nb, n, v->bkeys,
                           v->pool, v->R, v->voxel_size, thr, e.c0, e.c1, e.o0, e.o1, e.faces, g->pos, g->nrm, g->tri);
    }
    MQR_CHECK_HIP(hipGetLastError());
    MQR_CHECK_HIP(hipStreamSynchronize(v->stream));
    return 0;
}

template <int RT>
static int point_passes(mqr_vbg* v, float thr, const ExScratch& e, mqr_geom* g) {
    const int64_t n = v->pool_count;
    int64_t np = 0;
    if constexpr (RT > 0) {
        uint4* rows4 = reinterpret_cast<uint4*>(e.faces);
        int64_t* tot = reinterpret_cast<int64_t*>(e.tmp);
        hipLaunchKernelGGL(k_mc_bits<RT>, dim3((unsigned)n), dim3(kMcThreads), 0, v->stream, v->pool, thr, e.bits,
                           v->bkeys, v->tab, e.nb);
        hipLaunchKernelGGL(k_pt_count<RT>, dim3((unsigned)n), dim3(kMcThreads), 0, v->stream, e.nb, e.bits, v->pool,
                           e.c0, rows4);
        const bool direct = ex_mode(v) & 4;
        hipLaunchKernelGGL(k_scan_counts, dim3(1), dim3(kScanThreads), 0, v->stream, e.c0, (const int32_t*)nullptr, n,
                           e.o0, (int32_t*)nullptr, direct ? v->h_ex : tot);
        MQR_CHECK_HIP(hipGetLastError());
        if (!direct) MQR_CHECK_HIP(hipMemcpyAsync(v->h_ex, tot, sizeof(int64_t), hipMemcpyDeviceToHost, v->stream));
        const int64_t cp = spec_cap(v->ex_hint[2]);  // speculative capacity, as in mesh_passes
        if (cp > 0) {
            if (alloc_geom(g, cp, 0)) return 1;
            hipLaunchKernelGGL(k_pt_emit<RT>, dim3((unsigned)n), dim3(kMcThreads), 0, v->stream, e.nb, v->bkeys,
                               v->pool, v->voxel_size, e.c0, e.o0, reinterpret_cast<const uint4*>(e.faces), g->pos,
                               g->nrm, cp);
            MQR_CHECK_HIP(hipGetLastError());
        }
        MQR_CHECK_HIP(hipStreamSynchronize(v->stream));
        np = v->h_ex[0];
        MQR_REQUIRE(np < (int64_t)1 << 31, "point cloud exceeds int32 offsets");
        v->ex_hint[2] = np;
        g->nv = np;
        if (cp > 0 && np <= cp) return 0;
        if (g->blk) {
            geom_block_release(g->device, g->blk, g->blk_cap);
            g->blk = nullptr;
        }
        if (alloc_geom(g, np, 0)) return 1;
        hipLaunchKernelGGL(k_pt_emit<RT>, dim3((unsigned)n), dim3(kMcThreads), 0, v->stream, e.nb, v->bkeys, v->pool,
                           v->voxel_size, e.c0, e.o0, reinterpret_cast<const uint4*>(e.faces), g->pos, g->nrm, np);
    } else {
        if (build_nb(v, e.nb)) return 1;
        hipLaunchKernelGGL(k_points<RT>, dim3((unsigned)n), dim3(kThreads), 0, v->stream, e.nb, n, v->bkeys, v->pool,
                           v->R, v->voxel_size, thr, e.c0, (const int32_t*)nullptr, (float*)nullptr, (float*)nullptr);
        MQR_CHECK_HIP(hipGetLastError());
        if (scan_totals(v, e, n, 1, &np, nullptr)) return 1;
        g->nv = np;
        if (alloc_geom(g, np, 0)) return 1;
        hipLaunchKernelGGL(k_points<RT>, dim3((unsigned)n), dim3(kThreads), 0, v->stream, e.nb, n, v->bkeys, v->pool,
                           v->R, v->voxel_size, thr, e.c0, e.o0, g->pos, g->nrm);
    }
    MQR_CHECK_HIP(hipGetLastError());
    MQR_CHECK_HIP(hipStreamSynchronize(v->stream));
    return 0;
}

}  // namespace mqr

using namespace mqr;

extern "C" {

int mqr_extract_mesh(mqr_vbg* v, float thr, mqr_geom** out) { return mqr_extract_mesh_owned(v, thr, -1, out); }

#if MQR_AB
// A/B library only: the extraction configuration (kExMode bits) for tools/ab_extract.py.
int mqr_vbg_set_extract_mode(mqr_vbg* v, int mode) {
    MQR_REQUIRE(v && mode < 8, "bad extraction mode");
    v->ex_mode = mode;
    return 0;
}
#endif

int mqr_extract_mesh_owned(mqr_vbg* v, float thr, int64_t n_owned, mqr_geom** out) {
    MQR_REQUIRE(v && out, "null argument");
    MQR_REQUIRE(v->R <= kMaxR, "extract_triangle_mesh supports block_resolution <= 16");
    MQR_REQUIRE(n_owned < 0 || v->R == 16 || v->R == 8, "owned-block extraction supports block_resolution 8 / 16");
    const int64_t tri_blocks = n_owned < 0 ? INT64_MAX : n_owned;
    MQR_CHECK_HIP(hipSetDevice(v->device));
    if (order_after_integrate(v)) return 1;  // an integrate may still be running on the second stream
    const int64_t n = v->pool_count;
    mqr_geom* g = new mqr_geom();
    g->device = v->device;
    *out = nullptr;
    int rc = 0;
    if (n > 0) {
        ExScratch e{};
        rc = ex_scratch(v, n, true, e);
        if (!rc) rc = v->R == 16 ? mesh_passes<16>(v, thr, e, g, tri_blocks)
                      : v->R == 8 ? mesh_passes<8>(v, thr, e, g, tri_blocks)
                                  : mesh_passes<0>(v, thr, e, g, tri_blocks);
    }
    if (rc) {  // release whatever the failed passes allocated; the caller gets no handle
        const std::string msg = get_error();
        mqr_geom_free(g);
        set_error(msg);
        return rc;
    }
    *out = g;
    return 0;
}

int mqr_extract_points(mqr_vbg* v, float thr, mqr_geom** out) {
    MQR_REQUIRE(v && out, "null argument");
    MQR_REQUIRE(v->R <= kMaxR, "extract_point_cloud supports block_resolution <= 16");
    MQR_CHECK_HIP(hipSetDevice(v->device));
    if (order_after_integrate(v)) return 1;
    const int64_t n = v->pool_count;
    mqr_geom* g = new mqr_geom();
    g->device = v->device;
    *out = nullptr;
    int rc = 0;
    if (n > 0) {
        ExScratch e{};
        rc = ex_scratch(v, n, true, e);  // the row records use the mesh path's slot
        if (!rc) rc = v->R == 16 ? point_passes<16>(v, thr, e, g) : v->R == 8 ? point_passes<8>(v, thr, e, g)
                                                                           : point_passes<0>(v, thr, e, g);
    }
    if (rc) {
        const std::string msg = get_error();
        mqr_geom_free(g);
        set_error(msg);
        return rc;
    }
    *out = g;
    return 0;
}

int mqr_geom_counts(mqr_geom* g, int64_t* nv, int64_t* nt) {
    MQR_REQUIRE(g, "null geometry");
    if (nv) *nv = g->nv;
    if (nt) *nt = g->nt;
    return 0;
}

}  // extern "C"

namespace mqr {
// Device -> pageable host copies of large results (mqr_geom_copy, mqr_memcpy).  hipMemcpy into pageable
// memory stages through the runtime's pinned buffers on the calling thread: ~10 GB/s for the 1 GB C5 mesh
// (BENCH_r04 c5.extract_ms 102.9 ms).  Here a copy kernel moves the range chunk by chunk into a ring of
// pinned slots (GPU stores over the fabric: 54.7 GB/s into pinned memory, SDMA 57.1, tools/d2h_modes.hip)
// on a stream the process already runs, and kD2HThreads host threads copy each slot out as its event
// completes (first-touching the destination pages in parallel).  Round 5's first version gave every host
// thread its own stream and DMA: the same ~41 GB/s once set up, but its set-up cost the process's first
// large copy 46.6 ms (first 48 MB copy, vs 1.6 ms for the second, tools/d2h_probe.py) -- four stream
// creations 50 ms and the copy engine's first use 16-19 ms on an MI355X box (tools/d2h_setup_probe.hip,
// profiles/r05_d2h_setup_probe.json).  The ring (one pinned allocation per device) is kept and the calls
// are serialised by a mutex: one large copy at a time per process.
constexpr int kD2HThreads = 8;  // 1 GiB into a fresh array: 44.4 GB/s with 4, 51.1 with 8 (profiles/r05_d2h_probe.jsonl)
constexpr int kD2HSlots = 8;
constexpr size_t kD2HChunk = size_t(8) << 20;
constexpr int kD2HDevices = 64;
struct D2HRing {
    char* buf = nullptr;
    hipEvent_t ev[kD2HSlots] = {};
};
static std::mutex g_d2h_mu;
static D2HRing g_d2h[kD2HDevices];

__global__ __launch_bounds__(256) void k_copy_out16(uint4* __restrict__ dst, const uint4* __restrict__ src, size_t n16) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) dst[i] = src[i];
}

__global__ __launch_bounds__(256) void k_copy_out1(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src, size_t n) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) dst[i] = src[i];
}

hipStream_t copy_stream(int device) {
    if (caller_stream()) {
        hipDevice_t sd = -1;
        const bool same = hipStreamGetDevice(caller_stream(), &sd) == hipSuccess && sd == device;
        (void)hipGetLastError();
        if (same) return caller_stream();
    }
    return nullptr;
}

static void launch_copy(char* to, const char* from, size_t len, hipStream_t s) {
    const bool aligned = ((reinterpret_cast<uintptr_t>(to) | reinterpret_cast<uintptr_t>(from)) & 15) == 0;
    const size_t n16 = aligned ? len / 16 : 0, tail = len - 16 * n16;
    if (n16) k_copy_out16<<<1024, 256, 0, s>>>(reinterpret_cast<uint4*>(to), reinterpret_cast<const uint4*>(from), n16);
    if (tail)
        k_copy_out1<<<(unsigned)std::min<size_t>(1024, (tail + 255) / 256), 256, 0, s>>>(
            reinterpret_cast<uint8_t*>(to) + 16 * n16, reinterpret_cast<const uint8_t*>(from) + 16 * n16, tail);
}

// One ring transfer: the GPU fills slot k % S with chunk k, host thread k % T copies it out once its
// event completes; this thread queues the GPU copies in chunk order, each into a slot whose previous
// chunk has been copied out.
static int ring_copy(int device, char* dst, const char* src, size_t bytes, hipStream_t s) {
    MQR_REQUIRE(device >= 0 && device < kD2HDevices, "device index out of range");
    std::lock_guard<std::mutex> lk(g_d2h_mu);
    D2HRing& r = g_d2h[device];
    if (!r.buf) {
        MQR_CHECK_HIP(hipHostMalloc(reinterpret_cast<void**>(&r.buf), kD2HSlots * kD2HChunk, hipHostMallocDefault));
        for (auto& e : r.ev) MQR_CHECK_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    const size_t nchunks = (bytes + kD2HChunk - 1) / kD2HChunk;
    // MQR_D2H_THREADS (1..8): another thread count, for tools/d2h_probe.py
    static const int env_threads =
        getenv("MQR_D2H_THREADS") ? std::max(1, std::min(8, atoi(getenv("MQR_D2H_THREADS")))) : kD2HThreads;
    const int T = (int)std::min<size_t>(env_threads, nchunks);
    auto len_of = [&](size_t k) { return std::min(kD2HChunk, bytes - k * kD2HChunk); };
    std::atomic<int64_t> issued{0};            // chunks whose GPU copy and event are queued
    std::atomic<int64_t> host_done[kD2HSlots];  // the last chunk copied out of each slot
    for (auto& d : host_done) d.store(-1);
    std::atomic<int> failed{0};
    std::vector<std::string> errs(T + 1);
    auto host_side = [&](int t) {
        for (size_t k = (size_t)t; k < nchunks; k += (size_t)T) {
            while (issued.load(std::memory_order_acquire) <= (int64_t)k && !failed.load()) std::this_thread::yield();
            if (failed.load()) return;
            const int slot = (int)(k % kD2HSlots);
            hipError_t e = hipEventSynchronize(r.ev[slot]);
            if (e != hipSuccess) {
                errs[t] = std::string("host copy: hipEventSynchronize: ") + hipGetErrorString(e);
                failed.store(1);
                return;
            }
            std::memcpy(dst + k * kD2HChunk, r.buf + slot * kD2HChunk, len_of(k));
            host_done[slot].store((int64_t)k, std::memory_order_release);
        }
    };
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t) th.emplace_back(host_side, t);
    for (size_t k = 0; k < nchunks && !failed.load(); ++k) {
        const int slot = (int)(k % kD2HSlots);
        if (k >= (size_t)kD2HSlots)
            while (host_done[slot].load(std::memory_order_acquire) != (int64_t)(k - kD2HSlots) && !failed.load())
                std::this_thread::yield();
        if (failed.load()) break;
        launch_copy(r.buf + slot * kD2HChunk, src + k * kD2HChunk, len_of(k), s);
        hipError_t e = hipGetLastError();
        if (e == hipSuccess) e = hipEventRecord(r.ev[slot], s);
        if (e != hipSuccess) {
            errs[T] = std::string("host copy: chunk copy launch: ") + hipGetErrorString(e);
            failed.store(1);
            break;
        }
        issued.store((int64_t)k + 1, std::memory_order_release);
    }
    for (auto& x : th) x.join();
    if (failed.load()) {
        (void)hipStreamSynchronize(s);  // no slot write left in flight for the next call
        for (auto& m : errs)
            if (!m.empty()) {
                set_error(m);
                return 1;
            }
    }
    return 0;
}

int d2h_parallel(int device, void* dst, const void* src, size_t bytes) {
    return copy_to_host(device, dst, src, bytes, copy_stream(device));
}

// page-locked host memory (hipHostMalloc / hipHostRegister, e.g. torch's pin_memory()): the DMA engine
// reads or writes it directly, no staging
static bool host_pinned(const void* p) {
    hipPointerAttribute_t a{};
    const bool pinned = hipPointerGetAttributes(&a, p) == hipSuccess && a.type == hipMemoryTypeHost;
    (void)hipGetLastError();
    return pinned;
}

int copy_to_host(int device, void* dst, const void* src, size_t bytes, hipStream_t s) {
    if (bytes >= kD2HParallelMin && !host_pinned(dst)) return ring_copy(device, static_cast<char*>(dst), static_cast<const char*>(src), bytes, s);
    if (bytes) {
        MQR_CHECK_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, s));
        MQR_CHECK_HIP(hipStreamSynchronize(s));
    }
    return 0;
}

// uploads: HIP's own pageable path already runs at the link's rate from present pages (1 GiB: 55.8 GB/s,
// against 44.1 through a ring like the one above, profiles/r05_d2h_probe.jsonl)
int copy_to_device(int device, void* dst, const void* src, size_t bytes, hipStream_t s) {
    (void)device;
    if (bytes) {
        MQR_CHECK_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s));
        MQR_CHECK_HIP(hipStreamSynchronize(s));
    }
    return 0;
}

static int geom_copy_one(int device, void* dst, const void* src, size_t bytes, hipMemcpyKind k) {
    if (k == hipMemcpyDeviceToHost && bytes >= kD2HParallelMin) return d2h_parallel(device, dst, src, bytes);
    MQR_CHECK_HIP(hipMemcpy(dst, src, bytes, k));
    return 0;
}
}  // namespace mqr

extern "C" {

int mqr_geom_copy(mqr_geom* g, float* positions, float* normals, int32_t* triangles, int loc) {
    MQR_REQUIRE(g, "null geometry");
    MQR_CHECK_HIP(hipSetDevice(g->device));
    const hipMemcpyKind k = loc == MQR_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
    // hipMemcpy orders after the null stream only: the caller's stream may still use the buffers
    if (loc == MQR_DEVICE && caller_stream()) MQR_CHECK_HIP(hipStreamSynchronize(caller_stream()));
    if (positions && g->nv && geom_copy_one(g->device, positions, g->pos, sizeof(float) * 3 * g->nv, k)) return 1;
    if (normals && g->nv && geom_copy_one(g->device, normals, g->nrm, sizeof(float) * 3 * g->nv, k)) return 1;
    if (triangles && g->nt && geom_copy_one(g->device, triangles, g->tri, sizeof(int32_t) * 3 * g->nt, k)) return 1;
    return 0;
}

int mqr_geom_device_ptrs(mqr_geom* g, void** positions, void** normals, void** triangles) {
    MQR_REQUIRE(g, "null geometry");
    if (positions) *positions = g->nv ? g->pos : nullptr;
    if (normals) *normals = g->nv ? g->nrm : nullptr;
    if (triangles) *triangles = g->nt ? g->tri : nullptr;
    return 0;
}

int mqr_geom_free(mqr_geom* g) {
    if (!g) return 0;
    (void)hipSetDevice(g->device);
    if (g->blk) {
        // the block may still be read by work queued on a stream (a device-side copy): drain first
        (void)hipDeviceSynchronize();
        geom_block_release(g->device, g->blk, g->blk_cap);
    } else {
        if (g->pos) (void)hipFree(g->pos);
        if (g->nrm) (void)hipFree(g->nrm);
        if (g->tri) (void)hipFree(g->tri);
    }
    delete g;
    return 0;
}

}  // extern "C"

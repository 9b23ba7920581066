// vbg.hip -- the HBM-resident voxel-block TSDF volume: block hash, touch, integrate,
// export/import and the multi-GPU pack/unpack.  Replaces Open3D 0.19's VoxelBlockGrid
// (reference call sites: scripts/processing/reconstruction/utils/o3d_utils.py:170-229).
//
// Data layout in HBM (one volume):
//   pool   [pool_cap][R^3] float2 (tsdf, weight), voxel [z][y][x] inside a block -> 32 KiB/block at R=16
//   bkeys  [pool_cap] packed block key of each buffer (for extraction / export)
//   table  keys u64 / vals i32 / mask u32, open addressing, capacity >= 2x live keys
//   list   slots touched by the current batch (appended once per batch, on first touch)
//
// Per batch of <= 32 frames: k_touch (one thread per stride-4 pixel per frame, 4 ray samples,
// hash insert, per-slot frame bitmask) -> host reads 8 counters (pool growth) -> k_integrate
// (one workgroup per touched block, every voxel applies that block's frames in frame order =
// bit-identical to sequential per-frame integration).
#include <algorithm>
#include <cmath>
#include <cstring>

#include "mqr_common.hpp"

namespace mqr {

static thread_local std::string g_err;
void set_error(const std::string& msg) { g_err = msg; }
const char* get_error() { return g_err.c_str(); }

constexpr int kMaxBatch = 32;
constexpr int kFrameCounterBase = 8;  // per-frame raw touch counts live at counters[8 + f]
constexpr int kCountersTotal = kFrameCounterBase + kMaxBatch;

void make_frame_params(const double* K, const double* T, FrameParams* fp) {
    fp->fx = (float)K[0];
    fp->fy = (float)K[4];
    fp->cx = (float)K[2];
    fp->cy = (float)K[5];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 4; ++j) fp->ext[i * 4 + j] = (float)T[i * 4 + j];
    // Rigid inverse in float64 (upstream t::geometry::InverseTransformation), then float32.
    double P[12];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) P[i * 4 + j] = T[j * 4 + i];
    for (int i = 0; i < 3; ++i)
        P[i * 4 + 3] = -(P[i * 4 + 0] * T[0 * 4 + 3] + P[i * 4 + 1] * T[1 * 4 + 3] + P[i * 4 + 2] * T[2 * 4 + 3]);
    for (int k = 0; k < 12; ++k) fp->pose[k] = (float)P[k];
}

// ------------------------------------------------------------------ device helpers
__device__ inline int64_t table_find(const Table t, uint64_t k) {
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

// Insert-or-find.  A CAS winner allocates a pool buffer when `alloc`.
__device__ inline int64_t table_insert(Table t, uint64_t k, bool alloc, int* counters, int64_t pool_cap,
                                       uint64_t* bkeys) {
    const uint64_t m = (uint64_t)t.cap - 1;
    uint64_t h = mix64(k) & m;
    for (int64_t p = 0; p < t.cap; ++p) {
        const uint64_t cur = t.keys[h];
        if (cur == k) return (int64_t)h;
        if (cur == kEmpty) {
            const uint64_t old = atomicCAS((unsigned long long*)&t.keys[h], (unsigned long long)kEmpty,
                                           (unsigned long long)k);
            if (old == kEmpty) {
                if (alloc) {
                    const int b = atomicAdd(&counters[kPoolCount], 1);
                    if (b < pool_cap) {
                        t.vals[h] = b;
                        bkeys[b] = k;
                    } else {
                        t.vals[h] = -2;
                        atomicOr(&counters[kOverflow], 1);
                    }
                }
                return (int64_t)h;
            }
            if (old == k) return (int64_t)h;
        }
        h = (h + 1) & m;
    }
    atomicOr(&counters[kOverflow], 2);
    return -1;
}

__device__ inline void mark_slot(Table t, int64_t slot, int f, int* counters, int32_t* list, int64_t list_cap) {
    const uint32_t bit = 1u << f;
    const uint32_t old = atomicOr(&t.mask[slot], bit);
    if (!(old & bit)) atomicAdd(&counters[kFrameBlocks], 1);
    if (old == 0) {
        const int pos = atomicAdd(&counters[kListCount], 1);
        if (pos < list_cap)
            list[pos] = (int32_t)slot;
        else
            atomicOr(&counters[kOverflow], 4);
    }
}

__device__ inline uint64_t shfl_up_u64(uint64_t v, int d) {
    const int lo = __shfl_up((int)(uint32_t)v, d, 64);
    const int hi = __shfl_up((int)(uint32_t)(v >> 32), d, 64);
    return ((uint64_t)(uint32_t)hi << 32) | (uint64_t)(uint32_t)lo;
}

// ------------------------------------------------------------------ kernels
// compute_unique_block_coordinates for a batch: blockIdx.y = batch frame (bit), one thread per
// stride-4 pixel, 4 samples over [max(d - trunc, 0), min(d + trunc, depth_max)] (Appendix A.2).
__global__ __launch_bounds__(256) void k_touch(const float* __restrict__ depths, int64_t HW, int H, int W,
                                               const FrameParams* __restrict__ fps,
                                               const int64_t* __restrict__ depth_frame, float depth_scale,
                                               float depth_max, float sdf_trunc, float block_size, Table t,
                                               int alloc, int* counters, int64_t pool_cap, uint64_t* bkeys,
                                               int32_t* list, int64_t list_cap) {
    const int f = blockIdx.y;
    const FrameParams& fp = fps[f];
    const int cols = W / 4, rows = H / 4, n = rows * cols;
    const int w = blockIdx.x * blockDim.x + threadIdx.x;
    const int lane = threadIdx.x & 63;
    uint64_t key[4] = {kEmpty, kEmpty, kEmpty, kEmpty};
    if (w < n) {
        const int y = (w / cols) * 4, x = (w % cols) * 4;
        const float d = depths[depth_frame[f] * HW + (int64_t)y * W + x] / depth_scale;
        if (d > 0 && d < depth_max) {
            const float xc = ((float)x - fp.cx) * 1.0f / fp.fx;
            const float yc = ((float)y - fp.cy) * 1.0f / fp.fy;
            const float zc = 1.0f;
            const float xg = xc * fp.pose[0] + yc * fp.pose[1] + zc * fp.pose[2] + fp.pose[3];
            const float yg = xc * fp.pose[4] + yc * fp.pose[5] + zc * fp.pose[6] + fp.pose[7];
            const float zg = xc * fp.pose[8] + yc * fp.pose[9] + zc * fp.pose[10] + fp.pose[11];
            const float xo = fp.pose[3], yo = fp.pose[7], zo = fp.pose[11];
            const float xd = xg - xo, yd = yg - yo, zd = zg - zo;
            const float t_min = fmaxf(d - sdf_trunc, 0.0f);
            const float t_max = fminf(d + sdf_trunc, depth_max);
            const float t_step = (t_max - t_min) / 3;
            float tt = t_min;
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const int xb = (int)floorf((xo + tt * xd) / block_size);
                const int yb = (int)floorf((yo + tt * yd) / block_size);
                const int zb = (int)floorf((zo + tt * zd) / block_size);
                if (key_in_range(xb, yb, zb))
                    key[s] = pack_key(xb, yb, zb);
                else
                    atomicOr(&counters[kOverflow], 8);
                tt += t_step;
            }
            atomicAdd(&counters[kFrameCounterBase + f], 4);
        }
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const uint64_t k = key[s];
        const uint64_t up = shfl_up_u64(k, 1);
        bool dup = (lane > 0 && up == k);
        if (s > 0 && key[s - 1] == k) dup = true;
        if (k != kEmpty && !dup) {
            const int64_t slot = table_insert(t, k, alloc != 0, counters, pool_cap, bkeys);
            if (slot >= 0) mark_slot(t, slot, f, counters, list, list_cap);
        }
    }
}

// Activate explicit keys (vbg.integrate(block_coords, ...)); marks frame bit 0.
__global__ void k_activate(const int32_t* __restrict__ keys, int64_t n, Table t, int* counters, int64_t pool_cap,
                           uint64_t* bkeys, int32_t* list, int64_t list_cap, int mark) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int x = keys[3 * i], y = keys[3 * i + 1], z = keys[3 * i + 2];
    if (!key_in_range(x, y, z)) {
        atomicOr(&counters[kOverflow], 8);
        return;
    }
    const int64_t slot = table_insert(t, pack_key(x, y, z), true, counters, pool_cap, bkeys);
    if (slot >= 0 && mark) mark_slot(t, slot, 0, counters, list, list_cap);
}

// Projective TSDF update of every voxel of every listed block, frames applied in bit order.
// Arithmetic = Open3D 0.19 Integrate kernel (Appendix A.3), float32, no contraction.
__global__ __launch_bounds__(256) void k_integrate(const int32_t* __restrict__ list, const int* __restrict__ counters,
                                                   int64_t list_cap, Table t, float2* __restrict__ pool, int R,
                                                   float voxel_size, const float* __restrict__ depths, int64_t HW,
                                                   int H, int W, const FrameParams* __restrict__ fps,
                                                   const int64_t* __restrict__ depth_frame, float depth_scale,
                                                   float depth_max, float sdf_trunc) {
    const int64_t n = min((int64_t)counters[kListCount], list_cap);
    const int R3 = R * R * R;
    const float hm1 = (float)H - 1.0f, wm1 = (float)W - 1.0f;
    for (int64_t i = blockIdx.x; i < n; i += gridDim.x) {
        const int32_t slot = list[i];
        const int buf = t.vals[slot];
        const uint32_t mask = t.mask[slot];
        int xb, yb, zb;
        unpack_key(t.keys[slot], xb, yb, zb);
        if (buf >= 0) {
            float2* vox = pool + (int64_t)buf * R3;
            for (int p = threadIdx.x; p < R3; p += blockDim.x) {
                const int xv = p % R, yv = (p / R) % R, zv = p / (R * R);
                const float xs = (float)(xb * R + xv) * voxel_size;
                const float ys = (float)(yb * R + yv) * voxel_size;
                const float zs = (float)(zb * R + zv) * voxel_size;
                float2 tw = vox[p];
                bool dirty = false;
                uint32_t m = mask;
                while (m) {
                    const int f = __builtin_ctz(m);
                    m &= m - 1;
                    const FrameParams& fp = fps[f];
                    const float xc = xs * fp.ext[0] + ys * fp.ext[1] + zs * fp.ext[2] + fp.ext[3];
                    const float yc = xs * fp.ext[4] + ys * fp.ext[5] + zs * fp.ext[6] + fp.ext[7];
                    const float zc = xs * fp.ext[8] + ys * fp.ext[9] + zs * fp.ext[10] + fp.ext[11];
                    const float inv_z = 1.0f / zc;
                    const float u = fp.fx * xc * inv_z + fp.cx;
                    const float v = fp.fy * yc * inv_z + fp.cy;
                    if (!(v >= 0 && u >= 0 && v <= hm1 && u <= wm1)) continue;
                    const int ui = (int)u, vi = (int)v;
                    const float d = depths[depth_frame[f] * HW + (int64_t)vi * W + ui] / depth_scale;
                    float sdf = d - zc;
                    if (d <= 0 || d > depth_max || zc <= 0 || sdf < -sdf_trunc) continue;
                    sdf = sdf < sdf_trunc ? sdf : sdf_trunc;
                    sdf /= sdf_trunc;
                    const float inv_wsum = 1.0f / (tw.y + 1);
                    const float wgt = tw.y;
                    tw.x = (wgt * tw.x + sdf) * inv_wsum;
                    tw.y = wgt + 1;
                    dirty = true;
                }
                if (dirty) vox[p] = tw;
            }
        }
        __syncthreads();
        if (threadIdx.x == 0) t.mask[slot] = 0;
    }
}

// ---- correctly rounded division without the v_div_scale / v_div_fixup wrapper ----------------
// The instruction sequence below is exactly what hipcc emits for IEEE float division
// (v_rcp_f32, Newton step, two residual corrections, final FMA = v_div_fmas without scaling).
// v_div_scale only rescales operands whose exponents put the quotient near over/underflow, and
// v_div_fixup only rewrites 0/inf/NaN cases, so for |num|, |den| in [2^-60, 2^60] the result
// equals a/b bit for bit; outside that range we call the real division.  Verified
// exhaustively on the GPU by tests/test_gpu_numerics.py.
__device__ __forceinline__ float div_rn_core(float a, float b) {
    const float y0 = __builtin_amdgcn_rcpf(b);
    const float nb = -b;
    const float e0 = __builtin_fmaf(nb, y0, 1.0f);
    const float y1 = __builtin_fmaf(e0, y0, y0);
    const float q0 = a * y1;
    const float r0 = __builtin_fmaf(nb, q0, a);
    const float q1 = __builtin_fmaf(r0, y1, q0);
    const float r1 = __builtin_fmaf(nb, q1, a);
    return __builtin_fmaf(r1, y1, q1);
}

__device__ __forceinline__ bool div_safe(float v) {
    const float m = fabsf(v);
    return m >= 0x1p-60f && m <= 0x1p60f;
}

__device__ __forceinline__ float div_rn(float a, float b) {
    return (div_safe(a) && div_safe(b)) ? div_rn_core(a, b) : a / b;
}

__device__ __forceinline__ float rcp_rn(float b) { return div_safe(b) ? div_rn_core(1.0f, b) : 1.0f / b; }

// Integrate, R known at compile time (R = 16 / 8): thread t owns the voxel column (x, y) =
// (t % R, t / R % R) for z in its z-range, keeps those voxels' (tsdf, weight) in registers for
// all frames of the batch, and evaluates Open3D's transform ((xs*e0 + ys*e1) + zs*e2) + e3 with
// the z-independent partial product hoisted per frame -- the same float operations in the same
// order, so the result is bit-identical to k_integrate.
template <int R, int G>
__global__ __launch_bounds__(256) void k_integrate_t(const int32_t* __restrict__ list, const int* __restrict__ counters,
                                                     int64_t list_cap, Table t, float2* __restrict__ pool,
                                                     float voxel_size, const float* __restrict__ depths, int64_t HW,
                                                     int H, int W, const FrameParams* __restrict__ fps,
                                                     const int64_t* __restrict__ depth_frame, float depth_scale,
                                                     float depth_max, float sdf_trunc) {
    constexpr int R2 = R * R;
    constexpr int R3 = R2 * R;
    constexpr int ZPER = R3 / 256;         // voxels per thread (16 at R=16, 2 at R=8)
    constexpr int ZSTEP = 256 / R2;        // z stride between a thread's voxels (1 at R=16, 4 at R=8)
    static_assert(R3 % 256 == 0, "R^3 must be a multiple of 256");
    static_assert(ZPER % G == 0, "group size must divide the voxels per thread");
    const bool unit_scale = depth_scale == 1.0f;  // d / 1 == d exactly: skip the division
    const int64_t n = min((int64_t)counters[kListCount], list_cap);
    const float hm1 = (float)H - 1.0f, wm1 = (float)W - 1.0f;
    const int tid = threadIdx.x;
    const int xv = tid % R, yv = (tid / R) % R, z0 = tid / R2;
    for (int64_t i = blockIdx.x; i < n; i += gridDim.x) {
        const int32_t slot = list[i];
        const int buf = t.vals[slot];
        const uint32_t mask = __builtin_amdgcn_readfirstlane(t.mask[slot]);
        int xb, yb, zb;
        unpack_key(t.keys[slot], xb, yb, zb);
        if (buf >= 0) {
            float2* vox = pool + (int64_t)buf * R3;
            float2 tw[ZPER];
            float zs[ZPER];
#pragma unroll
            for (int k = 0; k < ZPER; ++k) {
                tw[k] = vox[k * 256 + tid];
                zs[k] = (float)(zb * R + z0 + k * ZSTEP) * voxel_size;
            }
            const float xs = (float)(xb * R + xv) * voxel_size;
            const float ys = (float)(yb * R + yv) * voxel_size;
            uint32_t dirty = 0;
            uint32_t m = mask;
            while (m) {
                const int f = __builtin_ctz(m);
                m &= m - 1;
                const FrameParams& fp = fps[f];
                const float* __restrict__ dep = depths + depth_frame[f] * HW;
                const float ax = xs * fp.ext[0] + ys * fp.ext[1];
                const float ay = xs * fp.ext[4] + ys * fp.ext[5];
                const float az = xs * fp.ext[8] + ys * fp.ext[9];
                // Groups of G voxels: project all, issue all G depth gathers (branch-free, out-of-image
                // lanes read pixel 0 and are masked), then update -- G loads in flight per wave.
#pragma unroll
                for (int g = 0; g < ZPER; g += G) {
                    int pix[G];
                    float zcs[G];
                    bool in[G];
#pragma unroll
                    for (int j = 0; j < G; ++j) {
                        const int k = g + j;
                        const float xc = (ax + zs[k] * fp.ext[2]) + fp.ext[3];
                        const float yc = (ay + zs[k] * fp.ext[6]) + fp.ext[7];
                        const float zc = (az + zs[k] * fp.ext[10]) + fp.ext[11];
                        const float inv_z = rcp_rn(zc);
                        const float u = fp.fx * xc * inv_z + fp.cx;
                        const float v = fp.fy * yc * inv_z + fp.cy;
                        in[j] = v >= 0 && u >= 0 && v <= hm1 && u <= wm1;
                        const int ui = (int)(in[j] ? u : 0.f), vi = (int)(in[j] ? v : 0.f);
                        pix[j] = vi * W + ui;
                        zcs[j] = zc;
                    }
                    float dv[G];
#pragma unroll
                    for (int j = 0; j < G; ++j) dv[j] = dep[pix[j]];
#pragma unroll
                    for (int j = 0; j < G; ++j) {
                        const int k = g + j;
                        const float d = unit_scale ? dv[j] : div_rn(dv[j], depth_scale);
                        const float zc = zcs[j];
                        float sdf = d - zc;
                        if (!in[j] || d <= 0 || d > depth_max || zc <= 0 || sdf < -sdf_trunc) continue;
                        sdf = sdf < sdf_trunc ? sdf : sdf_trunc;
                        sdf = div_rn(sdf, sdf_trunc);
                        const float wgt = tw[k].y;
                        const float inv_wsum = rcp_rn(wgt + 1);
                        tw[k].x = (wgt * tw[k].x + sdf) * inv_wsum;
                        tw[k].y = wgt + 1;
                        dirty |= 1u << k;
                    }
                }
            }
#pragma unroll
            for (int k = 0; k < ZPER; ++k)
                if (dirty & (1u << k)) vox[k * 256 + tid] = tw[k];
        }
        __syncthreads();
        if (tid == 0) t.mask[slot] = 0;
    }
}

// Exhaustive-check kernels for the division shortcut (tests/test_gpu_numerics.py).
__global__ void k_check_rcp(uint32_t lo_bits, uint64_t count, uint32_t* mismatches, uint32_t* first_bad) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    const uint32_t bits = lo_bits + (uint32_t)i;
    const float b = __uint_as_float(bits);
    const float fast = rcp_rn(b), ref = 1.0f / b;
    if (__float_as_uint(fast) != __float_as_uint(ref)) {
        atomicAdd(mismatches, 1u);
        atomicMin(first_bad, bits);
    }
}

__global__ void k_check_div(float b, uint32_t lo_bits, uint64_t count, uint32_t* mismatches, uint32_t* first_bad) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    const uint32_t bits = lo_bits + (uint32_t)i;
    const float a = __uint_as_float(bits);
    const float fast = div_rn(a, b), ref = a / b;
    if (__float_as_uint(fast) != __float_as_uint(ref) && !(isnan(fast) && isnan(ref))) {
        atomicAdd(mismatches, 1u);
        atomicMin(first_bad, bits);
    }
}

__global__ void k_rehash(Table src, Table dst) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= src.cap) return;
    const uint64_t k = src.keys[i];
    if (k == kEmpty) return;
    const uint64_t m = (uint64_t)dst.cap - 1;
    uint64_t h = mix64(k) & m;
    for (;;) {
        const uint64_t old =
            atomicCAS((unsigned long long*)&dst.keys[h], (unsigned long long)kEmpty, (unsigned long long)k);
        if (old == kEmpty) break;
        h = (h + 1) & m;
    }
    dst.vals[h] = src.vals[i];
    dst.mask[h] = src.mask[i];
}

__global__ void k_set_counter(int* counters, int which, int value) { counters[which] = value; }

__global__ void k_fixup_alloc(Table t, int* counters, int64_t pool_cap, uint64_t* bkeys) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= t.cap) return;
    if (t.keys[i] == kEmpty || t.vals[i] != -2) return;
    const int b = atomicAdd(&counters[kPoolCount], 1);
    if (b < pool_cap) {
        t.vals[i] = b;
        bkeys[b] = t.keys[i];
    } else {
        atomicOr(&counters[kOverflow], 1);
    }
}

__global__ void k_gather_keys(const int32_t* __restrict__ list, int64_t n, const Table t, int32_t* keys_out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int x, y, z;
    unpack_key(t.keys[list[i]], x, y, z);
    keys_out[3 * i] = x;
    keys_out[3 * i + 1] = y;
    keys_out[3 * i + 2] = z;
}

__global__ void k_clear_slots(const int32_t* __restrict__ list, int64_t n, Table t, int clear_keys) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int32_t s = list[i];
    t.mask[s] = 0;
    if (clear_keys) {
        t.keys[s] = kEmpty;
        t.vals[s] = -1;
    }
}

__global__ void k_export(const float2* __restrict__ pool, const uint64_t* __restrict__ bkeys, int64_t n, int R3,
                         int32_t* keys, float* tsdf, float* weight) {
    const int64_t b = blockIdx.x;
    if (b >= n) return;
    if (threadIdx.x == 0 && keys) {
        int x, y, z;
        unpack_key(bkeys[b], x, y, z);
        keys[3 * b] = x;
        keys[3 * b + 1] = y;
        keys[3 * b + 2] = z;
    }
    for (int p = threadIdx.x; p < R3; p += blockDim.x) {
        const float2 tw = pool[b * R3 + p];
        if (tsdf) tsdf[b * R3 + p] = tw.x;
        if (weight) weight[b * R3 + p] = tw.y;
    }
}

__global__ void k_import(const int32_t* __restrict__ keys, int64_t n, const Table t, float2* pool, int R3,
                         const float* __restrict__ tsdf, const float* __restrict__ weight) {
    const int64_t b = blockIdx.x;
    if (b >= n) return;
    const int64_t slot = table_find(t, pack_key(keys[3 * b], keys[3 * b + 1], keys[3 * b + 2]));
    if (slot < 0) return;
    const int buf = t.vals[slot];
    if (buf < 0) return;
    for (int p = threadIdx.x; p < R3; p += blockDim.x)
        pool[(int64_t)buf * R3 + p] = make_float2(tsdf[b * R3 + p], weight[b * R3 + p]);
}

__global__ void k_pack(const int32_t* __restrict__ ukeys, int64_t U, const Table t, const float2* __restrict__ pool,
                       int R3, float2* out) {
    const int64_t b = blockIdx.x;
    if (b >= U) return;
    const int64_t slot = table_find(t, pack_key(ukeys[3 * b], ukeys[3 * b + 1], ukeys[3 * b + 2]));
    const int buf = slot >= 0 ? t.vals[slot] : -1;
    for (int p = threadIdx.x; p < R3; p += blockDim.x) {
        float2 r = make_float2(0.f, 0.f);
        if (buf >= 0) {
            const float2 tw = pool[(int64_t)buf * R3 + p];
            r = make_float2(tw.y * tw.x, tw.y);
        }
        out[b * R3 + p] = r;
    }
}

__global__ void k_unpack(const int32_t* __restrict__ ukeys, int64_t U, const Table t, float2* pool, int R3,
                         const float2* __restrict__ in) {
    const int64_t b = blockIdx.x;
    if (b >= U) return;
    const int64_t slot = table_find(t, pack_key(ukeys[3 * b], ukeys[3 * b + 1], ukeys[3 * b + 2]));
    if (slot < 0) return;
    const int buf = t.vals[slot];
    if (buf < 0) return;
    for (int p = threadIdx.x; p < R3; p += blockDim.x) {
        const float2 s = in[b * R3 + p];
        pool[(int64_t)buf * R3 + p] = make_float2(s.y > 0.f ? s.x / s.y : 0.f, s.y);
    }
}

// ------------------------------------------------------------------ host helpers
static int64_t next_pow2(int64_t x) {
    int64_t p = 1024;
    while (p < x) p <<= 1;
    return p;
}

static int alloc_table(Table& t, int64_t cap, hipStream_t s) {
    MQR_CHECK_HIP(hipMalloc(&t.keys, sizeof(uint64_t) * cap));
    MQR_CHECK_HIP(hipMalloc(&t.vals, sizeof(int32_t) * cap));
    MQR_CHECK_HIP(hipMalloc(&t.mask, sizeof(uint32_t) * cap));
    MQR_CHECK_HIP(hipMemsetAsync(t.keys, 0xff, sizeof(uint64_t) * cap, s));
    MQR_CHECK_HIP(hipMemsetAsync(t.vals, 0xff, sizeof(int32_t) * cap, s));
    MQR_CHECK_HIP(hipMemsetAsync(t.mask, 0, sizeof(uint32_t) * cap, s));
    t.cap = cap;
    return 0;
}

static void free_table(Table& t) {
    if (t.keys) (void)hipFree(t.keys);
    if (t.vals) (void)hipFree(t.vals);
    if (t.mask) (void)hipFree(t.mask);
    t = Table{};
}

static int ensure_list(mqr_vbg* v, int64_t cap) {
    if (v->list_cap >= cap) return 0;
    if (v->list) MQR_CHECK_HIP(hipFree(v->list));
    MQR_CHECK_HIP(hipMalloc(&v->list, sizeof(int32_t) * cap));
    v->list_cap = cap;
    return 0;
}

// Grow the main table (between batches only: masks clear, list empty) to hold `live` keys at <= 50 % load.
static int ensure_table(mqr_vbg* v, int64_t live) {
    const int64_t want = next_pow2(2 * live);
    if (v->tab.cap >= want) return ensure_list(v, v->tab.cap);
    Table nt{};
    if (alloc_table(nt, want, v->stream)) return 1;
    if (v->tab.cap) {
        const int64_t blocks = (v->tab.cap + 255) / 256;
        hipLaunchKernelGGL(k_rehash, dim3((unsigned)blocks), dim3(256), 0, v->stream, v->tab, nt);
        MQR_CHECK_HIP(hipGetLastError());
        MQR_CHECK_HIP(hipStreamSynchronize(v->stream));
        free_table(v->tab);
    }
    v->tab = nt;
    return ensure_list(v, v->tab.cap);
}

int grow_pool(mqr_vbg* v, int64_t need) {
    if (need <= v->pool_cap) return 0;
    int64_t ncap = std::max<int64_t>(need, v->pool_cap + v->pool_cap / 2);
    float2* np = nullptr;
    uint64_t* nk = nullptr;
    MQR_CHECK_HIP(hipMalloc(&np, sizeof(float2) * ncap * v->R3));
    MQR_CHECK_HIP(hipMalloc(&nk, sizeof(uint64_t) * ncap));
    MQR_CHECK_HIP(hipMemsetAsync(np, 0, sizeof(float2) * ncap * v->R3, v->stream));
    if (v->pool_cap) {
        MQR_CHECK_HIP(hipMemcpyAsync(np, v->pool, sizeof(float2) * v->pool_cap * v->R3, hipMemcpyDeviceToDevice,
                                     v->stream));
        MQR_CHECK_HIP(
            hipMemcpyAsync(nk, v->bkeys, sizeof(uint64_t) * v->pool_cap, hipMemcpyDeviceToDevice, v->stream));
    }
    MQR_CHECK_HIP(hipStreamSynchronize(v->stream));
    if (v->pool) MQR_CHECK_HIP(hipFree(v->pool));
    if (v->bkeys) MQR_CHECK_HIP(hipFree(v->bkeys));
    v->pool = np;
    v->bkeys = nk;
    v->pool_cap = ncap;
    return 0;
}

int ensure_fp(mqr_vbg* v, int n) {
    if (v->fp_cap >= n) return 0;
    if (v->d_fp) MQR_CHECK_HIP(hipFree(v->d_fp));
    if (v->h_fp) MQR_CHECK_HIP(hipHostFree(v->h_fp));
    const int cap = std::max(n, kMaxBatch);
    // FrameParams followed by the int64 depth-frame index array
    MQR_CHECK_HIP(hipMalloc(&v->d_fp, (sizeof(FrameParams) + sizeof(int64_t)) * cap));
    MQR_CHECK_HIP(hipHostMalloc(&v->h_fp, (sizeof(FrameParams) + sizeof(int64_t)) * cap, hipHostMallocDefault));
    v->fp_cap = cap;
    return 0;
}

int ensure_depth(mqr_vbg* v, int64_t floats) {
    if (v->depth_cap >= floats) return 0;
    if (v->d_depth) MQR_CHECK_HIP(hipFree(v->d_depth));
    MQR_CHECK_HIP(hipMalloc(&v->d_depth, sizeof(float) * floats));
    v->depth_cap = floats;
    return 0;
}

int sync_counters(mqr_vbg* v) {
    MQR_CHECK_HIP(hipMemcpyAsync(v->h_counters, v->counters, sizeof(int) * kCountersTotal, hipMemcpyDeviceToHost,
                                 v->stream));
    MQR_CHECK_HIP(hipStreamSynchronize(v->stream));
    return 0;
}

static int reset_batch_counters(mqr_vbg* v) {
    // keep kPoolCount; zero list/overflow/touch/frame-block and per-frame counters
    MQR_CHECK_HIP(hipMemsetAsync(v->counters + 1, 0, sizeof(int) * (kCountersTotal - 1), v->stream));
    return 0;
}

// After a touch/activate: allocate pool buffers that did not fit, if any.
static int resolve_pool_overflow(mqr_vbg* v) {
    if (sync_counters(v)) return 1;
    int* c = v->h_counters;
    if (c[kOverflow] & 2) {
        set_error("internal: block table full");
        return 1;
    }
    if (c[kOverflow] & 4) {
        set_error("internal: batch list overflow");
        return 1;
    }
    if (c[kOverflow] & 8) {
        set_error("block coordinate out of the supported range (|key| < 2^20 blocks)");
        return 2;
    }
    if (c[kOverflow] & 1) {
        const int64_t attempted = c[kPoolCount];
        const int64_t old_cap = v->pool_cap;
        if (grow_pool(v, std::max<int64_t>(attempted, old_cap * 2))) return 1;
        hipLaunchKernelGGL(k_set_counter, dim3(1), dim3(1), 0, v->stream, v->counters, (int)kPoolCount, (int)old_cap);
        MQR_CHECK_HIP(hipMemsetAsync(v->counters + kOverflow, 0, sizeof(int), v->stream));
        const int64_t blocks = (v->tab.cap + 255) / 256;
        hipLaunchKernelGGL(k_fixup_alloc, dim3((unsigned)blocks), dim3(256), 0, v->stream, v->tab, v->counters,
                           v->pool_cap, v->bkeys);
        MQR_CHECK_HIP(hipGetLastError());
        if (sync_counters(v)) return 1;
        if (c[kOverflow] & 1) {
            set_error("internal: pool growth failed");
            return 1;
        }
    }
    v->pool_count = c[kPoolCount];
    return 0;
}

static int launch_integrate(mqr_vbg* v, const float* depths, int64_t HW, int H, int W, int nframes,
                            float depth_scale, float depth_max, float sdf_trunc) {
    const int64_t n = std::min<int64_t>(v->h_counters[kListCount], v->list_cap);
    if (n == 0) return 0;
    const unsigned grid = (unsigned)std::min<int64_t>(n, 8192);
    const int64_t* depth_frame = reinterpret_cast<const int64_t*>(v->d_fp + v->fp_cap);
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (v->profile) {
        MQR_CHECK_HIP(hipEventCreate(&e0));
        MQR_CHECK_HIP(hipEventCreate(&e1));
        MQR_CHECK_HIP(hipEventRecord(e0, v->stream));
    }
#define MQR_LAUNCH_INT(RR, GG)                                                                                \
    hipLaunchKernelGGL((k_integrate_t<RR, GG>), dim3(grid), dim3(256), 0, v->stream, v->list, v->counters,          \
                       v->list_cap, v->tab, v->pool, v->voxel_size, depths, HW, H, W, v->d_fp, depth_frame,          \
                       depth_scale, depth_max, sdf_trunc)
    if (v->R == 16 && v->kernel_variant == 0)
        MQR_LAUNCH_INT(16, 8);
    else if (v->R == 16 && v->kernel_variant == 2)
        MQR_LAUNCH_INT(16, 4);
    else if (v->R == 16 && v->kernel_variant == 3)
        MQR_LAUNCH_INT(16, 16);
    else if (v->R == 16 && v->kernel_variant == 4)
        MQR_LAUNCH_INT(16, 2);
    else if (v->R == 8 && v->kernel_variant != 1)
        MQR_LAUNCH_INT(8, 2);
    else
        hipLaunchKernelGGL(k_integrate, dim3(grid), dim3(256), 0, v->stream, v->list, v->counters, v->list_cap,
                           v->tab, v->pool, v->R, v->voxel_size, depths, HW, H, W, v->d_fp, depth_frame, depth_scale,
                           depth_max, sdf_trunc);
    MQR_CHECK_HIP(hipGetLastError());
    if (v->profile) {
        MQR_CHECK_HIP(hipEventRecord(e1, v->stream));
        v->int_events.emplace_back(e0, e1);
        v->stats.integrate_launches += 1;
        v->stats.union_blocks += n;
        v->stats.frame_blocks += v->h_counters[kFrameBlocks];
        v->stats.frames += nframes;
    }
    return 0;
}

static void drain_events(mqr_vbg* v) {
    for (auto& e : v->int_events) {
        float ms = 0.f;
        if (hipEventSynchronize(e.second) == hipSuccess && hipEventElapsedTime(&ms, e.first, e.second) == hipSuccess)
            v->stats.integrate_ms += ms;
        (void)hipEventDestroy(e.first);
        (void)hipEventDestroy(e.second);
    }
    v->int_events.clear();
    for (auto& e : v->touch_events) {
        float ms = 0.f;
        if (hipEventSynchronize(e.second) == hipSuccess && hipEventElapsedTime(&ms, e.first, e.second) == hipSuccess)
            v->stats.touch_ms += ms;
        (void)hipEventDestroy(e.first);
        (void)hipEventDestroy(e.second);
    }
    v->touch_events.clear();
}

}  // namespace mqr

using namespace mqr;

// ====================================================================== C ABI
extern "C" {

int mqr_version(void) { return 100; }
const char* mqr_last_error(void) { return get_error(); }

int mqr_device_count(int* n) {
    MQR_CHECK_HIP(hipGetDeviceCount(n));
    return 0;
}

int mqr_device_alloc(int device, int64_t bytes, void** ptr) {
    MQR_CHECK_HIP(hipSetDevice(device));
    MQR_CHECK_HIP(hipMalloc(ptr, (size_t)bytes));
    return 0;
}

int mqr_device_free(int device, void* ptr) {
    MQR_CHECK_HIP(hipSetDevice(device));
    MQR_CHECK_HIP(hipFree(ptr));
    return 0;
}

int mqr_memcpy(void* dst, int dst_loc, const void* src, int src_loc, int64_t bytes, int device) {
    MQR_CHECK_HIP(hipSetDevice(device));
    hipMemcpyKind kind = dst_loc == MQR_DEVICE ? (src_loc == MQR_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice)
                                               : (src_loc == MQR_DEVICE ? hipMemcpyDeviceToHost : hipMemcpyHostToHost);
    MQR_CHECK_HIP(hipMemcpy(dst, src, (size_t)bytes, kind));
    return 0;
}

int mqr_device_synchronize(int device) {
    MQR_CHECK_HIP(hipSetDevice(device));
    MQR_CHECK_HIP(hipDeviceSynchronize());
    return 0;
}

int mqr_vbg_create(float voxel_size, int block_resolution, int64_t block_count, int device, mqr_vbg** out) {
    MQR_REQUIRE(out, "out is NULL");
    MQR_REQUIRE(voxel_size > 0.f, "voxel_size must be positive");
    MQR_REQUIRE(block_resolution >= 1 && block_resolution <= 64, "block_resolution must be in [1, 64]");
    MQR_REQUIRE(block_count >= 1, "block_count must be positive");
    int ndev = 0;
    MQR_CHECK_HIP(hipGetDeviceCount(&ndev));
    MQR_REQUIRE(device >= 0 && device < ndev, "device index out of range");
    MQR_CHECK_HIP(hipSetDevice(device));
    mqr_vbg* v = new mqr_vbg();
    v->device = device;
    v->voxel_size = voxel_size;
    v->R = block_resolution;
    v->R3 = (int64_t)block_resolution * block_resolution * block_resolution;
    if (hipStreamCreateWithFlags(&v->stream, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc(&v->counters, sizeof(int) * kCountersTotal) != hipSuccess ||
        hipHostMalloc(&v->h_counters, sizeof(int) * kCountersTotal, hipHostMallocDefault) != hipSuccess ||
        hipMemsetAsync(v->counters, 0, sizeof(int) * kCountersTotal, v->stream) != hipSuccess) {
        set_error("mqr_vbg_create: device allocation failed");
        mqr_vbg_destroy(v);
        return 1;
    }
    if (grow_pool(v, block_count) || ensure_table(v, block_count) || ensure_fp(v, kMaxBatch)) {
        mqr_vbg_destroy(v);
        return 1;
    }
    *out = v;
    return 0;
}

int mqr_vbg_destroy(mqr_vbg* v) {
    if (!v) return 0;
    (void)hipSetDevice(v->device);
    if (v->stream) (void)hipStreamSynchronize(v->stream);
    drain_events(v);
    free_table(v->tab);
    free_table(v->ftab);
    if (v->pool) (void)hipFree(v->pool);
    if (v->bkeys) (void)hipFree(v->bkeys);
    if (v->list) (void)hipFree(v->list);
    if (v->counters) (void)hipFree(v->counters);
    if (v->h_counters) (void)hipHostFree(v->h_counters);
    if (v->d_fp) (void)hipFree(v->d_fp);
    if (v->h_fp) (void)hipHostFree(v->h_fp);
    if (v->d_depth) (void)hipFree(v->d_depth);
    if (v->stream) (void)hipStreamDestroy(v->stream);
    delete v;
    return 0;
}

int mqr_vbg_reset(mqr_vbg* v) {
    MQR_REQUIRE(v, "null volume");
    MQR_CHECK_HIP(hipSetDevice(v->device));
    MQR_CHECK_HIP(hipMemsetAsync(v->tab.keys, 0xff, sizeof(uint64_t) * v->tab.cap, v->stream));
    MQR_CHECK_HIP(hipMemsetAsync(v->tab.vals, 0xff, sizeof(int32_t) * v->tab.cap, v->stream));
    MQR_CHECK_HIP(hipMemsetAsync(v->tab.mask, 0, sizeof(uint32_t) * v->tab.cap, v->stream));
    if (v->pool_count > 0)
        MQR_CHECK_HIP(hipMemsetAsync(v->pool, 0, sizeof(float2) * v->pool_count * v->R3, v->stream));
    MQR_CHECK_HIP(hipMemsetAsync(v->counters, 0, sizeof(int) * kCountersTotal, v->stream));
    MQR_CHECK_HIP(hipStreamSynchronize(v->stream));
    v->pool_count = 0;
    return 0;
}

int mqr_vbg_size(mqr_vbg* v, int64_t* n) {
    MQR_REQUIRE(v && n, "null argument");
    *n = v->pool_count;
    return 0;
}

int mqr_vbg_capacity(mqr_vbg* v, int64_t* c) {
    MQR_REQUIRE(v && c, "null argument");
    *c = v->pool_cap;
    return 0;
}

int mqr_vbg_params(mqr_vbg* v, float* voxel_size, int* R, int* device) {
    MQR_REQUIRE(v, "null volume");
    if (voxel_size) *voxel_size = v->voxel_size;
    if (R) *R = v->R;
    if (device) *device = v->device;
    return 0;
}

// Upload B frames' parameters; depth_frame[f] = index of frame f in the depth array.
static int upload_frames(mqr_vbg* v, const double* K, const double* T, const int* idx, int b, const int64_t* dframe) {
    if (ensure_fp(v, b)) return 1;
    // The stream was synchronised after the previous batch's touch, so the pinned mirror is free.
    int64_t* h_dframe = reinterpret_cast<int64_t*>(v->h_fp + v->fp_cap);
    for (int f = 0; f < b; ++f) {
        make_frame_params(K + 9 * idx[f], T + 16 * idx[f], &v->h_fp[f]);
        h_dframe[f] = dframe[f];
    }
    MQR_CHECK_HIP(hipMemcpyAsync(v->d_fp, v->h_fp, sizeof(FrameParams) * b, hipMemcpyHostToDevice, v->stream));
    MQR_CHECK_HIP(hipMemcpyAsync(v->d_fp + v->fp_cap, h_dframe, sizeof(int64_t) * b, hipMemcpyHostToDevice, v->stream));
    return 0;
}

int mqr_integrate_frames(mqr_vbg* v, const float* depths, int depth_loc, int B, int H, int W, const double* K,
                         const double* T_wc, const uint8_t* frame_ok, float depth_scale, float depth_max,
                         float trunc_mult) {
    MQR_REQUIRE(v && depths && K && T_wc, "null argument");
    MQR_REQUIRE(B >= 0 && H > 0 && W > 0, "bad frame shape");
    MQR_CHECK_HIP(hipSetDevice(v->device));
    const int64_t HW = (int64_t)H * W;
    const float sdf_trunc = v->voxel_size * trunc_mult;
    const float block_size = v->voxel_size * v->R;
    const int64_t max_touch = 4LL * (H / 4) * (W / 4);
    std::vector<int> valid;
    for (int i = 0; i < B; ++i)
        if (!frame_ok || frame_ok[i]) valid.push_back(i);
    for (size_t s = 0; s < valid.size(); s += kMaxBatch) {
        const int b = (int)std::min<size_t>(kMaxBatch, valid.size() - s);
        const int* idx = valid.data() + s;
        // table headroom for every key this batch could add (so no rehash mid-batch)
        if (ensure_table(v, v->pool_count + b * max_touch)) return 1;
        const float* dbase = depths;
        std::vector<int64_t> dframe(b);
        if (depth_loc == MQR_DEVICE) {
            for (int f = 0; f < b; ++f) dframe[f] = idx[f];
        } else {
            if (ensure_depth(v, b * HW)) return 1;
            for (int f = 0; f < b; ++f) {
                MQR_CHECK_HIP(hipMemcpyAsync(v->d_depth + f * HW, depths + (int64_t)idx[f] * HW, sizeof(float) * HW,
                                             hipMemcpyHostToDevice, v->stream));
                dframe[f] = f;
            }
            dbase = v->d_depth;
        }
        if (upload_frames(v, K, T_wc, idx, b, dframe.data())) return 1;
        if (reset_batch_counters(v)) return 1;
        const int64_t* d_dframe = reinterpret_cast<const int64_t*>(v->d_fp + v->fp_cap);
        const int n = (H / 4) * (W / 4);
        hipEvent_t e0 = nullptr, e1 = nullptr;
        if (v->profile) {
            MQR_CHECK_HIP(hipEventCreate(&e0));
            MQR_CHECK_HIP(hipEventCreate(&e1));
            MQR_CHECK_HIP(hipEventRecord(e0, v->stream));
        }
        if (n > 0)
            hipLaunchKernelGGL(k_touch, dim3((n + 255) / 256, b), dim3(256), 0, v->stream, dbase, HW, H, W, v->d_fp,
                               d_dframe, depth_scale, depth_max, sdf_trunc, block_size, v->tab, 1, v->counters,
                               v->pool_cap, v->bkeys, v->list, v->list_cap);
        MQR_CHECK_HIP(hipGetLastError());
        if (v->profile) {
            MQR_CHECK_HIP(hipEventRecord(e1, v->stream));
            v->touch_events.emplace_back(e0, e1);
            v->stats.touch_launches += 1;
            v->stats.pixels += (int64_t)b * HW;
        }
        if (resolve_pool_overflow(v)) return 1;
        for (int f = 0; f < b; ++f)
            if (v->h_counters[kFrameCounterBase + f] == 0) {
                set_error("No block is touched in TSDF volume, abort integration. Please check specified parameters, "
                          "especially depth_scale and voxel_size");
                return 3;
            }
        if (launch_integrate(v, dbase, HW, H, W, b, depth_scale, depth_max, sdf_trunc)) return 1;
    }
    MQR_CHECK_HIP(hipStreamSynchronize(v->stream));
    return 0;
}

int mqr_touch(mqr_vbg* v, const float* depth, int depth_loc, int H, int W, const double* K, const double* T_wc,
              float depth_scale, float depth_max, float trunc_mult, int32_t* keys_out, int64_t* n_out) {
    MQR_REQUIRE(v && depth && K && T_wc && keys_out && n_out, "null argument");
    MQR_CHECK_HIP(hipSetDevice(v->device));
    const int64_t HW = (int64_t)H * W;
    const int64_t max_touch = 4LL * (H / 4) * (W / 4);
    const int64_t want = next_pow2(2 * std::max<int64_t>(max_touch, 1));
    if (v->ftab.cap < want) {
        free_table(v->ftab);
        if (alloc_table(v->ftab, want, v->stream)) return 1;
    }
    if (ensure_list(v, std::max(v->tab.cap, v->ftab.cap))) return 1;
    const float* dptr = depth;
    if (depth_loc != MQR_DEVICE) {
        if (ensure_depth(v, HW)) return 1;
        MQR_CHECK_HIP(hipMemcpyAsync(v->d_depth, depth, sizeof(float) * HW, hipMemcpyHostToDevice, v->stream));
        dptr = v->d_depth;
    }
    const int idx = 0;
    const int64_t dframe = 0;
    if (upload_frames(v, K, T_wc, &idx, 1, &dframe)) return 1;
    if (reset_batch_counters(v)) return 1;
    const int n = (H / 4) * (W / 4);
    if (n > 0)
        hipLaunchKernelGGL(k_touch, dim3((n + 255) / 256, 1), dim3(256), 0, v->stream, dptr, HW, H, W, v->d_fp,
                           reinterpret_cast<const int64_t*>(v->d_fp + v->fp_cap), depth_scale, depth_max,
                           v->voxel_size * trunc_mult, v->voxel_size * v->R, v->ftab, 0, v->counters, v->pool_cap,
                           v->bkeys, v->list, v->list_cap);
    MQR_CHECK_HIP(hipGetLastError());
    if (sync_counters(v)) return 1;
    const int64_t cnt = v->h_counters[kListCount];
    int32_t* dkeys = nullptr;
    if (cnt > 0) {
        MQR_CHECK_HIP(hipMalloc(&dkeys, sizeof(int32_t) * 3 * cnt));
        hipLaunchKernelGGL(k_gather_keys, dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0, v->stream, v->list, cnt,
                           v->ftab, dkeys);
        MQR_CHECK_HIP(hipMemcpyAsync(keys_out, dkeys, sizeof(int32_t) * 3 * cnt, hipMemcpyDeviceToHost, v->stream));
        hipLaunchKernelGGL(k_clear_slots, dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0, v->stream, v->list, cnt,
                           v->ftab, 1);
        MQR_CHECK_HIP(hipStreamSynchronize(v->stream));
        MQR_CHECK_HIP(hipFree(dkeys));
    }
    *n_out = cnt;
    if (v->h_counters[kFrameCounterBase] == 0) {
        set_error("No block is touched in TSDF volume, abort integration. Please check specified parameters, "
                  "especially depth_scale and voxel_size");
        return 3;
    }
    return 0;
}

int mqr_integrate(mqr_vbg* v, const int32_t* keys, int64_t n, const float* depth, int depth_loc, int H, int W,
                  const double* K, const double* T_wc, float depth_scale, float depth_max, float trunc_mult) {
    MQR_REQUIRE(v && depth && K && T_wc && (keys || n == 0), "null argument");
    MQR_CHECK_HIP(hipSetDevice(v->device));
    if (n == 0) return 0;
    const int64_t HW = (int64_t)H * W;
    if (ensure_table(v, v->pool_count + n)) return 1;
    const float* dptr = depth;
    if (depth_loc != MQR_DEVICE) {
        if (ensure_depth(v, HW)) return 1;
        MQR_CHECK_HIP(hipMemcpyAsync(v->d_depth, depth, sizeof(float) * HW, hipMemcpyHostToDevice, v->stream));
        dptr = v->d_depth;
    }
    int32_t* dkeys = nullptr;
    MQR_CHECK_HIP(hipMalloc(&dkeys, sizeof(int32_t) * 3 * n));
    MQR_CHECK_HIP(hipMemcpyAsync(dkeys, keys, sizeof(int32_t) * 3 * n, hipMemcpyHostToDevice, v->stream));
    const int idx = 0;
    const int64_t dframe = 0;
    if (upload_frames(v, K, T_wc, &idx, 1, &dframe)) return 1;
    if (reset_batch_counters(v)) return 1;
    hipLaunchKernelGGL(k_activate, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, v->stream, dkeys, n, v->tab,
                       v->counters, v->pool_cap, v->bkeys, v->list, v->list_cap, 1);
    MQR_CHECK_HIP(hipGetLastError());
    if (resolve_pool_overflow(v)) {
        (void)hipFree(dkeys);
        return 1;
    }
    int rc = launch_integrate(v, dptr, HW, H, W, 1, depth_scale, depth_max, v->voxel_size * trunc_mult);
    MQR_CHECK_HIP(hipStreamSynchronize(v->stream));
    MQR_CHECK_HIP(hipFree(dkeys));
    return rc;
}

int mqr_vbg_export(mqr_vbg* v, int32_t* keys, float* tsdf, float* weight, int loc) {
    MQR_REQUIRE(v, "null volume");
    MQR_CHECK_HIP(hipSetDevice(v->device));
    const int64_t n = v->pool_count;
    if (n == 0) return 0;
    int32_t* dk = keys;
    float* dt = tsdf;
    float* dw = weight;
    if (loc != MQR_DEVICE) {
        dk = nullptr;
        dt = nullptr;
        dw = nullptr;
        if (keys) MQR_CHECK_HIP(hipMalloc(&dk, sizeof(int32_t) * 3 * n));
        if (tsdf) MQR_CHECK_HIP(hipMalloc(&dt, sizeof(float) * n * v->R3));
        if (weight) MQR_CHECK_HIP(hipMalloc(&dw, sizeof(float) * n * v->R3));
    }
    hipLaunchKernelGGL(k_export, dim3((unsigned)n), dim3(256), 0, v->stream, v->pool, v->bkeys, n, (int)v->R3, dk, dt,
                       dw);
    MQR_CHECK_HIP(hipGetLastError());
    if (loc != MQR_DEVICE) {
        if (keys) MQR_CHECK_HIP(hipMemcpyAsync(keys, dk, sizeof(int32_t) * 3 * n, hipMemcpyDeviceToHost, v->stream));
        if (tsdf) MQR_CHECK_HIP(hipMemcpyAsync(tsdf, dt, sizeof(float) * n * v->R3, hipMemcpyDeviceToHost, v->stream));
        if (weight)
            MQR_CHECK_HIP(hipMemcpyAsync(weight, dw, sizeof(float) * n * v->R3, hipMemcpyDeviceToHost, v->stream));
        MQR_CHECK_HIP(hipStreamSynchronize(v->stream));
        if (dk) (void)hipFree(dk);
        if (dt) (void)hipFree(dt);
        if (dw) (void)hipFree(dw);
    } else {
        MQR_CHECK_HIP(hipStreamSynchronize(v->stream));
    }
    return 0;
}

// Activate `ukeys` (device, U triplets) without marking frames.
static int activate_device_keys(mqr_vbg* v, const int32_t* dkeys, int64_t U) {
    if (ensure_table(v, v->pool_count + U)) return 1;
    if (reset_batch_counters(v)) return 1;
    if (U > 0)
        hipLaunchKernelGGL(k_activate, dim3((unsigned)((U + 255) / 256)), dim3(256), 0, v->stream, dkeys, U, v->tab,
                           v->counters, v->pool_cap, v->bkeys, v->list, v->list_cap, 0);
    MQR_CHECK_HIP(hipGetLastError());
    return resolve_pool_overflow(v);
}

int mqr_vbg_import(mqr_vbg* v, const int32_t* keys, const float* tsdf, const float* weight, int64_t n, int loc) {
    MQR_REQUIRE(v && ((keys && tsdf && weight) || n == 0), "null argument");
    MQR_CHECK_HIP(hipSetDevice(v->device));
    if (n == 0) return 0;
    const int32_t* dk = keys;
    const float* dt = tsdf;
    const float* dw = weight;
    int32_t* hk = nullptr;
    float *ht = nullptr, *hw = nullptr;
    if (loc != MQR_DEVICE) {
        MQR_CHECK_HIP(hipMalloc(&hk, sizeof(int32_t) * 3 * n));
        MQR_CHECK_HIP(hipMalloc(&ht, sizeof(float) * n * v->R3));
        MQR_CHECK_HIP(hipMalloc(&hw, sizeof(float) * n * v->R3));
        MQR_CHECK_HIP(hipMemcpyAsync(hk, keys, sizeof(int32_t) * 3 * n, hipMemcpyHostToDevice, v->stream));
        MQR_CHECK_HIP(hipMemcpyAsync(ht, tsdf, sizeof(float) * n * v->R3, hipMemcpyHostToDevice, v->stream));
        MQR_CHECK_HIP(hipMemcpyAsync(hw, weight, sizeof(float) * n * v->R3, hipMemcpyHostToDevice, v->stream));
        dk = hk;
        dt = ht;
        dw = hw;
    }
    int rc = activate_device_keys(v, dk, n);
    if (!rc) {
        hipLaunchKernelGGL(k_import, dim3((unsigned)n), dim3(256), 0, v->stream, dk, n, v->tab, v->pool, (int)v->R3,
                           dt, dw);
        if (hipGetLastError() != hipSuccess || hipStreamSynchronize(v->stream) != hipSuccess) {
            set_error("mqr_vbg_import: kernel failed");
            rc = 1;
        }
    }
    if (hk) (void)hipFree(hk);
    if (ht) (void)hipFree(ht);
    if (hw) (void)hipFree(hw);
    return rc;
}

int mqr_vbg_pack_weighted(mqr_vbg* v, const int32_t* union_keys, int64_t U, float* packed) {
    MQR_REQUIRE(v && (U == 0 || (union_keys && packed)), "null argument");
    MQR_CHECK_HIP(hipSetDevice(v->device));
    if (U == 0) return 0;
    hipLaunchKernelGGL(k_pack, dim3((unsigned)U), dim3(256), 0, v->stream, union_keys, U, v->tab, v->pool, (int)v->R3,
                       reinterpret_cast<float2*>(packed));
    MQR_CHECK_HIP(hipGetLastError());
    MQR_CHECK_HIP(hipStreamSynchronize(v->stream));
    return 0;
}

int mqr_vbg_unpack_weighted(mqr_vbg* v, const int32_t* union_keys, int64_t U, const float* packed) {
    MQR_REQUIRE(v && (U == 0 || (union_keys && packed)), "null argument");
    MQR_CHECK_HIP(hipSetDevice(v->device));
    if (U == 0) return 0;
    if (activate_device_keys(v, union_keys, U)) return 1;
    hipLaunchKernelGGL(k_unpack, dim3((unsigned)U), dim3(256), 0, v->stream, union_keys, U, v->tab, v->pool,
                       (int)v->R3, reinterpret_cast<const float2*>(packed));
    MQR_CHECK_HIP(hipGetLastError());
    MQR_CHECK_HIP(hipStreamSynchronize(v->stream));
    return 0;
}

int mqr_vbg_set_variant(mqr_vbg* v, int variant) {
    MQR_REQUIRE(v, "null volume");
    v->kernel_variant = variant;
    return 0;
}

int mqr_check_division(int device, int which, float b, uint32_t lo_bits, uint64_t count, uint32_t* mismatches,
                       uint32_t* first_bad) {
    MQR_REQUIRE(mismatches && first_bad, "null argument");
    MQR_CHECK_HIP(hipSetDevice(device));
    uint32_t* d = nullptr;
    MQR_CHECK_HIP(hipMalloc(&d, 2 * sizeof(uint32_t)));
    const uint32_t init[2] = {0u, 0xffffffffu};
    MQR_CHECK_HIP(hipMemcpy(d, init, sizeof(init), hipMemcpyHostToDevice));
    const uint64_t chunk = 1ull << 30;
    for (uint64_t off = 0; off < count; off += chunk) {
        const uint64_t c = std::min<uint64_t>(chunk, count - off);
        const unsigned blocks = (unsigned)((c + 255) / 256);
        if (which == 0)
            hipLaunchKernelGGL(k_check_rcp, dim3(blocks), dim3(256), 0, 0, lo_bits + (uint32_t)off, c, d, d + 1);
        else
            hipLaunchKernelGGL(k_check_div, dim3(blocks), dim3(256), 0, 0, b, lo_bits + (uint32_t)off, c, d, d + 1);
        MQR_CHECK_HIP(hipGetLastError());
    }
    uint32_t out[2];
    MQR_CHECK_HIP(hipMemcpy(out, d, sizeof(out), hipMemcpyDeviceToHost));
    (void)hipFree(d);
    *mismatches = out[0];
    *first_bad = out[1];
    return 0;
}

int mqr_vbg_profile(mqr_vbg* v, int enable) {
    MQR_REQUIRE(v, "null volume");
    v->profile = enable != 0;
    return 0;
}

int mqr_vbg_stats(mqr_vbg* v, mqr_stats* out, int reset) {
    MQR_REQUIRE(v && out, "null argument");
    MQR_CHECK_HIP(hipSetDevice(v->device));
    drain_events(v);
    *out = v->stats;
    if (reset) v->stats = mqr_stats{};
    return 0;
}

}  // extern "C"

// vbg_kernels.hpp -- device code of the TSDF volume (included once, by vbg.hip).
// Open3D 0.19 VoxelBlockGrid semantics; float32 with no FMA contraction.
#pragma once
#include "mqr_common.hpp"

namespace mqr {

// ------------------------------------------------------------------ device helpers
__device__ __forceinline__ bmask_t readfirstlane_u64(bmask_t v) {
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return (bmask_t)hi << 32 | lo;
}

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
__device__ inline int64_t table_insert(Table t, uint64_t k, bool alloc, int* counters, int* pool_ctr,
                                       int64_t pool_cap, uint64_t* bkeys) {
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
                    const int b = atomicAdd(pool_ctr, 1);
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

// Sets frame bit f of the slot (appending the slot to the batch list at its first bit); returns
// whether the bit was new -- the caller counts those per wave (kFrameBlocks).
__device__ inline bool mark_slot(Table t, int64_t slot, int f, int* counters, int32_t* list, int64_t list_cap) {
    const bmask_t bit = (bmask_t)1 << f;
    // every workgroup of a frame that sees the block marks it: read the word at L2 first and only
    // the workgroups that still find the bit clear issue the (same-address, serialised) atomic
    if (__hip_atomic_load(&t.mask[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & bit) return false;
    const bmask_t old = atomicOr((unsigned long long*)&t.mask[slot], (unsigned long long)bit);
    if (old == 0) {
        const int pos = atomicAdd(&counters[kListCount], 1);
        if (pos < list_cap)
            list[pos] = (int32_t)slot;
        else
            atomicOr(&counters[kOverflow], 4);
    }
    return !(old & bit);
}

// Sum of a per-lane count over the wave, added to *ctr by one lane (an LDS word of the workgroup
// here; per-thread global atomics on the batch counters serialised on a handful of addresses).
__device__ inline void wave_add(int* ctr, int v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(ctr, v);
}

// ------------------------------------------------------------------ kernels
// compute_unique_block_coordinates for a batch: blockIdx.y = batch frame (bit), one thread per
// stride-4 pixel, 4 samples over [max(d - trunc, 0), min(d + trunc, depth_max)] (Appendix A.2).
__global__ __launch_bounds__(256) void k_touch(const float* __restrict__ depths, int64_t HW, int H, int W,
                                               const FrameParams* __restrict__ fps,
                                               const int64_t* __restrict__ depth_frame, float depth_scale,
                                               float depth_max, float sdf_trunc, float block_size, Table t,
                                               int alloc, int* counters, int* pool_ctr, int64_t pool_cap,
                                               uint64_t* bkeys, int32_t* list, int64_t list_cap) {
    // keys already inserted by this workgroup (a 256-pixel strip of one frame shares most of its
    // blocks): only a key's first occurrence probes the global table and sets the frame bit
    constexpr int kSeen = 2048;
    __shared__ unsigned long long seen[kSeen];
    __shared__ int wg_count[2];  // valid samples, new frame bits: one global atomic per workgroup
    for (int i = threadIdx.x; i < kSeen; i += blockDim.x) seen[i] = kEmpty;
    if (threadIdx.x < 2) wg_count[threadIdx.x] = 0;
    __syncthreads();
    const int f = blockIdx.y;
    const FrameParams& fp = fps[f];
    const int cols = W / 4, rows = H / 4, n = rows * cols;
    const int w = blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t key[4] = {kEmpty, kEmpty, kEmpty, kEmpty};
    int valid = 0, fresh = 0;
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
            valid = 4;
        }
    }
    wave_add(&wg_count[0], valid);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const uint64_t k = key[s];
        if (k == kEmpty || (s > 0 && key[s - 1] == k)) continue;
        bool first = false;
        uint32_t h = (uint32_t)mix64(k) & (kSeen - 1);
        for (int p = 0; p < kSeen; ++p) {  // <= 1024 keys per workgroup: at most half full
            const unsigned long long old = atomicCAS(&seen[h], (unsigned long long)kEmpty, (unsigned long long)k);
            if (old == kEmpty) first = true;
            if (old == kEmpty || old == k) break;
            h = (h + 1) & (kSeen - 1);
        }
        if (first) {
            const int64_t slot = table_insert(t, k, alloc != 0, counters, pool_ctr, pool_cap, bkeys);
            if (slot >= 0) fresh += mark_slot(t, slot, f, counters, list, list_cap);
        }
    }
    wave_add(&wg_count[1], fresh);
    __syncthreads();
    if (threadIdx.x == 0) {
        if (wg_count[0]) atomicAdd(&counters[kFrameCounterBase + f], wg_count[0]);
        if (wg_count[1]) atomicAdd(&counters[kFrameBlocks], wg_count[1]);
    }
}

// Activate explicit keys (vbg.integrate(block_coords, ...)); marks frame bit 0.
__global__ void k_activate(const int32_t* __restrict__ keys, int64_t n, Table t, int* counters, int* pool_ctr,
                           int64_t pool_cap, uint64_t* bkeys, int32_t* list, int64_t list_cap, int mark) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int x = keys[3 * i], y = keys[3 * i + 1], z = keys[3 * i + 2];
    if (!key_in_range(x, y, z)) {
        atomicOr(&counters[kOverflow], 8);
        return;
    }
    const int64_t slot = table_insert(t, pack_key(x, y, z), true, counters, pool_ctr, pool_cap, bkeys);
    if (slot >= 0 && mark && mark_slot(t, slot, 0, counters, list, list_cap)) atomicAdd(&counters[kFrameBlocks], 1);
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
        const bmask_t mask = t.mask[slot];
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
                bmask_t m = mask;
                while (m) {
                    const int f = __builtin_ctzll(m);
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

// XCD-aware list order: consecutive workgroups are dealt round-robin over the 8 XCDs, so hand XCD
// x (= L % 8) chunks of C consecutive list entries in turn.  List entries are appended in touch
// (pixel) order, so a chunk is a spatially coherent set of blocks whose depth gathers share
// pixels and can hit in that XCD's L2; interleaving the chunks keeps the XCDs' loads balanced.
// Bijective on [0, n) (the tail past the last full round keeps its order); speed only.
template <int C>
__device__ __forceinline__ int64_t xcd_swizzle(int64_t L, int64_t n) {
    const int64_t full = n / (8 * C) * (8 * C);
    if (L >= full) return L;
    const int64_t x = L & 7, s = L >> 3;
    return ((s / C) * 8 + x) * C + s % C;
}

// Operand checks of the unguarded division core, on the float bits (|x| = e):
//   denominator / reciprocal: 2^-60 <= |x| <= 2^60 (also rejects 0, inf, NaN);
//   numerator below a safe denominator: 0 or |x| >= 2^-60 (the clamp keeps it <= the denominator).
__device__ __forceinline__ bool den_unsafe(float v) {
    return ((__float_as_uint(v) & 0x7fffffffu) - 0x21800000u) > 0x3c000000u;
}
__device__ __forceinline__ bool num_unsafe(float v) {
    return ((__float_as_uint(v) & 0x7fffffffu) - 1u) < 0x217fffffu;
}

// All frames of the batch over one thread's voxel column (see k_integrate_t).  EXACT = false
// evaluates every division with the bare core and returns whether any operand left the range in
// which the core is exact (den_unsafe / num_unsafe); the caller then discards the column results
// of the whole block and re-runs it with EXACT = true.  The flag is data-independent of which
// path ran, so the exact pass reproduces k_integrate bit for bit, and the fast pass has no
// per-voxel branches around its divisions.
template <int ZPER, int G, bool EXACT>
__device__ __forceinline__ bool integrate_column(float2 (&tw)[ZPER], uint32_t& dirty, bmask_t mask,
                                                 const float (&zs)[ZPER], float xs, float ys,
                                                 const float* __restrict__ depths, int64_t HW, int W, float hm1,
                                                 float wm1, const FrameParams* __restrict__ fps,
                                                 const int64_t* __restrict__ depth_frame, float depth_scale,
                                                 bool unit_scale, float depth_max, float sdf_trunc) {
    bool bad = false;
    bmask_t m = mask;
    while (m) {
        const int f = __builtin_ctzll(m);
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
                float inv_z;
                if (EXACT) {
                    inv_z = rcp_rn(zc);
                } else {
                    inv_z = div_rn_core(1.0f, zc);
                    bad |= den_unsafe(zc);
                }
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
                float d;
                if (unit_scale) {
                    d = dv[j];
                } else if (EXACT) {
                    d = div_rn(dv[j], depth_scale);
                } else {
                    d = div_rn_core(dv[j], depth_scale);
                    bad |= in[j] && dv[j] != 0.0f && den_unsafe(dv[j]);  // 0 / s = +0 in the core
                }
                const float zc = zcs[j];
                float sdf = d - zc;
                if (!in[j] || d <= 0 || d > depth_max || zc <= 0 || sdf < -sdf_trunc) continue;
                sdf = sdf < sdf_trunc ? sdf : sdf_trunc;
                const float wgt = tw[k].y;
                float inv_wsum;
                if (EXACT) {
                    sdf = div_rn(sdf, sdf_trunc);
                    inv_wsum = rcp_rn(wgt + 1);
                } else {
                    bad |= num_unsafe(sdf) || den_unsafe(wgt + 1);
                    sdf = div_rn_core(sdf, sdf_trunc);
                    inv_wsum = div_rn_core(1.0f, wgt + 1);
                }
                tw[k].x = (wgt * tw[k].x + sdf) * inv_wsum;
                tw[k].y = wgt + 1;
                dirty |= 1u << k;
            }
        }
    }
    return bad;
}

// Integrate, R known at compile time (R = 16 / 8): thread t owns the voxel column (x, y) =
// (t % R, t / R % R) for z in its z-range, keeps those voxels' (tsdf, weight) in registers for
// all frames of the batch, and evaluates Open3D's transform ((xs*e0 + ys*e1) + zs*e2) + e3 with
// the z-independent partial product hoisted per frame -- the same float operations in the same
// order, so the result is bit-identical to k_integrate.  FAST: unguarded division core with a
// block-level exact re-run when any operand is out of its range (host guarantees sdf_trunc and
// depth_scale are in range).
//
// SPLIT > 1: SPLIT workgroups per block, each on R / SPLIT consecutive z-layers (finer grain for the
// longest-first schedule); needs lmask, the batch masks in list order (k_lpt_order), because the
// part-0 workgroup clears the table mask while its sibling may not have read it yet.
//
// FAST with bad_out != nullptr: a block whose operands left the core's exact range is not written
// back; its (slot, mask) goes to bad_out (count at counters[kBadCount]) for an exact re-run by a
// follow-up launch of the exact kernel over that list.  The fast kernel then carries no second,
// exact copy of the column loop (fewer registers, no per-voxel branches).
template <int R, int G, int SWZ = 0, bool FAST = false, int NT = 256, int WPE = 1, int SPLIT = 1, bool EXTFIX = false>
__global__ __launch_bounds__(NT, WPE) void k_integrate_t(const int32_t* __restrict__ list,
                                                     const bmask_t* __restrict__ lmask,
                                                     int32_t* __restrict__ bad_out,
                                                     int* __restrict__ counters,
                                                     int64_t list_cap, Table t, float2* __restrict__ pool,
                                                     float voxel_size, const float* __restrict__ depths, int64_t HW,
                                                     int H, int W, const FrameParams* __restrict__ fps,
                                                     const int64_t* __restrict__ depth_frame, float depth_scale,
                                                     float depth_max, float sdf_trunc) {
    constexpr int R2 = R * R;
    constexpr int R3 = R2 * R;
    constexpr int ZPER = R3 / (NT * SPLIT);  // voxels per thread (16 at R=16, NT=256; 2 at R=8)
    constexpr int ZSTEP = NT / R2;           // z stride between a thread's voxels (1 at R=16, NT=256)
    static_assert(R3 % (NT * SPLIT) == 0 && NT % R2 == 0, "NT * SPLIT must divide R^3, NT a multiple of R^2");
    static_assert(SPLIT == 1 || SWZ == 0, "split blocks use the plain list order");
    static_assert(ZPER % G == 0, "group size must divide the voxels per thread");
    const bool unit_scale = depth_scale == 1.0f;  // d / 1 == d exactly: skip the division
    const int64_t n = min((int64_t)counters[kListCount], list_cap);
    const float hm1 = (float)H - 1.0f, wm1 = (float)W - 1.0f;
    const int tid = threadIdx.x;
    const int xv = tid % R, yv = (tid / R) % R;
    for (int64_t U = blockIdx.x; U < n * SPLIT; U += gridDim.x) {
        const int64_t L = SPLIT > 1 ? U / SPLIT : U;
        const int part = SPLIT > 1 ? (int)(U % SPLIT) : 0;
        const int z0 = tid / R2 + part * (R / SPLIT);
        const int64_t i = SWZ > 0 ? xcd_swizzle<(SWZ > 0 ? SWZ : 1)>(L, n) : L;
        const int32_t slot = list[i];
        const int buf = t.vals[slot];
        const bmask_t mask = readfirstlane_u64(lmask ? lmask[i] : t.mask[slot]);
        int xb, yb, zb;
        unpack_key(t.keys[slot], xb, yb, zb);
        if (buf >= 0) {
            float2* vox = pool + (int64_t)buf * R3 + part * (R3 / SPLIT);
            float2 tw[ZPER];
            float zs[ZPER];
#pragma unroll
            for (int k = 0; k < ZPER; ++k) {
                tw[k] = vox[k * NT + tid];
                zs[k] = (float)(zb * R + z0 + k * ZSTEP) * voxel_size;
            }
            const float xs = (float)(xb * R + xv) * voxel_size;
            const float ys = (float)(yb * R + yv) * voxel_size;
            uint32_t dirty = 0;
            const bool bad = integrate_column<ZPER, G, !FAST>(tw, dirty, mask, zs, xs, ys, depths, HW, W, hm1, wm1,
                                                           fps, depth_frame, depth_scale, unit_scale, depth_max,
                                                           sdf_trunc);
            if (FAST && __syncthreads_or(bad)) {  // block-uniform
                if (EXTFIX) {  // hand the block to the exact fix-up launch, leave it unwritten
                    if (tid == 0) {
                        const int j = atomicAdd(&counters[kBadCount], 1);
                        bad_out[j] = slot;
                        reinterpret_cast<bmask_t*>(bad_out + list_cap)[j] = mask;
                    }
                    dirty = 0;
                } else {  // redo this block exactly
#pragma unroll
                    for (int k = 0; k < ZPER; ++k) tw[k] = vox[k * NT + tid];
                    dirty = 0;
                    integrate_column<ZPER, G, true>(tw, dirty, mask, zs, xs, ys, depths, HW, W, hm1, wm1, fps,
                                                    depth_frame, depth_scale, unit_scale, depth_max, sdf_trunc);
                }
            }
#pragma unroll
            for (int k = 0; k < ZPER; ++k)
                if (dirty & (1u << k)) vox[k * NT + tid] = tw[k];
        }
        __syncthreads();
        if (tid == 0 && part == 0) t.mask[slot] = 0;
    }
}

// Longest-processing-time order of a batch list: counting sort by the number of the batch's frames
// that touched each block (popcount of its slot mask), descending.  The integrate grid then ends on
// short blocks instead of whichever long blocks the touch order happened to put last.  One
// workgroup; order within a bin is arbitrary (blocks are independent, results unchanged).
__global__ __launch_bounds__(1024) void k_lpt_order(const int32_t* __restrict__ list, const int* __restrict__ counters,
                                                    int64_t list_cap, const bmask_t* __restrict__ mask,
                                                    int32_t* __restrict__ out, bmask_t* __restrict__ out_mask) {
    __shared__ int hist[kMaxBatch + 1];
    const int n = (int)min((int64_t)counters[kListCount], list_cap);
    if (threadIdx.x <= kMaxBatch) hist[threadIdx.x] = 0;
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += blockDim.x) atomicAdd(&hist[__popcll(mask[list[i]])], 1);
    __syncthreads();
    if (threadIdx.x == 0) {
        int acc = 0;
        for (int c = kMaxBatch; c >= 0; --c) {
            const int h = hist[c];
            hist[c] = acc;
            acc += h;
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const int32_t s = list[i];
        const bmask_t m = mask[s];
        const int pos = atomicAdd(&hist[__popcll(m)], 1);
        out[pos] = s;
        out_mask[pos] = m;
    }
}

// ---- packed-f32 integrate (v_pk_mul/add/fma_f32: two voxels per VALU instruction) ------------
typedef float f2v __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f2v fma2(f2v a, f2v b, f2v c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f2v splat2(float x) { return f2v{x, x}; }

// 1 / b through the core sequence (q0 = 1 * y1 = y1), elementwise; exact for 2^-60 <= |b| <= 2^60.
__device__ __forceinline__ f2v rcp_core2(f2v b) {
    const f2v one = splat2(1.0f);
    const f2v y0 = {__builtin_amdgcn_rcpf(b.x), __builtin_amdgcn_rcpf(b.y)};
    const f2v nb = -b;
    const f2v y1 = fma2(fma2(nb, y0, one), y0, y0);
    const f2v q1 = fma2(fma2(nb, y1, one), y1, y1);
    return fma2(fma2(nb, q1, one), y1, q1);
}

// a / t for a launch-constant t with its refined reciprocal y1t precomputed (same core sequence).
__device__ __forceinline__ f2v div_const2(f2v a, f2v nbt, f2v y1t) {
    const f2v q0 = a * y1t;
    const f2v q1 = fma2(fma2(nbt, q0, a), y1t, q0);
    return fma2(fma2(nbt, q1, a), y1t, q1);
}

// Fast pass of one column with the (tsdf, weight) of voxels (2q, 2q+1) packed in T[q], Wt[q].
// Preconditions (checked by the caller): depth_scale == 1, sdf_trunc in [2^-60, 2^60], every
// weight in [0, 2^59].  Returns true if some |zc| left [2^-36, 2^60]; the caller then re-runs the
// block exactly.  Inside that range the core divisions are exact: 1/zc directly, and the numerator
// sdf = d - zc is 0 or >= 2^-60 in magnitude (zc >= 2^-36 => the difference is a multiple of
// 2^-60 or at least zc / 2), so the result is bit-identical to integrate_column<.., true>.
template <int ZPER, int G>
__device__ __forceinline__ bool integrate_column_pk(f2v (&T)[ZPER / 2], f2v (&Wt)[ZPER / 2],
                                                    uint32_t& dirty, bmask_t mask,
                                                    const f2v (&zs2)[ZPER / 2], float xs, float ys,
                                                    const float* __restrict__ depths, int64_t HW, int W,
                                                    float hm1, float wm1, const FrameParams* __restrict__ fps,
                                                    const int64_t* __restrict__ depth_frame, float depth_max,
                                                    float sdf_trunc) {
    const float y0t = __builtin_amdgcn_rcpf(sdf_trunc);
    const float y1t_s = __builtin_fmaf(__builtin_fmaf(-sdf_trunc, y0t, 1.0f), y0t, y0t);
    const f2v y1t = splat2(y1t_s), nbt = splat2(-sdf_trunc), one = splat2(1.0f);
    float zmin = 0x1p100f, zmax = 0.0f;
    bmask_t m = mask;
    while (m) {
        const int f = __builtin_ctzll(m);
        m &= m - 1;
        const FrameParams& fp = fps[f];
        const float* __restrict__ dep = depths + depth_frame[f] * HW;
        const f2v ax = splat2(xs * fp.ext[0] + ys * fp.ext[1]);
        const f2v ay = splat2(xs * fp.ext[4] + ys * fp.ext[5]);
        const f2v az = splat2(xs * fp.ext[8] + ys * fp.ext[9]);
        const f2v e2 = splat2(fp.ext[2]), e3 = splat2(fp.ext[3]), e6 = splat2(fp.ext[6]);
        const f2v e7 = splat2(fp.ext[7]), e10 = splat2(fp.ext[10]), e11 = splat2(fp.ext[11]);
        const f2v fx = splat2(fp.fx), fy = splat2(fp.fy), cx = splat2(fp.cx), cy = splat2(fp.cy);
#pragma unroll
        for (int g = 0; g < ZPER; g += G) {
            constexpr int GP = G / 2;
            int pix[G];
            bool in[G];
            f2v zc[GP];
#pragma unroll
            for (int q = 0; q < GP; ++q) {
                const f2v zz = zs2[g / 2 + q];
                const f2v xc = (ax + zz * e2) + e3;
                const f2v yc = (ay + zz * e6) + e7;
                zc[q] = (az + zz * e10) + e11;
                zmin = fminf(zmin, fminf(fabsf(zc[q].x), fabsf(zc[q].y)));
                zmax = fmaxf(zmax, fmaxf(fabsf(zc[q].x), fabsf(zc[q].y)));
                const f2v inv = rcp_core2(zc[q]);
                const f2v u = fx * xc * inv + cx;
                const f2v v = fy * yc * inv + cy;
#pragma unroll
                for (int e = 0; e < 2; ++e) {
                    const float ue = e ? u.y : u.x, ve = e ? v.y : v.x;
                    const bool ok = ve >= 0 && ue >= 0 && ve <= hm1 && ue <= wm1;
                    in[2 * q + e] = ok;
                    pix[2 * q + e] = (int)(ok ? ve : 0.f) * W + (int)(ok ? ue : 0.f);
                }
            }
            float dv[G];
#pragma unroll
            for (int j = 0; j < G; ++j) dv[j] = dep[pix[j]];
#pragma unroll
            for (int q = 0; q < GP; ++q) {
                const int qq = g / 2 + q;
                const f2v d = {dv[2 * q], dv[2 * q + 1]};
                const f2v sdf = d - zc[q];
                bool up[2];
                f2v s;
#pragma unroll
                for (int e = 0; e < 2; ++e) {
                    const float de = e ? d.y : d.x, ze = e ? zc[q].y : zc[q].x, se = e ? sdf.y : sdf.x;
                    up[e] = !(!in[2 * q + e] || de <= 0 || de > depth_max || ze <= 0 || se < -sdf_trunc);
                    s[e] = se < sdf_trunc ? se : sdf_trunc;
                }
                const f2v sn = div_const2(s, nbt, y1t);
                const f2v wp = Wt[qq] + one;
                const f2v nt = (Wt[qq] * T[qq] + sn) * rcp_core2(wp);
                T[qq].x = up[0] ? nt.x : T[qq].x;
                T[qq].y = up[1] ? nt.y : T[qq].y;
                Wt[qq].x = up[0] ? wp.x : Wt[qq].x;
                Wt[qq].y = up[1] ? wp.y : Wt[qq].y;
                dirty |= (up[0] ? 1u << (2 * qq) : 0u) | (up[1] ? 2u << (2 * qq) : 0u);
            }
        }
    }
    return !(zmin >= 0x1p-36f) || zmax > 0x1p60f;
}

// Packed-f32 integrate (R = 16 / 8, unit depth scale): fast pass with exact block re-run, exact
// pass directly for blocks whose weights are outside [0, 2^59] (imported volumes).
template <int R, int G, int NT = 256>
__global__ __launch_bounds__(NT) void k_integrate_pk(const int32_t* __restrict__ list,
                                                      const int* __restrict__ counters, int64_t list_cap, Table t,
                                                      float2* __restrict__ pool, float voxel_size,
                                                      const float* __restrict__ depths, int64_t HW, int H, int W,
                                                      const FrameParams* __restrict__ fps,
                                                      const int64_t* __restrict__ depth_frame, float depth_max,
                                                      float sdf_trunc) {
    constexpr int R2 = R * R;
    constexpr int R3 = R2 * R;
    constexpr int ZPER = R3 / NT;
    constexpr int NP = ZPER / 2;
    constexpr int ZSTEP = NT / R2;
    static_assert(R3 % NT == 0 && NT % R2 == 0, "NT must divide R^3 and be a multiple of R^2");
    static_assert(ZPER % G == 0 && G % 2 == 0, "group size must be even and divide the voxels per thread");
    const int64_t n = min((int64_t)counters[kListCount], list_cap);
    const float hm1 = (float)H - 1.0f, wm1 = (float)W - 1.0f;
    const int tid = threadIdx.x;
    const int xv = tid % R, yv = (tid / R) % R, z0 = tid / R2;
    for (int64_t i = blockIdx.x; i < n; i += gridDim.x) {
        const int32_t slot = list[i];
        const int buf = t.vals[slot];
        const bmask_t mask = readfirstlane_u64(t.mask[slot]);
        int xb, yb, zb;
        unpack_key(t.keys[slot], xb, yb, zb);
        if (buf >= 0) {
            float2* vox = pool + (int64_t)buf * R3;
            float2 tw[ZPER];
            float zs[ZPER];
            bool wbad = false;
#pragma unroll
            for (int k = 0; k < ZPER; ++k) {
                tw[k] = vox[k * NT + tid];
                zs[k] = (float)(zb * R + z0 + k * ZSTEP) * voxel_size;
                wbad |= !(tw[k].y >= 0.0f && tw[k].y <= 0x1p59f);
            }
            const float xs = (float)(xb * R + xv) * voxel_size;
            const float ys = (float)(yb * R + yv) * voxel_size;
            uint32_t dirty = 0;
            bool exact = __syncthreads_or(wbad);
            if (!exact) {
                f2v T[NP], Wt[NP], zs2[NP];
#pragma unroll
                for (int q = 0; q < NP; ++q) {
                    T[q] = f2v{tw[2 * q].x, tw[2 * q + 1].x};
                    Wt[q] = f2v{tw[2 * q].y, tw[2 * q + 1].y};
                    zs2[q] = f2v{zs[2 * q], zs[2 * q + 1]};
                }
                const bool zbad = integrate_column_pk<ZPER, G>(T, Wt, dirty, mask, zs2, xs, ys, depths, HW, W, hm1,
                                                            wm1, fps, depth_frame, depth_max, sdf_trunc);
                exact = __syncthreads_or(zbad);
                if (!exact) {
#pragma unroll
                    for (int q = 0; q < NP; ++q) {
                        tw[2 * q] = make_float2(T[q].x, Wt[q].x);
                        tw[2 * q + 1] = make_float2(T[q].y, Wt[q].y);
                    }
                } else {
#pragma unroll
                    for (int k = 0; k < ZPER; ++k) tw[k] = vox[k * NT + tid];
                    dirty = 0;
                }
            }
            if (exact)
                integrate_column<ZPER, G, true>(tw, dirty, mask, zs, xs, ys, depths, HW, W, hm1, wm1, fps,
                                                depth_frame, 1.0f, true, depth_max, sdf_trunc);
#pragma unroll
            for (int k = 0; k < ZPER; ++k)
                if (dirty & (1u << k)) vox[k * NT + tid] = tw[k];
        }
        __syncthreads();
        if (tid == 0) t.mask[slot] = 0;
    }
}

// ---- lean integrate (variants 40-47) -----------------------------------------------------------
// The exact kernel's arithmetic with (i) shortened reciprocals, (ii) gathers through a raw buffer
// view (out-of-image voxels read past its end, which returns 0), (iii) predicated updates instead
// of per-voxel branches and (iv) optionally the next frame's projections and gathers issued before
// the current frame's updates (PIPE), so a wave keeps ZPER gathers in flight across a whole frame
// of arithmetic.  Blocks whose operands leave the ranges below are handed to the exact fix-up
// launch unwritten (as the EXTFIX variants do).
//
// rcp_nm: v_rcp + one Newton step + one Markstein correction (5 VALU);
// rcp_m:  v_rcp + one Markstein correction (3 VALU).
// Both are compared with IEEE 1.0f / b over every float of the ranges they are used on
// (tests/test_gpu_numerics.py, mqr_check_division modes 3 / 4): 1 / zc for 2^-36 <= zc <= 2^60
// (rcp_nm, or rcp_m when RZ == 2) and 1 / (w + 1) for integer weights w <= 2^23 + 64 (rcp_m).
__device__ __forceinline__ float rcp_nm(float b) {
    const float y0 = __builtin_amdgcn_rcpf(b);
    const float y1 = __builtin_fmaf(__builtin_fmaf(-b, y0, 1.0f), y0, y0);
    return __builtin_fmaf(__builtin_fmaf(-b, y1, 1.0f), y1, y1);
}
__device__ __forceinline__ float rcp_m(float b) {
    const float y0 = __builtin_amdgcn_rcpf(b);
    return __builtin_fmaf(__builtin_fmaf(-b, y0, 1.0f), y0, y0);
}

// Raw buffer view of one depth frame: a load at or past `bytes` returns 0 instead of faulting.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t frame_rsrc(const float* base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0, (int)bytes, 0x00020000);
}

// (tsdf, weight) of a block through a buffer view: 32-bit offsets recomputed at the store, where
// plain pointers made the compiler keep a 64-bit address per voxel live across the frame loop.
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float2 pool_load(__amdgpu_buffer_rsrc_t rs, uint32_t voff, int soff) {
    const u32x2 r = __builtin_amdgcn_raw_buffer_load_b64(rs, voff, soff, 0);
    return make_float2(__uint_as_float(r.x), __uint_as_float(r.y));
}
__device__ __forceinline__ void pool_store(__amdgpu_buffer_rsrc_t rs, uint32_t voff, int soff, float2 v) {
    u32x2 r;
    r.x = __float_as_uint(v.x);
    r.y = __float_as_uint(v.y);
    __builtin_amdgcn_raw_buffer_store_b64(r, rs, voff, soff, 0);
}

// Projection and gather of one frame for a thread's column -- Open3D's transform and projection,
// the same float operations as integrate_column.  An out-of-image voxel gets row H, whose byte
// offset is >= 4HW, past the end of the frame (host: 4 (HW + W) <= 2^31, so the 24-bit multiply
// is exact): its depth reads as 0 and fails the update's d > 0 test, exactly like the out-of-image
// skip (an in-image
// NaN depth still reaches the update, as in Open3D).  `bad` is set unless 2^-36 <= zc <= 2^60 (zc
// <= 0 included, which the update would skip anyway): inside that range the reciprocal shortcut is
// exact and a non-zero sdf = d - zc is >= 2^-60 in magnitude, which keeps the division core exact.
template <int ZPER, int RZ>
__device__ __forceinline__ void lean_gather(float (&dv)[ZPER], bool& bad, const FrameParams& fp,
                                            __amdgpu_buffer_rsrc_t rs, const float (&xs)[ZPER],
                                            const float (&ys)[ZPER], const float (&zs)[ZPER], uint32_t W4, float hf,
                                            float hm1, float wm1) {
    // frame constants as values (the scheduling barriers below would otherwise force a reload of
    // every field per voxel and keep the partial products apart)
    float e[12];
#pragma unroll
    for (int j = 0; j < 12; ++j) e[j] = fp.ext[j];
    const float fx = fp.fx, fy = fp.fy, cx = fp.cx, cy = fp.cy;
#pragma unroll
    for (int k = 0; k < ZPER; ++k) {
        // z-independent partial products: one per thread in the column mapping (equal operands are
        // merged by the compiler), one per cube column in the cube mapping
        const float ax = xs[k] * e[0] + ys[k] * e[1];
        const float ay = xs[k] * e[4] + ys[k] * e[5];
        const float az = xs[k] * e[8] + ys[k] * e[9];
        const float xc = (ax + zs[k] * e[2]) + e[3];
        const float yc = (ay + zs[k] * e[6]) + e[7];
        const float zc = (az + zs[k] * e[10]) + e[11];
        bad |= (__float_as_uint(zc) - 0x2D800000u) > 0x30000000u;  // not 2^-36 <= zc <= 2^60
        const float inv_z = RZ == 2 ? rcp_m(zc) : rcp_nm(zc);
        const float u = fx * xc * inv_z + cx;
        const float v = fy * yc * inv_z + cy;
        const bool in = (v >= 0) & (u >= 0) & (v <= hm1) & (u <= wm1);
        const int ui = (int)(in ? u : 0.f), vi = (int)(in ? v : hf);
        const uint32_t off = __umul24((uint32_t)vi, W4) + ((uint32_t)ui << 2);
        dv[k] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0));
        // keep each voxel's projection next to its load: hoisting all projections above the loads
        // (the scheduler's choice) keeps ~6 more VGPRs per voxel live and halves the occupancy
        __builtin_amdgcn_sched_barrier(0);
    }
}

// Running-average update of one frame's gathered depths (zc recomputed by the same operations).
template <int ZPER>
__device__ __forceinline__ void lean_update(float2 (&tw)[ZPER], const float (&dv)[ZPER], const FrameParams& fp,
                                            const float (&xs)[ZPER], const float (&ys)[ZPER],
                                            const float (&zs)[ZPER], float depth_max, float sdf_trunc, float y1t) {
    const float e8 = fp.ext[8], e9 = fp.ext[9], e10 = fp.ext[10], e11 = fp.ext[11];
#pragma unroll
    for (int k = 0; k < ZPER; ++k) {
        const float az = xs[k] * e8 + ys[k] * e9;
        const float zc = (az + zs[k] * e10) + e11;
        const float d = dv[k];
        const float sdf = d - zc;
        // zc > 0 holds in every block that is not handed to the fix-up launch
        const bool up = !(d <= 0) && !(d > depth_max) && !(sdf < -sdf_trunc);
        const float s = sdf < sdf_trunc ? sdf : sdf_trunc;
        const float q0 = s * y1t;  // s / sdf_trunc: div_rn_core with the reciprocal refinement hoisted
        const float q1 = __builtin_fmaf(__builtin_fmaf(-sdf_trunc, q0, s), y1t, q0);
        const float sn = __builtin_fmaf(__builtin_fmaf(-sdf_trunc, q1, s), y1t, q1);
        const float wgt = tw[k].y, wp = wgt + 1;
        const float nt = (wgt * tw[k].x + sn) * rcp_m(wp);
        tw[k].x = up ? nt : tw[k].x;
        tw[k].y = up ? wp : wgt;
        __builtin_amdgcn_sched_barrier(0);  // one voxel's chain at a time (register pressure)
    }
}

// Voxel (x, y, z) of a block handled by thread `tid` as its k-th voxel.  COLUMN: the layout of
// k_integrate_t (thread = voxel column, a wave = a 16 x 4 slab of one z layer).  CUBE: a wave's 64
// lanes form a 4 x 4 x 4 voxel cube (lane bits x:0-1, y:2-3, z:4-5) and a thread's voxels walk the
// cubes of R/4-cube columns, so every gather instruction reads the projection of a compact cube --
// far fewer distinct cache lines than a slab, which is what bounds the gathers (L1 tag lookups).
template <int R, int NT, bool CUBE>
__device__ __forceinline__ void lean_voxel(int tid, int k, int& x, int& y, int& z) {
    constexpr int R2 = R * R, ZPER = R * R2 / NT;
    if (CUBE) {
        constexpr int C = R / 4, CPT = ZPER / C;  // cubes per axis, cube columns per thread
        static_assert(R % 4 == 0 && ZPER % C == 0 && (NT / 64) * CPT == C * C, "cube mapping does not tile");
        const int w = tid >> 6, l = tid & 63, cxy = w * CPT + k / C;
        x = 4 * (cxy % C) + (l & 3);
        y = 4 * (cxy / C) + ((l >> 2) & 3);
        z = 4 * (k % C) + (l >> 4);
    } else {
        x = tid % R;
        y = (tid / R) % R;
        z = tid / R2 + k * (NT / R2);
    }
}

// Lean integrate, unit depth scale only (host: sdf_trunc in the division core's range).  Block per
// workgroup as in k_integrate_t; every voxel of a block that is not handed off is written back.
template <int R, int NT, bool PIPE, int RZ, int WPE = 1, bool CUBE = false>
__global__ __launch_bounds__(NT, WPE) void k_integrate_lean(const int32_t* __restrict__ list,
                                                        const bmask_t* __restrict__ lmask,
                                                        int32_t* __restrict__ bad_out, int* __restrict__ counters,
                                                        int64_t list_cap, Table t, float2* __restrict__ pool,
                                                        float voxel_size, const float* __restrict__ depths,
                                                        int64_t HW, int H, int W,
                                                        const FrameParams* __restrict__ fps,
                                                        const int64_t* __restrict__ depth_frame, float depth_max,
                                                        float sdf_trunc) {
    constexpr int R2 = R * R;
    constexpr int R3 = R2 * R;
    constexpr int ZPER = R3 / NT;
    static_assert(R3 % NT == 0 && NT % R2 == 0, "NT must divide R^3 and be a multiple of R^2");
    const int64_t n = min((int64_t)counters[kListCount], list_cap);
    const float hf = (float)H, hm1 = (float)H - 1.0f, wm1 = (float)W - 1.0f;
    const uint32_t W4 = 4u * (uint32_t)W, bytes = 4u * (uint32_t)HW;
    const float y0t = __builtin_amdgcn_rcpf(sdf_trunc);
    const float y1t = __builtin_fmaf(__builtin_fmaf(-sdf_trunc, y0t, 1.0f), y0t, y0t);
    const int tid = threadIdx.x;
    for (int64_t i = blockIdx.x; i < n; i += gridDim.x) {
        const int32_t slot = list[i];
        const int buf = t.vals[slot];
        const bmask_t mask = readfirstlane_u64(lmask ? lmask[i] : t.mask[slot]);
        int xb, yb, zb;
        unpack_key(t.keys[slot], xb, yb, zb);
        if (buf >= 0 && mask) {
            const __amdgpu_buffer_rsrc_t vox = __builtin_amdgcn_make_buffer_rsrc(
                pool + (int64_t)buf * R3, (short)0, (int)(R3 * sizeof(float2)), 0x00020000);
            float2 tw[ZPER];
            float xs[ZPER], ys[ZPER], zs[ZPER];
            bool bad = false;
            // column mapping: one (x, y) per thread, shared by all its voxels (one value, not ZPER copies)
            const float xs0 = (float)(xb * R + tid % R) * voxel_size;
            const float ys0 = (float)(yb * R + (tid / R) % R) * voxel_size;
#pragma unroll
            for (int k = 0; k < ZPER; ++k) {
                int x, y, z;
                lean_voxel<R, NT, CUBE>(tid, k, x, y, z);
                // column mapping: voxel k * NT + tid, i.e. one VGPR offset and a constant per voxel
                tw[k] = CUBE ? pool_load(vox, 8u * (uint32_t)(z * R2 + y * R + x), 0)
                             : pool_load(vox, 8u * (uint32_t)tid, k * NT * (int)sizeof(float2));
                xs[k] = CUBE ? (float)(xb * R + x) * voxel_size : xs0;
                ys[k] = CUBE ? (float)(yb * R + y) * voxel_size : ys0;
                zs[k] = (float)(zb * R + z) * voxel_size;
                const float w = tw[k].y;  // rcp_m(w + 1) needs integer weights (a batch adds <= 64)
                bad |= !(w >= 0.0f && w <= 0x1p23f && w == __builtin_truncf(w));
            }
            bmask_t m = mask;
            int f = __builtin_ctzll(m);
            m &= m - 1;
            float da[ZPER], db[ZPER];
            lean_gather<ZPER, RZ>(da, bad, fps[f], frame_rsrc(depths + depth_frame[f] * HW, bytes), xs, ys, zs, W4,
                                  hf, hm1, wm1);
            // PIPE: the next frame's projections and gathers are issued before this frame's updates
            while (true) {
                const bool more = m != 0;  // wave-uniform
                const int g = more ? __builtin_ctzll(m) : 0;
                m &= m - 1;
                if (PIPE && more)
                    lean_gather<ZPER, RZ>(db, bad, fps[g], frame_rsrc(depths + depth_frame[g] * HW, bytes), xs, ys,
                                          zs, W4, hf, hm1, wm1);
                lean_update<ZPER>(tw, da, fps[f], xs, ys, zs, depth_max, sdf_trunc, y1t);
                if (!more) break;
                if (PIPE) {
#pragma unroll
                    for (int k = 0; k < ZPER; ++k) da[k] = db[k];
                } else {
                    lean_gather<ZPER, RZ>(da, bad, fps[g], frame_rsrc(depths + depth_frame[g] * HW, bytes), xs, ys,
                                          zs, W4, hf, hm1, wm1);
                }
                f = g;
            }
            if (__syncthreads_or(bad)) {  // block-uniform: the exact fix-up launch redoes it from the pool
                if (tid == 0) {
                    const int j = atomicAdd(&counters[kBadCount], 1);
                    bad_out[j] = slot;
                    reinterpret_cast<bmask_t*>(bad_out + list_cap)[j] = mask;
                }
            } else {
#pragma unroll
                for (int k = 0; k < ZPER; ++k) {
                    int x, y, z;
                    lean_voxel<R, NT, CUBE>(tid, k, x, y, z);
                    if (CUBE)
                        pool_store(vox, 8u * (uint32_t)(z * R2 + y * R + x), 0, tw[k]);
                    else
                        pool_store(vox, 8u * (uint32_t)tid, k * NT * (int)sizeof(float2), tw[k]);
                }
            }
        }
        __syncthreads();
        if (tid == 0) t.mask[slot] = 0;
    }
}

// ---- tiled lean integrate (variants 56-57) ------------------------------------------------------
// The lean kernel spends its time in the L1 (one tag lookup per distinct line per gather lane group:
// ~46 per 64-lane depth gather, rocprofv3 TCP_TOTAL_CACHE_ACCESSES).  Here the depth rectangle a
// block projects to is copied into LDS once per (block, frame) with row-coalesced loads and the
// voxel gathers read LDS.  The depth values are the same, so the result is the lean kernel's.
constexpr int kTilePx = 12288;  // 48 KiB of depth per workgroup

// Conservative pixel rectangle of block (xb, yb, zb)'s projection into one frame, computed by one
// whole wave: the 8 corner voxel centres are projected with the kernel's own operations (corner =
// lane & 7), padded by 2 px and clamped to the image.  Voxel centres inside the block project into
// the convex hull of the corners when every corner is in front of the camera (float rounding moves
// a projection by far less than the pad); a voxel that still falls outside reads global memory.
// rect = {u0, v0, width, height}; width 0 = no tile (a corner not in 2^-36 <= zc <= 2^60, a
// non-finite projection, or a rectangle larger than the tile).
__device__ __forceinline__ void block_rect(const FrameParams& fp, int xb, int yb, int zb, int R, float voxel_size,
                                           int H, int W, int (&rect)[4]) {
    const int c = threadIdx.x & 7;
    const float xs = (float)(xb * R + (c & 1) * (R - 1)) * voxel_size;
    const float ys = (float)(yb * R + ((c >> 1) & 1) * (R - 1)) * voxel_size;
    const float zs = (float)(zb * R + ((c >> 2) & 1) * (R - 1)) * voxel_size;
    const float xc = ((xs * fp.ext[0] + ys * fp.ext[1]) + zs * fp.ext[2]) + fp.ext[3];
    const float yc = ((xs * fp.ext[4] + ys * fp.ext[5]) + zs * fp.ext[6]) + fp.ext[7];
    const float zc = ((xs * fp.ext[8] + ys * fp.ext[9]) + zs * fp.ext[10]) + fp.ext[11];
    const float inv_z = rcp_m(zc);
    const float u = fp.fx * xc * inv_z + fp.cx;
    const float v = fp.fy * yc * inv_z + fp.cy;
    const bool ok = zc >= 0x1p-36f && zc <= 0x1p60f && fabsf(u) < 1e7f && fabsf(v) < 1e7f;
    float umin = u, umax = u, vmin = v, vmax = v;
#pragma unroll
    for (int o = 4; o >= 1; o >>= 1) {
        umin = fminf(umin, __shfl_xor(umin, o, 64));
        umax = fmaxf(umax, __shfl_xor(umax, o, 64));
        vmin = fminf(vmin, __shfl_xor(vmin, o, 64));
        vmax = fmaxf(vmax, __shfl_xor(vmax, o, 64));
    }
    const int u0 = max(0, (int)floorf(umin) - 2), u1 = min(W - 1, (int)floorf(umax) + 2);
    const int v0 = max(0, (int)floorf(vmin) - 2), v1 = min(H - 1, (int)floorf(vmax) + 2);
    const int tw = max(u1 - u0 + 1, 0), th = max(v1 - v0 + 1, 0);
    const bool use = __ballot(!ok) == 0 && tw * th <= kTilePx;
    rect[0] = u0;
    rect[1] = v0;
    rect[2] = use ? tw : 0;
    rect[3] = use ? th : 0;
}

// lean_gather with the depth read from the staged rectangle (global memory for an in-image voxel
// outside it, 0 for an out-of-image voxel).
template <int ZPER>
__device__ __forceinline__ void lean_gather_tile(float (&dv)[ZPER], bool& bad, const FrameParams& fp,
                                                 const float* __restrict__ dep, const float* tile, int u0, int v0,
                                                 int tlw, int tlh, const float (&xs)[ZPER], const float (&ys)[ZPER],
                                                 const float (&zs)[ZPER], int W, float hf, float hm1, float wm1) {
#pragma unroll
    for (int k = 0; k < ZPER; ++k) {
        const float ax = xs[k] * fp.ext[0] + ys[k] * fp.ext[1];
        const float ay = xs[k] * fp.ext[4] + ys[k] * fp.ext[5];
        const float az = xs[k] * fp.ext[8] + ys[k] * fp.ext[9];
        const float xc = (ax + zs[k] * fp.ext[2]) + fp.ext[3];
        const float yc = (ay + zs[k] * fp.ext[6]) + fp.ext[7];
        const float zc = (az + zs[k] * fp.ext[10]) + fp.ext[11];
        bad |= (__float_as_uint(zc) - 0x2D800000u) > 0x30000000u;  // not 2^-36 <= zc <= 2^60
        const float inv_z = rcp_m(zc);
        const float u = fp.fx * xc * inv_z + fp.cx;
        const float v = fp.fy * yc * inv_z + fp.cy;
        const bool in = (v >= 0) & (u >= 0) & (v <= hm1) & (u <= wm1);
        const int ui = (int)(in ? u : 0.f), vi = (int)(in ? v : hf);
        const uint32_t tu = (uint32_t)(ui - u0), tv = (uint32_t)(vi - v0);  // row H never lies in the tile
        float d = 0.f;
        if (tu < (uint32_t)tlw && tv < (uint32_t)tlh)
            d = tile[__umul24(tv, (uint32_t)tlw) + tu];
        else if (in)
            d = dep[vi * W + ui];
        dv[k] = d;
        __builtin_amdgcn_sched_barrier(0);
    }
}

// Tiled lean integrate (column mapping, RZ = 2; same preconditions and fix-up hand-off as the lean
// kernel).  Per (block, frame): wave 0 computes the rectangle, the workgroup copies it into LDS
// (one wave per row, lanes along the row), then every thread gathers and updates its voxels.
template <int R, int NT>
__global__ __launch_bounds__(NT) void k_integrate_tile(const int32_t* __restrict__ list,
                                                      const bmask_t* __restrict__ lmask,
                                                      int32_t* __restrict__ bad_out, int* __restrict__ counters,
                                                      int64_t list_cap, Table t, float2* __restrict__ pool,
                                                      float voxel_size, const float* __restrict__ depths, int64_t HW,
                                                      int H, int W, const FrameParams* __restrict__ fps,
                                                      const int64_t* __restrict__ depth_frame, float depth_max,
                                                      float sdf_trunc) {
    constexpr int R2 = R * R;
    constexpr int R3 = R2 * R;
    constexpr int ZPER = R3 / NT;
    constexpr int NW = NT / 64;
    static_assert(R3 % NT == 0 && NT % R2 == 0, "NT must divide R^3 and be a multiple of R^2");
    __shared__ float tile[kTilePx];
    __shared__ int s_rect[4];
    const int64_t n = min((int64_t)counters[kListCount], list_cap);
    const float hf = (float)H, hm1 = (float)H - 1.0f, wm1 = (float)W - 1.0f;
    const float y0t = __builtin_amdgcn_rcpf(sdf_trunc);
    const float y1t = __builtin_fmaf(__builtin_fmaf(-sdf_trunc, y0t, 1.0f), y0t, y0t);
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    for (int64_t i = blockIdx.x; i < n; i += gridDim.x) {
        const int32_t slot = list[i];
        const int buf = t.vals[slot];
        const bmask_t mask = readfirstlane_u64(lmask ? lmask[i] : t.mask[slot]);
        int xb, yb, zb;
        unpack_key(t.keys[slot], xb, yb, zb);
        if (buf >= 0 && mask) {
            const __amdgpu_buffer_rsrc_t vox = __builtin_amdgcn_make_buffer_rsrc(
                pool + (int64_t)buf * R3, (short)0, (int)(R3 * sizeof(float2)), 0x00020000);
            float2 tw[ZPER];
            float xs[ZPER], ys[ZPER], zs[ZPER];
            bool bad = false;
#pragma unroll
            for (int k = 0; k < ZPER; ++k) {
                int x, y, z;
                lean_voxel<R, NT, false>(tid, k, x, y, z);
                tw[k] = pool_load(vox, 8u * (uint32_t)(z * R2 + y * R + x), 0);
                xs[k] = (float)(xb * R + x) * voxel_size;
                ys[k] = (float)(yb * R + y) * voxel_size;
                zs[k] = (float)(zb * R + z) * voxel_size;
                const float w = tw[k].y;
                bad |= !(w >= 0.0f && w <= 0x1p23f && w == __builtin_truncf(w));
            }
            bmask_t m = mask;
            while (m) {
                const int f = __builtin_ctzll(m);
                m &= m - 1;
                const FrameParams& fp = fps[f];
                const float* __restrict__ dep = depths + depth_frame[f] * HW;
                if (wave == 0) {
                    int rect[4];
                    block_rect(fp, xb, yb, zb, R, voxel_size, H, W, rect);
                    if (lane < 4) s_rect[lane] = rect[lane];
                }
                __syncthreads();  // the rectangle is out, and every wave is done with the last tile
                const int u0 = __builtin_amdgcn_readfirstlane(s_rect[0]), v0 = __builtin_amdgcn_readfirstlane(s_rect[1]);
                const int tlw = __builtin_amdgcn_readfirstlane(s_rect[2]);
                const int tlh = __builtin_amdgcn_readfirstlane(s_rect[3]);
                for (int r = wave; r < tlh; r += NW) {
                    const float* src = dep + (int64_t)(v0 + r) * W + u0;
                    for (int c = lane; c < tlw; c += 64) tile[r * tlw + c] = src[c];
                }
                __syncthreads();
                float dv[ZPER];
                lean_gather_tile<ZPER>(dv, bad, fp, dep, tile, u0, v0, tlw, tlh, xs, ys, zs, W, hf, hm1, wm1);
                lean_update<ZPER>(tw, dv, fp, xs, ys, zs, depth_max, sdf_trunc, y1t);
            }
            if (__syncthreads_or(bad)) {  // block-uniform: the exact fix-up launch redoes it from the pool
                if (tid == 0) {
                    const int j = atomicAdd(&counters[kBadCount], 1);
                    bad_out[j] = slot;
                    reinterpret_cast<bmask_t*>(bad_out + list_cap)[j] = mask;
                }
            } else {
#pragma unroll
                for (int k = 0; k < ZPER; ++k) {
                    int x, y, z;
                    lean_voxel<R, NT, false>(tid, k, x, y, z);
                    pool_store(vox, 8u * (uint32_t)(z * R2 + y * R + x), 0, tw[k]);
                }
            }
        }
        __syncthreads();
        if (tid == 0) t.mask[slot] = 0;
    }
}

// ---- double-buffered tile integrate (variant 58) --------------------------------------------------
// The lean kernel is bound by the L1 path of its depth gathers: a scattered dword gather costs about
// one tag lookup per in-image lane (rocprofv3: ~43 TCP accesses and ~34 TA-busy cycles per gather
// instruction, TA busy ~80 % of the kernel).  Here the rectangle a block projects to (<= 64 x 64 px)
// is copied into LDS by async row loads (global_load_lds, one wave-instruction per row), the next
// frame's rectangle while the current frame is integrated, and the voxel gathers read LDS.  Same
// depth values and arithmetic as the lean kernel.  A frame whose rectangle does not fit (block close
// to the camera) or whose corners are not safely in front of the camera is gathered directly.
constexpr int kTileDim = 64;
typedef __attribute__((address_space(1))) void gvoid_t;
typedef __attribute__((address_space(3))) void lvoid_t;

// Rectangles of every frame of a block's batch mask in one pass of the workgroup (slot = thread / 8
// = rank of the frame in the mask, corner = thread % 8; NT >= 256): the 8 corner voxel centres are
// projected with the kernel's own operations, padded by 2 px and clamped to the image (voxel centres
// inside the block project into the hull of the corners when all corners are in front of the
// camera; rounding moves a projection far less than the pad, and a voxel found outside the
// rectangle sends the block to the exact fix-up launch).  {u0, v0, w, h}; w = -1: gather directly.
__device__ __forceinline__ void block_rects(const FrameParams* __restrict__ fps, bmask_t mask, int xb, int yb, int zb,
                                            int R, float voxel_size, int H, int W, int4* s_rect) {
    const int slot = threadIdx.x >> 3, c = threadIdx.x & 7;
    bmask_t m = mask;
    for (int q = 0; q < slot && m; ++q) m &= m - 1;
    const bool have = m != 0;
    const FrameParams& fp = fps[have ? __builtin_ctzll(m) : 0];
    const float xs = (float)(xb * R + (c & 1) * (R - 1)) * voxel_size;
    const float ys = (float)(yb * R + ((c >> 1) & 1) * (R - 1)) * voxel_size;
    const float zs = (float)(zb * R + ((c >> 2) & 1) * (R - 1)) * voxel_size;
    const float xc = ((xs * fp.ext[0] + ys * fp.ext[1]) + zs * fp.ext[2]) + fp.ext[3];
    const float yc = ((xs * fp.ext[4] + ys * fp.ext[5]) + zs * fp.ext[6]) + fp.ext[7];
    const float zc = ((xs * fp.ext[8] + ys * fp.ext[9]) + zs * fp.ext[10]) + fp.ext[11];
    const float inv_z = rcp_m(zc);
    const float u = fp.fx * xc * inv_z + fp.cx;
    const float v = fp.fy * yc * inv_z + fp.cy;
    int ok = zc >= 0x1p-36f && zc <= 0x1p60f && fabsf(u) < 1e7f && fabsf(v) < 1e7f;
    float umin = u, umax = u, vmin = v, vmax = v;
#pragma unroll
    for (int o = 4; o >= 1; o >>= 1) {
        umin = fminf(umin, __shfl_xor(umin, o, 64));
        umax = fmaxf(umax, __shfl_xor(umax, o, 64));
        vmin = fminf(vmin, __shfl_xor(vmin, o, 64));
        vmax = fmaxf(vmax, __shfl_xor(vmax, o, 64));
        ok &= __shfl_xor(ok, o, 64);
    }
    if (have && c == 0) {
        int4 r = make_int4(0, 0, -1, 0);
        if (ok) {
            const int u0 = max(0, (int)floorf(umin) - 2), u1 = min(W - 1, (int)floorf(umax) + 2);
            const int v0 = max(0, (int)floorf(vmin) - 2), v1 = min(H - 1, (int)floorf(vmax) + 2);
            const int w = u1 - u0 + 1, h = v1 - v0 + 1;
            if (w <= 0 || h <= 0)
                r = make_int4(0, 0, 0, 0);  // projection outside the image: nothing to stage
            else if (w <= kTileDim && h <= kTileDim)
                r = make_int4(u0, v0, w, h);
        }
        s_rect[slot] = r;
    }
}

// Async copy of a rectangle (w, h > 0, inside the image) into one LDS buffer of row pitch 64: one
// global_load_lds per row and wave (LDS destination = row base + lane * 4); lanes past the width
// re-read the last column.
__device__ __forceinline__ void tile_copy(const float* __restrict__ dep, int W, int4 r, float* buf, int nw) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int col = r.x + min(lane, r.z - 1);
    for (int row = wave; row < r.w; row += nw)
        __builtin_amdgcn_global_load_lds((gvoid_t*)(dep + (int64_t)(r.y + row) * W + col),
                                         (lvoid_t*)(buf + row * kTileDim), 4, 0, 0);
}

// lean_gather reading the staged rectangle; an in-image voxel outside it sets `bad`.
template <int ZPER>
__device__ __forceinline__ void tile_gather(float (&dv)[ZPER], bool& bad, const FrameParams& fp, const float* tile,
                                            int4 r, const float (&xs)[ZPER], const float (&ys)[ZPER],
                                            const float (&zs)[ZPER], float hm1, float wm1) {
    float e[12];
#pragma unroll
    for (int j = 0; j < 12; ++j) e[j] = fp.ext[j];
    const float fx = fp.fx, fy = fp.fy, cx = fp.cx, cy = fp.cy;
#pragma unroll
    for (int k = 0; k < ZPER; ++k) {
        const float ax = xs[k] * e[0] + ys[k] * e[1];
        const float ay = xs[k] * e[4] + ys[k] * e[5];
        const float az = xs[k] * e[8] + ys[k] * e[9];
        const float xc = (ax + zs[k] * e[2]) + e[3];
        const float yc = (ay + zs[k] * e[6]) + e[7];
        const float zc = (az + zs[k] * e[10]) + e[11];
        bad |= (__float_as_uint(zc) - 0x2D800000u) > 0x30000000u;  // not 2^-36 <= zc <= 2^60
        const float inv_z = rcp_m(zc);
        const float u = fx * xc * inv_z + cx;
        const float v = fy * yc * inv_z + cy;
        const bool in = (v >= 0) & (u >= 0) & (v <= hm1) & (u <= wm1);
        const int ui = (int)(in ? u : 0.f), vi = (int)(in ? v : 0.f);
        const uint32_t tu = (uint32_t)(ui - r.x), tv = (uint32_t)(vi - r.y);
        const bool hit = (tu < (uint32_t)r.z) & (tv < (uint32_t)r.w);
        bad |= in & !hit;
        const float t = tile[hit ? tv * kTileDim + tu : 0];
        dv[k] = (in & hit) ? t : 0.f;
        __builtin_amdgcn_sched_barrier(0);
    }
}

template <int R, int NT, int WPE = 1>
__global__ __launch_bounds__(NT, WPE) void k_integrate_dbt(const int32_t* __restrict__ list,
                                                     const bmask_t* __restrict__ lmask,
                                                     int32_t* __restrict__ bad_out, int* __restrict__ counters,
                                                     int64_t list_cap, Table t, float2* __restrict__ pool,
                                                     float voxel_size, const float* __restrict__ depths, int64_t HW,
                                                     int H, int W, const FrameParams* __restrict__ fps,
                                                     const int64_t* __restrict__ depth_frame, float depth_max,
                                                     float sdf_trunc) {
    constexpr int R2 = R * R;
    constexpr int R3 = R2 * R;
    constexpr int ZPER = R3 / NT;
    constexpr int NW = NT / 64;
    static_assert(R3 % NT == 0 && NT % R2 == 0 && NT >= 8 * kMaxBatch, "layout");
    __shared__ float tiles[2][kTileDim * kTileDim];
    __shared__ int4 s_rect[kMaxBatch];
    const int64_t n = min((int64_t)counters[kListCount], list_cap);
    const float hf = (float)H, hm1 = (float)H - 1.0f, wm1 = (float)W - 1.0f;
    const uint32_t W4 = 4u * (uint32_t)W, bytes = 4u * (uint32_t)HW;
    const float y0t = __builtin_amdgcn_rcpf(sdf_trunc);
    const float y1t = __builtin_fmaf(__builtin_fmaf(-sdf_trunc, y0t, 1.0f), y0t, y0t);
    const int tid = threadIdx.x;
    for (int64_t i = blockIdx.x; i < n; i += gridDim.x) {
        const int32_t slot = list[i];
        const int buf = t.vals[slot];
        const bmask_t mask = readfirstlane_u64(lmask ? lmask[i] : t.mask[slot]);
        int xb, yb, zb;
        unpack_key(t.keys[slot], xb, yb, zb);
        if (buf >= 0 && mask) {
            const __amdgpu_buffer_rsrc_t vox = __builtin_amdgcn_make_buffer_rsrc(
                pool + (int64_t)buf * R3, (short)0, (int)(R3 * sizeof(float2)), 0x00020000);
            float2 tw[ZPER];
            float xs[ZPER], ys[ZPER], zs[ZPER];
            bool bad = false;
            const float xs0 = (float)(xb * R + tid % R) * voxel_size;
            const float ys0 = (float)(yb * R + (tid / R) % R) * voxel_size;
#pragma unroll
            for (int k = 0; k < ZPER; ++k) {
                tw[k] = pool_load(vox, 8u * (uint32_t)tid, k * NT * (int)sizeof(float2));
                xs[k] = xs0;
                ys[k] = ys0;
                zs[k] = (float)(zb * R + tid / R2 + k * (NT / R2)) * voxel_size;
                const float w = tw[k].y;
                bad |= !(w >= 0.0f && w <= 0x1p23f && w == __builtin_truncf(w));
            }
            block_rects(fps, mask, xb, yb, zb, R, voxel_size, H, W, s_rect);
            __syncthreads();
            bmask_t m = mask;
            int f = __builtin_ctzll(m);
            m &= m - 1;
            int j = 0;
            int4 r = s_rect[0];
            r = make_int4(__builtin_amdgcn_readfirstlane(r.x), __builtin_amdgcn_readfirstlane(r.y),
                          __builtin_amdgcn_readfirstlane(r.z), __builtin_amdgcn_readfirstlane(r.w));
            if (r.z > 0 && r.w > 0) tile_copy(depths + depth_frame[f] * HW, W, r, tiles[0], NW);
            __syncthreads();  // waits for the copy (vmcnt) as well
            while (true) {
                const bool more = m != 0;  // wave-uniform
                const int g = more ? __builtin_ctzll(m) : 0;
                m &= m - 1;
                int4 rn = make_int4(0, 0, 0, 0);
                if (more) {
                    rn = s_rect[j + 1];
                    rn = make_int4(__builtin_amdgcn_readfirstlane(rn.x), __builtin_amdgcn_readfirstlane(rn.y),
                                   __builtin_amdgcn_readfirstlane(rn.z), __builtin_amdgcn_readfirstlane(rn.w));
                    if (rn.z > 0 && rn.w > 0) tile_copy(depths + depth_frame[g] * HW, W, rn, tiles[(j + 1) & 1], NW);
                }
                float dv[ZPER];
                if (r.z >= 0)
                    tile_gather<ZPER>(dv, bad, fps[f], tiles[j & 1], r, xs, ys, zs, hm1, wm1);
                else
                    lean_gather<ZPER, 2>(dv, bad, fps[f], frame_rsrc(depths + depth_frame[f] * HW, bytes), xs, ys, zs,
                                         W4, hf, hm1, wm1);
                lean_update<ZPER>(tw, dv, fps[f], xs, ys, zs, depth_max, sdf_trunc, y1t);
                if (!more) break;
                __syncthreads();  // the next rectangle has landed, this one is free
                f = g;
                r = rn;
                ++j;
            }
            if (__syncthreads_or(bad)) {
                if (tid == 0) {
                    const int jj = atomicAdd(&counters[kBadCount], 1);
                    bad_out[jj] = slot;
                    reinterpret_cast<bmask_t*>(bad_out + list_cap)[jj] = mask;
                }
            } else {
#pragma unroll
                for (int k = 0; k < ZPER; ++k) pool_store(vox, 8u * (uint32_t)tid, k * NT * (int)sizeof(float2), tw[k]);
            }
        }
        __syncthreads();
        if (tid == 0) t.mask[slot] = 0;
    }
}

// Exhaustive-check kernels for the division shortcut (tests/test_gpu_numerics.py).
// mode 0: rcp_rn, 1: rcp_nm, 2: rcp_m.
__global__ void k_check_rcp(int mode, uint32_t lo_bits, uint64_t count, uint32_t* mismatches, uint32_t* first_bad) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    const uint32_t bits = lo_bits + (uint32_t)i;
    const float b = __uint_as_float(bits);
    const float fast = mode == 1 ? rcp_nm(b) : mode == 2 ? rcp_m(b) : rcp_rn(b), ref = 1.0f / b;
    if (__float_as_uint(fast) != __float_as_uint(ref)) {
        atomicAdd(mismatches, 1u);
        atomicMin(first_bad, bits);
    }
}

__global__ void k_check_div(int which_core, float b, uint32_t lo_bits, uint64_t count, uint32_t* mismatches, uint32_t* first_bad) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    const uint32_t bits = lo_bits + (uint32_t)i;
    const float a = __uint_as_float(bits);
    const float fast = which_core ? div_rn_core(a, b) : div_rn(a, b), ref = a / b;
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

__global__ void k_set_counter(int* ctr, int value) { *ctr = value; }

__global__ void k_fixup_alloc(Table t, int* counters, int* pool_ctr, int64_t pool_cap, uint64_t* bkeys) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= t.cap) return;
    if (t.keys[i] == kEmpty || t.vals[i] != -2) return;
    const int b = atomicAdd(pool_ctr, 1);
    if (b < pool_cap) {
        t.vals[i] = b;
        bkeys[b] = t.keys[i];
    } else {
        atomicOr(&counters[kOverflow], 1);
    }
}

// Undo the allocations of a batch that failed (a frame touched no block): every key whose buffer
// index is >= `first_buf` was inserted by that batch.  Keys inserted earlier never probe through a
// slot claimed later (linear probing), so removing exactly the later keys keeps every remaining
// probe chain intact.  Their pool buffers were never integrated and are still zero.
__global__ void k_rollback(Table t, int first_buf) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= t.cap) return;
    if (t.keys[i] == kEmpty) return;
    const int b = t.vals[i];
    if (b >= first_buf || b == -2) {
        t.keys[i] = kEmpty;
        t.vals[i] = -1;
        t.mask[i] = 0;
    }
}

// Insert packed keys with buffer index = position (an empty volume filled in a chosen order: the
// multi-GPU merge places owned blocks first).  Keys are distinct.
__global__ void k_activate_ordered(const uint64_t* __restrict__ keys, int64_t n, Table t, uint64_t* bkeys,
                                   int* counters) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t k = keys[i];
    const uint64_t m = (uint64_t)t.cap - 1;
    uint64_t h = mix64(k) & m;
    for (int64_t p = 0; p < t.cap; ++p) {
        const uint64_t old = atomicCAS((unsigned long long*)&t.keys[h], (unsigned long long)kEmpty,
                                       (unsigned long long)k);
        if (old == kEmpty) {
            t.vals[h] = (int32_t)i;
            bkeys[i] = k;
            return;
        }
        h = (h + 1) & m;
    }
    atomicOr(&counters[kOverflow], 2);
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

}  // namespace mqr

// vbg_kernels.hpp -- device code of the TSDF volume (included once, by vbg.hip).
// Open3D 0.19 VoxelBlockGrid semantics; float32 with no FMA contraction.
#pragma once
#ifndef MQR_DIAG
#define MQR_DIAG 0  // 1 / 2: timing-only builds of the lean kernel, 3 / 4 / 5 of the tile kernels (wrong results; never shipped)
#endif
#ifndef MQR_AB
#define MQR_AB 0  // 1: the A/B kernels of vbg_ab.hpp (tools/_ab/libmqr_ab.so only)
#endif
#include <climits>

#include "mqr_common.hpp"

namespace mqr {

// ------------------------------------------------------------------ device helpers
__device__ __forceinline__ uint64_t readfirstlane_u64(uint64_t v) {
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return (uint64_t)hi << 32 | lo;
}
__device__ __forceinline__ bmask_t readfirstlane_mask(bmask_t v) {
    return (bmask_t)readfirstlane_u64((uint64_t)(v >> 64)) << 64 | readfirstlane_u64((uint64_t)v);
}

// Frame bit f of a slot mask, word by word: returns the old value of f's word.  `first` when the slot
// joins the batch list here: its word was empty and this mark won the listed flag (word 1, bit 63).
__device__ __forceinline__ unsigned long long mask_set_frame(bmask_t* m, int f, bool& first) {
    unsigned long long* w = reinterpret_cast<unsigned long long*>(m);
    const unsigned long long bit = 1ull << (f & 63);
    const unsigned long long old = atomicOr(&w[f >> 6], bit);
    first = false;
    if (old == 0 || (f >> 6 == 1 && old == kListedBit))  // the word held no frame bit yet
        first = !(atomicOr(&w[1], kListedBit) & kListedBit);
    return old;
}
__device__ __forceinline__ bool mask_has_frame(const bmask_t* m, int f) {
    const unsigned long long* w = reinterpret_cast<const unsigned long long*>(m);
    return (__hip_atomic_load(&w[f >> 6], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> (f & 63)) & 1;
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
    // every workgroup of a frame that sees the block marks it: read the word at L2 first and only
    // the workgroups that still find the bit clear issue the (same-address, serialised) atomic
    if (mask_has_frame(&t.mask[slot], f)) return false;
    bool first;
    const unsigned long long old = mask_set_frame(&t.mask[slot], f, first);
    if (first) {
        const int pos = atomicAdd(&counters[kListCount], 1);
        if (pos < list_cap)
            list[pos] = (int32_t)slot;
        else
            atomicOr(&counters[kOverflow], 4);
    }
    return !((old >> (f & 63)) & 1);
}

// ---- wave-aggregated table updates of k_touch (call with the whole wave converged) ----------------
// Same-address device atomics serialise (a few ns each at the home agent): per-lane list appends and
// pool allocations of a batch's ~3 000 new blocks, one per workgroup on a shared counter, cost tens
// of microseconds of the touch launch.  One atomic per wave per counter instead.

// Insert-or-find without allocation: `won` is set for the lane whose CAS created the entry.  A key
// that finds no free slot within `max_probe` slots sets the table-full bit (the host then undoes the
// batch's touch, grows the table to the worst case and touches again with max_probe = cap).
__device__ inline int64_t table_claim(Table t, uint64_t k, int* counters, bool& won, int64_t max_probe) {
    const uint64_t m = (uint64_t)t.cap - 1;
    uint64_t h = mix64(k) & m;
    for (int64_t p = 0; p < max_probe; ++p) {
        const uint64_t cur = t.keys[h];
        if (cur == k) return (int64_t)h;
        if (cur == kEmpty) {
            const uint64_t old = atomicCAS((unsigned long long*)&t.keys[h], (unsigned long long)kEmpty,
                                           (unsigned long long)k);
            if (old == kEmpty) {
                won = true;
                return (int64_t)h;
            }
            if (old == k) return (int64_t)h;
        }
        h = (h + 1) & m;
    }
    atomicOr(&counters[kOverflow], 2);
    return -1;
}

// Rank of this lane among the lanes of mask m below it, and the base one lane reserved for all of
// them with a single atomicAdd(ctr, popcount(m)).
__device__ inline int wave_reserve(uint64_t m, int* ctr) {
    const int lane = threadIdx.x & 63, leader = __builtin_ctzll(m);
    int base = 0;
    if (lane == leader) base = atomicAdd(ctr, __popcll(m));
    base = __shfl(base, leader, 64);
    return base + __popcll(m & ((1ull << lane) - 1));
}

// Pool buffers for the entries this wave's lanes created (won).
__device__ inline void wave_alloc(bool won, int64_t slot, uint64_t k, Table t, int* counters, int* pool_ctr,
                                  int64_t pool_cap, uint64_t* bkeys) {
    const uint64_t m = __ballot(won);
    if (!m) return;  // wave-uniform
    const int b = wave_reserve(m, pool_ctr);
    if (won) {
        if (b < pool_cap) {
            t.vals[slot] = b;
            bkeys[b] = k;
        } else {
            t.vals[slot] = -2;
            atomicOr(&counters[kOverflow], 1);
        }
    }
}

// Frame bit f of the slot; `first` when the slot's batch mask was empty (the slot joins the list).
__device__ inline bool mark_slot_bit(Table t, int64_t slot, int f, bool& first) {
    if (mask_has_frame(&t.mask[slot], f)) return false;
    const unsigned long long old = mask_set_frame(&t.mask[slot], f, first);
    return !((old >> (f & 63)) & 1);
}

// Batch-list appends of this wave's first-marked slots.
__device__ inline void wave_append(bool app, int64_t slot, int* counters, int32_t* list, int64_t list_cap) {
    const uint64_t m = __ballot(app);
    if (!m) return;  // wave-uniform
    const int pos = wave_reserve(m, &counters[kListCount]);
    if (app) {
        if (pos < list_cap)
            list[pos] = (int32_t)slot;
        else
            atomicOr(&counters[kOverflow], 4);
    }
}

// Sum of a per-lane count over the wave, added to *ctr by one lane (an LDS word of the workgroup
// here; per-thread global atomics on the batch counters serialised on a handful of addresses).
__device__ inline void wave_add(int* ctr, int v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(ctr, v);
}

// ------------------------------------------------------------------ kernels
// compute_unique_block_coordinates for a batch: blockIdx.y = batch frame (bit), PPT stride-4 pixels
// per thread (a workgroup covers 256 PPT consecutive ones), 4 samples each over
// [max(d - trunc, 0), min(d + trunc, depth_max)] (Appendix A.2).
template <int PPT>
__global__ __launch_bounds__(256) void k_touch(const float* __restrict__ depths, int64_t HW, int H, int W,
                                               const FrameParams* __restrict__ fps,
                                               const int64_t* __restrict__ depth_frame, float depth_scale,
                                               float depth_max, float sdf_trunc, float block_size, Table t,
                                               int64_t max_probe, int alloc, int* counters, int* pool_ctr,
                                               int64_t pool_cap, uint64_t* bkeys, int32_t* list, int64_t list_cap) {
    // keys already inserted by this workgroup (a strip of one frame shares most of its blocks): only
    // a key's first occurrence probes the global table and sets the frame bit.  The first
    // occurrences are collected in LDS and then claimed all at once, one per thread: each claim is a
    // chain of device-coherent round trips (probe, mask read, atomicOr, list append; ~2 200 cycles
    // per L2 read in this kernel), and claiming per sample left four such chains in sequence.  With
    // PPT > 1 a workgroup covers a longer strip: the touch is latency-bound and holds its wave slots
    // (taken from the overlapped integrate) for about one claim round, so fewer, longer-lived
    // workgroups with better deduplication hold fewer slot-microseconds.
    constexpr int kSeen = 1024 * PPT;  // >= the 4 x 256 x PPT keys a workgroup can produce: never full
    __shared__ unsigned long long seen[kSeen];
    __shared__ uint16_t uniq[kSeen];  // seen-slots of the first occurrences (LDS: workgroups per CU)
    __shared__ int wg_count[3];  // valid samples, new frame bits (one global atomic each), first keys
    for (int i = threadIdx.x; i < kSeen; i += blockDim.x) seen[i] = kEmpty;
    if (threadIdx.x < 3) wg_count[threadIdx.x] = 0;
    __syncthreads();
    const int f = blockIdx.y;
    const FrameParams& fp = fps[f];
    const int cols = W / 4, rows = H / 4, n = rows * cols;
    const float* __restrict__ dep = depths + depth_frame[f] * HW;
    int wpx[PPT];
    float dd[PPT];
#pragma unroll
    for (int jp = 0; jp < PPT; ++jp) {  // all of the thread's depth reads in flight together
        const int w = (blockIdx.x * PPT + jp) * blockDim.x + threadIdx.x;
        wpx[jp] = w;
        dd[jp] = w < n ? dep[(int64_t)((w / cols) * 4) * W + (w % cols) * 4] : 0.f;
    }
    int valid = 0, fresh = 0;
#pragma unroll
    for (int jp = 0; jp < PPT; ++jp) {
        const int w = wpx[jp];
        uint64_t key[4] = {kEmpty, kEmpty, kEmpty, kEmpty};
        if (w < n) {
            const int y = (w / cols) * 4, x = (w % cols) * 4;
            const float d = dd[jp] / depth_scale;
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
                valid += 4;
            }
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const uint64_t k = key[s];
            if (k == kEmpty || (s > 0 && key[s - 1] == k)) continue;
            uint32_t h = (uint32_t)mix64(k) & (kSeen - 1);
            bool first = false;
            for (;;) {  // terminates: the set has room for every key of the workgroup
                const unsigned long long old = atomicCAS(&seen[h], (unsigned long long)kEmpty, (unsigned long long)k);
                first = old == kEmpty;
                if (old == kEmpty || old == k) break;
                h = (h + 1) & (kSeen - 1);
            }
            if (first) uniq[atomicAdd(&wg_count[2], 1)] = (uint16_t)h;
        }
    }
    wave_add(&wg_count[0], valid);
    __syncthreads();
    const int nu = wg_count[2];
    for (int base = 0; base < nu; base += blockDim.x) {  // uniform trip count: the wave_* calls need whole waves
        const int idx = base + (int)threadIdx.x;
        const uint64_t k = idx < nu ? seen[uniq[idx]] : kEmpty;
        int64_t slot = -1;
        bool won = false, app = false;
        if (k != kEmpty) slot = table_claim(t, k, counters, won, max_probe);
        if (alloc) wave_alloc(won, slot, k, t, counters, pool_ctr, pool_cap, bkeys);
        if (slot >= 0) fresh += mark_slot_bit(t, slot, f, app);
        wave_append(app, slot, counters, list, list_cap);
    }
    wave_add(&wg_count[1], fresh);
    __syncthreads();
    if (threadIdx.x == 0) {
        if (wg_count[0]) atomicAdd(&counters[kFrameCounterBase + f], wg_count[0]);
        if (wg_count[1]) atomicAdd(&counters[kFreshBase + f], wg_count[1]);  // spread: one word per frame
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
    if (slot >= 0 && mark && mark_slot(t, slot, 0, counters, list, list_cap)) atomicAdd(&counters[kFreshBase], 1);
}

// Projective TSDF update of every voxel of every listed block, frames applied in bit order.
// Arithmetic = Open3D 0.19 Integrate kernel (Appendix A.3), float32, no contraction.
__global__ __launch_bounds__(256) void k_integrate(const int32_t* __restrict__ list, const int* __restrict__ counters,
                                                   int64_t list_cap, Table t, float2* __restrict__ pool, int R,
                                                   float voxel_size, const float* __restrict__ depths, int64_t HW,
                                                   int H, int W, const FrameParams* __restrict__ fps,
                                                   const int64_t* __restrict__ depth_frame, float depth_scale,
                                                   float depth_max, float sdf_trunc, int first_new) {
    const int64_t n = min((int64_t)counters[kListCount], list_cap);
    const int R3 = R * R * R;
    const float hm1 = (float)H - 1.0f, wm1 = (float)W - 1.0f;
    for (int64_t i = blockIdx.x; i < n; i += gridDim.x) {
        const int32_t slot = list[i];
        const int buf = t.vals[slot];
        const bmask_t mask = bm_frames(t.mask[slot]);
        int xb, yb, zb;
        unpack_key(t.keys[slot], xb, yb, zb);
        if (buf >= 0) {
            float2* vox = pool + (int64_t)buf * R3;
            for (int p = threadIdx.x; p < R3; p += blockDim.x) {
                const int xv = p % R, yv = (p / R) % R, zv = p / (R * R);
                const float xs = (float)(xb * R + xv) * voxel_size;
                const float ys = (float)(yb * R + yv) * voxel_size;
                const float zs = (float)(zb * R + zv) * voxel_size;
                const bool fresh = buf >= first_new;  // allocated by this batch: starts at (0, 0)
                float2 tw = fresh ? make_float2(0.f, 0.f) : vox[p];
                bool dirty = fresh;
                bmask_t m = mask;
                while (m) {
                    const int f = bm_ctz(m);
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
// Exact integrate, R known at compile time (R = 16 / 8): thread t owns the voxel column (x, y) =
// (t % R, t / R % R) for z in its z-range, keeps those voxels' (tsdf, weight) in registers for
// all frames of the batch, and evaluates Open3D's transform ((xs*e0 + ys*e1) + zs*e2) + e3 with
// the z-independent partial product hoisted per frame -- the same float operations in the same
// order as k_integrate, so the result is bit-identical.  Groups of G voxels issue their depth
// gathers together.  The fallback kernel (depth_scale != 1, trunc or frame size outside the fast
// kernels' preconditions) and the exact fix-up launch behind the fast kernels (over the blocks
// they handed back through bad_out; lmask = those blocks' batch masks).
template <int ZPER, int G>
__device__ __forceinline__ void integrate_column(float2 (&tw)[ZPER], uint32_t& dirty, bmask_t mask,
                                                 const float (&zs)[ZPER], float xs, float ys,
                                                 const float* __restrict__ depths, int64_t HW, int W, float hm1,
                                                 float wm1, const FrameParams* __restrict__ fps,
                                                 const int64_t* __restrict__ depth_frame, float depth_scale,
                                                 bool unit_scale, float depth_max, float sdf_trunc) {
    bmask_t m = mask;
    while (m) {
        const int f = bm_ctz(m);
        m &= m - 1;
        const FrameParams& fp = fps[f];
        const float* __restrict__ dep = depths + depth_frame[f] * HW;
        const float ax = xs * fp.ext[0] + ys * fp.ext[1];
        const float ay = xs * fp.ext[4] + ys * fp.ext[5];
        const float az = xs * fp.ext[8] + ys * fp.ext[9];
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
                const float wgt = tw[k].y;
                sdf = div_rn(sdf, sdf_trunc);
                const float inv_wsum = rcp_rn(wgt + 1);
                tw[k].x = (wgt * tw[k].x + sdf) * inv_wsum;
                tw[k].y = wgt + 1;
                dirty |= 1u << k;
            }
        }
    }
}

// One block, exact arithmetic (k_integrate_t's body; also the in-kernel fallback of the lean
// kernel): thread tid owns column (tid % R, tid / R % R), voxels z = tid / R^2 + k NT / R^2.
template <int R, int G, int NT>
__device__ __forceinline__ void exact_block(float2* __restrict__ vox, bool fresh, bmask_t mask, int xb, int yb, int zb,
                                            int tid, float voxel_size, const float* __restrict__ depths, int64_t HW,
                                            int W, float hm1, float wm1, const FrameParams* __restrict__ fps,
                                            const int64_t* __restrict__ depth_frame, float depth_scale,
                                            float depth_max, float sdf_trunc) {
    constexpr int R2 = R * R;
    constexpr int ZPER = R2 * R / NT;  // voxels per thread
    constexpr int ZSTEP = NT / R2;     // z stride between a thread's voxels
    const int xv = tid % R, yv = (tid / R) % R, z0 = tid / R2;
    float2 tw[ZPER];
    float zs[ZPER];
#pragma unroll
    for (int k = 0; k < ZPER; ++k) {
        tw[k] = fresh ? make_float2(0.f, 0.f) : vox[k * NT + tid];
        zs[k] = (float)(zb * R + z0 + k * ZSTEP) * voxel_size;
    }
    const float xs = (float)(xb * R + xv) * voxel_size;
    const float ys = (float)(yb * R + yv) * voxel_size;
    uint32_t dirty = fresh ? 0xffffffffu : 0u;  // a fresh block is written whole
    integrate_column<ZPER, G>(tw, dirty, mask, zs, xs, ys, depths, HW, W, hm1, wm1, fps, depth_frame, depth_scale,
                              depth_scale == 1.0f, depth_max, sdf_trunc);
#pragma unroll
    for (int k = 0; k < ZPER; ++k)
        if (dirty & (1u << k)) vox[k * NT + tid] = tw[k];
}

template <int R, int NT>
__device__ __attribute__((noinline)) void exact_block_call(float2* __restrict__ vox, bool fresh, bmask_t mask, int xb,
                                                           int yb, int zb, float voxel_size,
                                                           const float* __restrict__ depths, int64_t HW, int W,
                                                           float hm1, float wm1, const FrameParams* __restrict__ fps,
                                                           const int64_t* __restrict__ depth_frame, float depth_max,
                                                           float sdf_trunc) {
    exact_block<R, 4, NT>(vox, fresh, mask, xb, yb, zb, (int)threadIdx.x, voxel_size, depths, HW, W, hm1, wm1, fps,
                          depth_frame, 1.0f, depth_max, sdf_trunc);
}

template <int R, int G, int NT>
__global__ __launch_bounds__(NT) void k_integrate_t(const int32_t* __restrict__ list, const bmask_t* __restrict__ lmask,
                                                    const int* __restrict__ count, int64_t list_cap, Table t,
                                                    float2* __restrict__ pool, float voxel_size,
                                                    const float* __restrict__ depths, int64_t HW, int H, int W,
                                                    const FrameParams* __restrict__ fps,
                                                    const int64_t* __restrict__ depth_frame, float depth_scale,
                                                    float depth_max, float sdf_trunc, int first_new) {
    constexpr int R2 = R * R;
    constexpr int R3 = R2 * R;
    static_assert(R3 % NT == 0 && NT % R2 == 0, "NT must divide R^3 and be a multiple of R^2");
    static_assert((R3 / NT) % G == 0, "group size must divide the voxels per thread");
    const int64_t n = min((int64_t)*count, list_cap);
    const float hm1 = (float)H - 1.0f, wm1 = (float)W - 1.0f;
    const int tid = threadIdx.x;
    for (int64_t i = blockIdx.x; i < n; i += gridDim.x) {
        const int32_t slot = list[i];
        const int buf = t.vals[slot];
        const bmask_t mask = readfirstlane_mask(lmask ? lmask[i] : bm_frames(t.mask[slot]));
        int xb, yb, zb;
        unpack_key(t.keys[slot], xb, yb, zb);
        if (buf >= 0)
            exact_block<R, G, NT>(pool + (int64_t)buf * R3, buf >= first_new, mask, xb, yb, zb, tid, voxel_size,
                                  depths, HW, W, hm1, wm1, fps, depth_frame, depth_scale, depth_max, sdf_trunc);
        __syncthreads();
        if (tid == 0) t.mask[slot] = 0;
    }
}

// Longest-processing-time order of a batch list: counting sort by the number of the batch's frames
// that touched each block (popcount of its slot mask), descending.  The integrate grid then ends on
// short blocks instead of whichever long blocks the touch order happened to put last.  One
// workgroup; order within a bin is arbitrary (blocks are independent, results unchanged).
// shadow (nullable): k_gate's work for a speculative integrate of the batch's `nframes` frames, done
// here -- the kernel runs right behind the touch anyway -- so the integrate needs no gate launch.
__device__ __forceinline__ void gate_counters(const int* __restrict__ ctr, int* __restrict__ shadow, bool stop) {
    for (int i = threadIdx.x; i < kCountersTotal; i += blockDim.x)
        shadow[i] = i == kListCount ? (stop ? 0 : ctr[kListCount]) : i == kBadCount ? 0 : ctr[i];
}

__global__ __launch_bounds__(1024) void k_lpt_order(const int32_t* __restrict__ list, const int* __restrict__ counters,
                                                    int64_t list_cap, const bmask_t* __restrict__ mask,
                                                    int32_t* __restrict__ out, bmask_t* __restrict__ out_mask,
                                                    int* __restrict__ shadow = nullptr, int nframes = 0) {
    __shared__ int hist[kMaxBatch + 1];
    const int n = (int)min((int64_t)counters[kListCount], list_cap);
    if (threadIdx.x <= kMaxBatch) hist[threadIdx.x] = 0;
    if (shadow) {
        const bool empty = (int)threadIdx.x < nframes && counters[kFrameCounterBase + threadIdx.x] == 0;
        gate_counters(counters, shadow, __syncthreads_or(empty) != 0 || counters[kOverflow] != 0);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += blockDim.x) atomicAdd(&hist[bm_popc(bm_frames(mask[list[i]]))], 1);
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
        const bmask_t m = bm_frames(mask[s]);
        const int pos = atomicAdd(&hist[bm_popc(m)], 1);
        out[pos] = s;
        out_mask[pos] = m;
    }
}

// ---- lean integrate ------------------------------------------------------------------------------
// The exact kernel's arithmetic with (i) shortened reciprocals, (ii) gathers through a raw buffer
// view (out-of-image voxels read past its end, which returns 0), (iii) predicated updates instead
// of per-voxel branches.  Blocks whose operands leave the ranges below are handed to the exact
// fix-up launch unwritten.
//
// rcp_m:  v_rcp + one Markstein correction (3 VALU);  rcp_nm: v_rcp + one Newton step + one
// Markstein correction (5 VALU).  Both are compared with IEEE 1.0f / b over every float of the
// ranges they are used on (tests/test_gpu_numerics.py, mqr_check_division modes 3 / 4): rcp_m for
// 1 / zc, 2^-60 <= zc <= 2^60, and 1 / (w + 1) for integer weights w <= 2^23 + 64.
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

// Projection and gather of one frame for a thread's voxels -- Open3D's transform and projection,
// the same float operations as integrate_column.  An out-of-image voxel gets row H, whose byte
// offset is >= 4HW, past the end of the frame (host: 4 (HW + W) <= 2^31, so the 24-bit multiply
// is exact): its depth reads as 0 and fails the update's d > 0 test, exactly like the out-of-image
// skip (an in-image NaN depth still reaches the update, as in Open3D).  `bad` is set unless
// 2^-36 <= zc <= 2^60 (zc <= 0 included, which the update would skip anyway): inside that range
// rcp_m is exact and a non-zero sdf = d - zc is >= 2^-60 in magnitude, which keeps the division
// core exact.
template <int ZPER, int ILP = 1>
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
        const float ax = xs[k] * e[0] + ys[k] * e[1];  // equal operands across k are merged
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
        // out of the image: row H (byte offset H W4 = 4HW, past the end of the frame)
        const uint32_t off = in ? __umul24((uint32_t)(int)v, W4) + ((uint32_t)(int)u << 2) : __umul24((uint32_t)hf, W4);
#if MQR_DIAG == 1  // timing diagnostics only (tools/diag_integrate.sh): projection without the gather
        dv[k] = zc + (float)(off & 1u) * 1e-30f;
#else
        dv[k] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0));
#endif
        // keep each group of ILP voxels' projections next to their loads: hoisting all projections
        // above the loads (the scheduler's choice) keeps ~6 more VGPRs per voxel live and halves the
        // occupancy; ILP > 1 lets the scheduler interleave that many independent chains
        if ((k + 1) % ILP == 0) __builtin_amdgcn_sched_barrier(0);
    }
}

// Running-average update of one frame's gathered depths (zc recomputed by the same operations).
template <int ZPER, int ILP = 1>
__device__ __forceinline__ void lean_update(float2 (&tw)[ZPER], const float (&dv)[ZPER], const FrameParams& fp,
                                            const float (&xs)[ZPER], const float (&ys)[ZPER],
                                            const float (&zs)[ZPER], float depth_max, float sdf_trunc, float y1t) {
    const float e8 = fp.ext[8], e9 = fp.ext[9], e10 = fp.ext[10], e11 = fp.ext[11];
#if MQR_DIAG == 2  // timing diagnostics only: the gather without the update
#pragma unroll
    for (int k = 0; k < ZPER; ++k) tw[k].x += dv[k];
    return;
#endif
#pragma unroll
    for (int k = 0; k < ZPER; ++k) {
        const float az = xs[k] * e8 + ys[k] * e9;
        const float zc = (az + zs[k] * e10) + e11;
        const float d = dv[k];
        const float sdf = d - zc;
        // zc > 0 holds in every block that is not handed to the fix-up launch
        const bool up = !(d <= 0) && !(d > depth_max) && !(sdf < -sdf_trunc);
        const float s = __builtin_fminf(sdf, sdf_trunc);  // = (sdf < trunc ? sdf : trunc), NaN -> trunc
        const float q0 = s * y1t;  // s / sdf_trunc: div_rn_core with the reciprocal refinement hoisted
        const float q1 = __builtin_fmaf(__builtin_fmaf(-sdf_trunc, q0, s), y1t, q0);
        const float sn = __builtin_fmaf(__builtin_fmaf(-sdf_trunc, q1, s), y1t, q1);
        const float wgt = tw[k].y, wp = wgt + 1;
        const float nt = (wgt * tw[k].x + sn) * rcp_m(wp);
        tw[k].x = up ? nt : tw[k].x;
        tw[k].y = up ? wp : wgt;
        if ((k + 1) % ILP == 0) __builtin_amdgcn_sched_barrier(0);  // ILP chains at a time (registers)
    }
}

// ---- window gathers (PAIR = 4: 16-byte, 5: 8-byte windows) ------------------------------------------
// Each lane loads the aligned 16- (8-) byte window holding its pixel and keeps its dword.  Lanes whose
// pixels share a window issue the same address, which the L1 serves once: in tools/gather_ceiling
// the brick map's 64-lane 16-byte window load costs half a 64-lane dword gather of the same pixels
// (6.9 vs 13.6 ns per instruction per CU).  The frame base must be 16- (8-) byte aligned and 4HW a
// multiple of the window (host): then an in-image window never crosses the end of the frame, and an
// out-of-image lane's window at 4HW is wholly past the end (reads 0).
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
template <int ZPER, int ILP = 1, int WIN = 16, bool ZCHK = true, int K0 = 0, int K1 = ZPER, int DIAGV = 0>
__device__ __forceinline__ void lean_gather_w(float (&dv)[ZPER], bool& bad, const FrameParams& fp,
                                              __amdgpu_buffer_rsrc_t rs, const float (&xs)[ZPER],
                                              const float (&ys)[ZPER], const float (&zs)[ZPER], uint32_t W4,
                                              uint32_t past_end, uint32_t hm1_bits, uint32_t wm1_bits) {
    float e[12];
#pragma unroll
    for (int j = 0; j < 12; ++j) e[j] = fp.ext[j];
    const float fx = fp.fx, fy = fp.fy, cx = fp.cx, cy = fp.cy;
#pragma unroll
    for (int k = K0; k < K1; ++k) {
        const float ax = xs[k] * e[0] + ys[k] * e[1];
        const float ay = xs[k] * e[4] + ys[k] * e[5];
        const float az = xs[k] * e[8] + ys[k] * e[9];
        const float xc = (ax + zs[k] * e[2]) + e[3];
        const float yc = (ay + zs[k] * e[6]) + e[7];
        const float zc = (az + zs[k] * e[10]) + e[11];
        if (ZCHK) bad |= (__float_as_uint(zc) - 0x2D800000u) > 0x30000000u;  // not 2^-36 <= zc <= 2^60
        // DIAGV (A/B library only): bit 0 = timing diagnostics (wrong results): the bare v_rcp; bit 1 = the
        // in-image offset computed for every lane and selected.  The default form lets the compiler branch
        // around the offset of out-of-image lanes: 0.595-0.603 vs 0.638-0.647 ms per launch for a form it
        // compiled without those branches (profiles/r05_ab_integrate_branchfree.json, variant 44 vs 0).
        const float inv_z = (DIAGV & 1) ? __builtin_amdgcn_rcpf(zc) : rcp_m(zc);
        const float u = fx * xc * inv_z + cx;
        const float v = fy * yc * inv_z + cy;
        const bool in = (__float_as_uint(v) <= hm1_bits) && (__float_as_uint(u) <= wm1_bits);
        uint32_t off;
        if constexpr ((DIAGV & 2) != 0) {
            uint32_t off_in = __umul24((uint32_t)(int)v, W4) + ((uint32_t)(int)u << 2);
            asm volatile("" : "+v"(off_in));
            off = in ? off_in : past_end;
        } else {
            off = in ? __umul24((uint32_t)(int)v, W4) + ((uint32_t)(int)u << 2) : past_end;
        }
        if constexpr (WIN == 16) {
            const u32x4 q = __builtin_amdgcn_raw_buffer_load_b128(rs, off & ~15u, 0, 0);
            const uint32_t lo = (off & 8u) ? q.z : q.x, hi = (off & 8u) ? q.w : q.y;
            dv[k] = __uint_as_float((off & 4u) ? hi : lo);
        } else {
            const u32x2 q = __builtin_amdgcn_raw_buffer_load_b64(rs, off & ~7u, 0, 0);
            dv[k] = __uint_as_float((off & 4u) ? q.y : q.x);
        }
        if ((k + 1) % ILP == 0) __builtin_amdgcn_sched_barrier(0);
    }
}

// DIV1: s / sdf_trunc with one Markstein correction (the host enables it only for an sdf_trunc whose
// every s in [0, sdf_trunc] it verified against IEEE division, strunc_one_correction_ok; the
// sequence is odd in s, so negative s follow).
template <int ZPER, int ILP = 1, int DIV1 = 0, int K0 = 0, int K1 = ZPER, int DIAGV = 0>
__device__ __forceinline__ void lean_update_v(float2 (&tw)[ZPER], const float (&dv)[ZPER], const FrameParams& fp,
                                              const float (&xs)[ZPER], const float (&ys)[ZPER],
                                              const float (&zs)[ZPER], float depth_max, float sdf_trunc, float y1t) {
    const float e8 = fp.ext[8], e9 = fp.ext[9], e10 = fp.ext[10], e11 = fp.ext[11];
#pragma unroll
    for (int k = K0; k < K1; ++k) {
        const float az = xs[k] * e8 + ys[k] * e9;
        const float zc = (az + zs[k] * e10) + e11;
        const float d = dv[k];
        const float sdf = d - zc;
        if constexpr ((DIAGV & 4) == 0) {
            if (!(d <= 0) && !(d > depth_max) && !(sdf < -sdf_trunc)) {
                float s;
                asm("v_min_f32 %0, %1, %2" : "=v"(s) : "s"(sdf_trunc), "v"(sdf));
                const float q0 = s * y1t;
                const float q1 = (DIAGV & 1) ? q0 : __builtin_fmaf(__builtin_fmaf(-sdf_trunc, q0, s), y1t, q0);
                const float sn = DIV1 || (DIAGV & 1) ? q1 : __builtin_fmaf(__builtin_fmaf(-sdf_trunc, q1, s), y1t, q1);
                const float wgt = tw[k].y, wp = wgt + 1;
                tw[k].x = (wgt * tw[k].x + sn) * ((DIAGV & 1) ? __builtin_amdgcn_rcpf(wp) : rcp_m(wp));
                tw[k].y = wp;
            }
        } else {  // DIAGV bit 2 (A/B library only): every lane evaluates the update and selects (no branch)
            const bool up = !(d <= 0) && !(d > depth_max) && !(sdf < -sdf_trunc);
            float s;
            asm("v_min_f32 %0, %1, %2" : "=v"(s) : "s"(sdf_trunc), "v"(sdf));
            const float q0 = s * y1t;
            const float q1 = (DIAGV & 1) ? q0 : __builtin_fmaf(__builtin_fmaf(-sdf_trunc, q0, s), y1t, q0);
            const float sn = DIV1 || (DIAGV & 1) ? q1 : __builtin_fmaf(__builtin_fmaf(-sdf_trunc, q1, s), y1t, q1);
            const float wgt = tw[k].y;
            float wp = wgt + 1;
            float nt = (wgt * tw[k].x + sn) * ((DIAGV & 1) ? __builtin_amdgcn_rcpf(wp) : rcp_m(wp));
            asm volatile("" : "+v"(nt), "+v"(wp));
            tw[k].x = up ? nt : tw[k].x;
            tw[k].y = up ? wp : wgt;
        }
        if ((k + 1) % ILP == 0) __builtin_amdgcn_sched_barrier(0);
    }
}

// Hand a block to the exact fix-up launch (its (slot, batch mask) appended to bad_out).
__device__ __forceinline__ void hand_off(int32_t* bad_out, int* counters, int64_t list_cap, int32_t slot,
                                         bmask_t mask) {
    const int j = atomicAdd(&counters[kBadCount], 1);
    bad_out[j] = slot;
    reinterpret_cast<bmask_t*>(bad_out + list_cap)[j] = mask;
}

// Thread -> voxels of the lean kernel.
// MAP 0 (plate): thread t owns column (x, y) = (t % R, t / R % R), voxels z = t / R^2 + k NT / R^2;
//   a wave's k-th voxels form a 16 x 4 x 1 plate (R = 16).
// MAP 1 (brick, R = 16, NT = 512): lane l of wave w owns x = l % 8 + 8 (w % 2), y = (l / 8) % 2 +
//   2 (w / 2), z = l / 16, and its voxel k sits at (x, y + 8 (k / 4), z + 4 (k % 4)); a wave's k-th
//   voxels form an 8 x 2 x 4 brick.  Voxels along a viewing ray share pixels, so a brick projects to
//   fewer image rows than a plate (5.8 vs 10.3 distinct cache lines per 64-lane gather on the C2
//   walk); with the occupancy hint below this is the faster map.
template <int R, int NT, int MAP>
__device__ __forceinline__ void lean_map(int tid, int& x, int& y, int& z) {
    if (MAP == 1) {
        const int l = tid & 63, w = tid >> 6;
        x = (l & 7) + 8 * (w & 1);
        y = ((l >> 3) & 1) + 2 * (w >> 1);
        z = l >> 4;
    } else {
        x = tid % R;
        y = (tid / R) % R;
        z = tid / (R * R);
    }
}
// Offsets (voxels along y and z) of a thread's voxel k from its voxel 0.
template <int R, int NT, int MAP>
__host__ __device__ constexpr int lean_dy(int k) { return MAP == 1 ? 8 * (k >> 2) : 0; }
template <int R, int NT, int MAP>
__host__ __device__ constexpr int lean_dz(int k) { return MAP == 1 ? 4 * (k & 3) : k * (NT / (R * R)); }

// Lean integrate with dword gathers (lean_gather / lean_update), unit depth scale only (host: sdf_trunc in
// the division core's range): the fallback of k_integrate_win for frame stacks the 8-byte window reads
// cannot take (an odd pixel count or a base not 8-byte aligned: variant 4) and the R = 8 kernel (plate
// map).  Block per workgroup, voxels per lean_map<MAP>; WPE: minimum waves per SIMD the register
// allocation must allow; ILP: voxel chains the scheduler may interleave.  A block whose operands leave
// the proven ranges is handed to the exact fix-up launch behind the kernel (hand_off) unwritten; every
// other block is written back whole.  (The round-2..4 variants of this kernel -- paired-lane gathers,
// VALU-lean forms, 16-byte windows, block-level zc checks, XCD-grouped lists -- are A/B-only:
// k_integrate_lean_ab in vbg_ab.hpp.)
template <int R, int NT, int MAP = 0, int WPE = 1, int ILP = 1>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(WPE, 8))) void k_integrate_lean(
    const int32_t* __restrict__ list, const bmask_t* __restrict__ lmask, int32_t* __restrict__ bad_out,
    int* __restrict__ counters, int64_t list_cap, Table t, float2* __restrict__ pool, float voxel_size,
    const float* __restrict__ depths, int64_t HW, int H, int W, const FrameParams* __restrict__ fps,
    const int64_t* __restrict__ depth_frame, float depth_max, float sdf_trunc, int first_new) {
    constexpr int R2 = R * R;
    constexpr int R3 = R2 * R;
    constexpr int ZPER = R3 / NT;
    static_assert(R3 % NT == 0 && NT % R2 == 0, "NT must divide R^3 and be a multiple of R^2");
    static_assert(MAP == 0 || (R == 16 && NT == 512), "the brick map is for R = 16, NT = 512");
    const int64_t n = min((int64_t)counters[kListCount], list_cap);
    const float hf = (float)H, hm1 = (float)H - 1.0f, wm1 = (float)W - 1.0f;
    const uint32_t W4 = 4u * (uint32_t)W, bytes = 4u * (uint32_t)HW;
    const float y0t = __builtin_amdgcn_rcpf(sdf_trunc);
    const float y1t = __builtin_fmaf(__builtin_fmaf(-sdf_trunc, y0t, 1.0f), y0t, y0t);
    const int tid = threadIdx.x;
    int vx, vy, vz;
    lean_map<R, NT, MAP>(tid, vx, vy, vz);
    const uint32_t voff = 8u * (uint32_t)(vx + R * vy + R2 * vz);  // byte offset of voxel 0 in its block
    for (int64_t i = blockIdx.x; i < n; i += gridDim.x) {
        const int32_t slot = list[i];
        const int buf = __builtin_amdgcn_readfirstlane(t.vals[slot]);
        const bmask_t mask = readfirstlane_mask(lmask ? lmask[i] : bm_frames(t.mask[slot]));
        int xb, yb, zb;
        unpack_key(t.keys[slot], xb, yb, zb);
        if (buf >= 0 && mask) {
            const __amdgpu_buffer_rsrc_t vox = __builtin_amdgcn_make_buffer_rsrc(
                pool + (int64_t)buf * R3, (short)0, (int)(R3 * sizeof(float2)), 0x00020000);
            float2 tw[ZPER];
            float xs[ZPER], ys[ZPER], zs[ZPER];
            bool bad = false;
            const float xs0 = (float)(xb * R + vx) * voxel_size;
#pragma unroll
            for (int k = 0; k < ZPER; ++k) {
                const int dy = lean_dy<R, NT, MAP>(k), dz = lean_dz<R, NT, MAP>(k);
                // a block allocated by this batch (buffer >= first_new) starts at (0, 0): the pool is
                // not cleared on reset or growth
                tw[k] = buf >= first_new ? make_float2(0.f, 0.f)
                                         : pool_load(vox, voff, (R * dy + R2 * dz) * (int)sizeof(float2));
                xs[k] = xs0;
                ys[k] = (float)(yb * R + vy + dy) * voxel_size;
                zs[k] = (float)(zb * R + vz + dz) * voxel_size;
                const float w = tw[k].y;  // rcp_m(w + 1) is exact for integer w <= 2^23 + 64: a batch adds <= 127
                bad |= !(w >= 0.0f && w <= 0x1p23f - 64.0f && w == __builtin_truncf(w));
            }
            bmask_t m = mask;
            while (m) {
                const int f = bm_ctz(m);
                m &= m - 1;
                float dv[ZPER];
                lean_gather<ZPER, ILP>(dv, bad, fps[f], frame_rsrc(depths + depth_frame[f] * HW, bytes), xs, ys, zs,
                                       W4, hf, hm1, wm1);
                lean_update<ZPER, ILP>(tw, dv, fps[f], xs, ys, zs, depth_max, sdf_trunc, y1t);
            }
            if (__syncthreads_or(bad)) {  // block-uniform: the exact fix-up launch redoes it from the pool
                if (tid == 0) hand_off(bad_out, counters, list_cap, slot, mask);
            } else {
#pragma unroll
                for (int k = 0; k < ZPER; ++k)
                    pool_store(vox, voff, (R * lean_dy<R, NT, MAP>(k) + R2 * lean_dz<R, NT, MAP>(k)) * (int)sizeof(float2),
                               tw[k]);
            }
        }
        __syncthreads();
        if (tid == 0) t.mask[slot] = 0;
    }
}

// ---- the default integrate kernel (R = 16): 8-byte window reads -----------------------------------------------
// 512-thread workgroup per touched block, 8 voxels per thread in registers for all frames of the batch
// (<= 127).  Map: lane l of wave w owns x = l % 8 + 8 (w % 2), y = (l / 8) % 2 + 2 (w / 2), z = l / 16 (a
// wave's voxels k form an 8 x 2 x 4 brick: voxels along a viewing ray share pixels, so a brick projects to
// few image rows), its voxel k sits at (x, y + 8 (k / 4), z + 4 (k % 4)).  Per frame: lean_gather_w
// (exact float32 transform and projection, 1 / zc by v_rcp + one Markstein correction -- exact on the
// proven ranges --, the depth read as the aligned 8-byte window holding the pixel: lanes whose pixels share
// a window issue one address) and lean_update_v (predicated running-average update).  A block whose
// operands leave the proven ranges is redone by the workgroup itself through the exact path
// (exact_block_call, not inlined: its registers stay out of the frame loop's allocation).  >= 7 waves per
// SIMD (three per-block address words spill to scratch outside the frame loop).  Bit-identical to the
// generic kernel (tests/test_gpu_numerics.py).  Measured alternatives, all A/B-only (vbg_ab.hpp,
// DESIGN.md §4.1): the frame loop software-pipelined (whole frames or half frames), 1024-thread
// workgroups, packed FP32 arithmetic -- none faster.
template <int NT>
__host__ __device__ constexpr int win_dy(int k) { return NT == 512 ? 8 * (k >> 2) : 0; }
template <int NT>
__host__ __device__ constexpr int win_dz(int k) { return NT == 512 ? 4 * (k & 3) : 4 * k; }

template <int WPE>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(WPE, 8))) void k_integrate_win(
    const int32_t* __restrict__ list, const bmask_t* __restrict__ lmask, int* __restrict__ counters, int64_t list_cap,
    Table t, float2* __restrict__ pool, float voxel_size, const float* __restrict__ depths, int64_t HW, int H, int W,
    const FrameParams* __restrict__ fps, const int64_t* __restrict__ depth_frame, float depth_max, float sdf_trunc,
    int first_new) {
    constexpr int NT = 512, R = 16, R2 = R * R, R3 = R2 * R;
    constexpr int ZPER = R3 / NT;
    const int64_t n = min((int64_t)counters[kListCount], list_cap);
    const float hm1 = (float)H - 1.0f, wm1 = (float)W - 1.0f;
    const uint32_t W4 = 4u * (uint32_t)W, bytes = 4u * (uint32_t)HW;
    const uint32_t hb = __float_as_uint(hm1), wb = __float_as_uint(wm1);
    const float y0t = __builtin_amdgcn_rcpf(sdf_trunc);
    const float y1t = __builtin_fmaf(__builtin_fmaf(-sdf_trunc, y0t, 1.0f), y0t, y0t);
    const int tid = threadIdx.x;
    const int l = tid & 63, w = tid >> 6;
    const int vx = (l & 7) + 8 * (w & 1), vy = ((l >> 3) & 1) + 2 * (w >> 1), vz = l >> 4;
    const uint32_t voff = 8u * (uint32_t)(vx + R * vy + R2 * vz);  // byte offset of voxel 0 in its block
    for (int64_t i = blockIdx.x; i < n; i += gridDim.x) {
        const int32_t slot = list[i];
        const int buf = __builtin_amdgcn_readfirstlane(t.vals[slot]);
        const bmask_t mask = readfirstlane_mask(lmask ? lmask[i] : bm_frames(t.mask[slot]));
        int xb, yb, zb;
        unpack_key(t.keys[slot], xb, yb, zb);
        if (buf >= 0 && mask) {
            const __amdgpu_buffer_rsrc_t vox = __builtin_amdgcn_make_buffer_rsrc(
                pool + (int64_t)buf * R3, (short)0, (int)(R3 * sizeof(float2)), 0x00020000);
            float2 tw[ZPER];
            float xs[ZPER], ys[ZPER], zs[ZPER];
            bool bad = false;
            const float xs0 = (float)(xb * R + vx) * voxel_size;
#pragma unroll
            for (int k = 0; k < ZPER; ++k) {
                const int dy = win_dy<NT>(k), dz = win_dz<NT>(k);
                // a block allocated by this batch (buffer >= first_new) starts at (0, 0): the pool is not
                // cleared on reset or growth
                tw[k] = buf >= first_new ? make_float2(0.f, 0.f)
                                         : pool_load(vox, voff, (R * dy + R2 * dz) * (int)sizeof(float2));
                xs[k] = xs0;
                ys[k] = (float)(yb * R + vy + dy) * voxel_size;
                zs[k] = (float)(zb * R + vz + dz) * voxel_size;
                const float wv = tw[k].y;  // rcp_m(w + 1) is exact for integer w <= 2^23 + 64: a batch adds <= 127
                bad |= !(wv >= 0.0f && wv <= 0x1p23f - 64.0f && wv == __builtin_truncf(wv));
            }
            bmask_t m = mask;
            while (m) {
                const int f = bm_ctz(m);
                m &= m - 1;
                float dv[ZPER];
                lean_gather_w<ZPER, 2, 8>(dv, bad, fps[f], frame_rsrc(depths + depth_frame[f] * HW, bytes), xs, ys, zs,
                                          W4, bytes, hb, wb);
                lean_update_v<ZPER, 2, 0>(tw, dv, fps[f], xs, ys, zs, depth_max, sdf_trunc, y1t);
            }
            if (__syncthreads_or(bad)) {  // block-uniform: the exact path redoes it from the pool
                exact_block_call<R, NT>(pool + (int64_t)buf * R3, buf >= first_new, mask, xb, yb, zb, voxel_size, depths,
                                        HW, W, hm1, wm1, fps, depth_frame, depth_max, sdf_trunc);
            } else {
#pragma unroll
                for (int k = 0; k < ZPER; ++k)
                    pool_store(vox, voff, (R * win_dy<NT>(k) + R2 * win_dz<NT>(k)) * (int)sizeof(float2), tw[k]);
            }
        }
        __syncthreads();
        if (tid == 0) t.mask[slot] = 0;
    }
}

// ---- the default integrate kernel since round 6: k_integrate_win's loop with the update through an LDS table ---
// k_integrate_win with each voxel's weight held as the byte offset 8 w of its entry in a per-workgroup LDS table
// rtab[w] = ((float) w, rcp_m(w + 1)) filled at kernel start for w < tcount (the host passes the volume's weight
// bound, mqr_vbg wbound): an update reads its entry (one ds_read_b64) instead of v_add + v_rcp + two Markstein
// FMAs, and steps the offset by 8.  (w tsdf + sn) * rcp(w + 1) is evaluated in the same order on the same
// values, so the volume is bit-identical; a block whose weights could leave the table (w + its frame count >
// tcount) or the proven ranges is handed, unwritten, to the exact fix-up launch behind the kernel (hand_off: no
// call inside the kernel, whose saved registers made the frame loop spill).  Launched when the host knows a weight bound
// of at most kRtabMax (launch_integrate); else k_integrate_win.  0.544 vs 0.577 ms per C2 launch
// (profiles/r06_ab_integrate_rtab.json): the update drops a v_rcp (8 issue cycles) and three VALU, and its
// LDS read overlaps the quotient.
constexpr int kRtabMax = 6000;  // table entries: 48 KB of LDS, 3 workgroups per CU still fit

// DIV1: s / sdf_trunc with one Markstein correction (host: strunc_one_correction_ok verified it for this
// sdf_trunc over every s in [-t, t]), as lean_update_v<DIV1>.  OPT (A/B library only): bit 0 keeps the table
// entries' LDS addresses themselves (no base add per read), bit 1 selects the pixel's dword of its 8-byte
// window by one 64-bit shift (v_lshrrev_b64 by 8 * the byte offset; the shifter takes its low 6 bits).
typedef __attribute__((address_space(3))) const float2 lds_float2;
template <int WPE, int DIV1 = 0, int OPT = 0>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(WPE, 8))) void k_integrate_wt(
    const int32_t* __restrict__ list, const bmask_t* __restrict__ lmask, int32_t* __restrict__ bad_out,
    int* __restrict__ counters, int64_t list_cap,
    Table t, float2* __restrict__ pool, float voxel_size, const float* __restrict__ depths, int64_t HW, int H, int W,
    const FrameParams* __restrict__ fps, const int64_t* __restrict__ depth_frame, float depth_max, float sdf_trunc,
    int first_new, int tcount) {
    extern __shared__ float2 rtab[];
    constexpr int NT = 512, R = 16, R2 = R * R, R3 = R2 * R;
    constexpr int ZPER = R3 / NT;
    const int tid = threadIdx.x;
    for (int i = tid; i < tcount; i += NT) rtab[i] = make_float2((float)i, rcp_m((float)i + 1.0f));
    __syncthreads();
    const int64_t n = min((int64_t)counters[kListCount], list_cap);
    const float hm1 = (float)H - 1.0f, wm1 = (float)W - 1.0f;
    const uint32_t W4 = 4u * (uint32_t)W, bytes = 4u * (uint32_t)HW;
    const uint32_t hb = __float_as_uint(hm1), wb = __float_as_uint(wm1);
    const float y0t = __builtin_amdgcn_rcpf(sdf_trunc);
    const float y1t = __builtin_fmaf(__builtin_fmaf(-sdf_trunc, y0t, 1.0f), y0t, y0t);
    const int l = tid & 63, w = tid >> 6;
    const int vx = (l & 7) + 8 * (w & 1), vy = ((l >> 3) & 1) + 2 * (w >> 1), vz = l >> 4;
    const uint32_t voff = 8u * (uint32_t)(vx + R * vy + R2 * vz);
    const char* tbase = reinterpret_cast<const char*>(rtab);
    const uint32_t lbase = (OPT & 1) ? (uint32_t)(uintptr_t)(lds_float2*)rtab : 0u;  // LDS address of entry 0
    for (int64_t i = blockIdx.x; i < n; i += gridDim.x) {
        const int32_t slot = list[i];
        const int buf = __builtin_amdgcn_readfirstlane(t.vals[slot]);
        const bmask_t mask = readfirstlane_mask(lmask ? lmask[i] : bm_frames(t.mask[slot]));
        int xb, yb, zb;
        unpack_key(t.keys[slot], xb, yb, zb);
        if (buf >= 0 && mask) {
            const __amdgpu_buffer_rsrc_t vox = __builtin_amdgcn_make_buffer_rsrc(
                pool + (int64_t)buf * R3, (short)0, (int)(R3 * sizeof(float2)), 0x00020000);
            float ts[ZPER];
            uint32_t wa[ZPER];  // 8 w: the byte offset of the voxel's table entry
            float xs[ZPER], ys[ZPER], zs[ZPER];
            bool bad = false;
            const float wlim = (float)(tcount - bm_popc(mask));  // every w read stays below tcount
            const float xs0 = (float)(xb * R + vx) * voxel_size;
#pragma unroll
            for (int k = 0; k < ZPER; ++k) {
                const int dy = win_dy<NT>(k), dz = win_dz<NT>(k);
                const float2 tw = buf >= first_new ? make_float2(0.f, 0.f)
                                                   : pool_load(vox, voff, (R * dy + R2 * dz) * (int)sizeof(float2));
                xs[k] = xs0;
                ys[k] = (float)(yb * R + vy + dy) * voxel_size;
                zs[k] = (float)(zb * R + vz + dz) * voxel_size;
                bad |= !(tw.y >= 0.0f && tw.y <= wlim && tw.y == __builtin_truncf(tw.y));
                ts[k] = tw.x;
                wa[k] = lbase + 8u * (uint32_t)(bad ? 0.0f : tw.y);
            }
            bmask_t m = mask;
            while (m) {
                const int f = bm_ctz(m);
                m &= m - 1;
                float dv[ZPER];
                u32x2 qv[ZPER];
                uint32_t shv[ZPER];
                if constexpr ((OPT & 2) != 0) {  // lean_gather_w<ZPER, 2, 8>'s operations, the window kept whole
                    const FrameParams& g = fps[f];
                    const __amdgpu_buffer_rsrc_t rs = frame_rsrc(depths + depth_frame[f] * HW, bytes);
                    float e[12];
#pragma unroll
                    for (int j = 0; j < 12; ++j) e[j] = g.ext[j];
#pragma unroll
                    for (int k = 0; k < ZPER; ++k) {
                        const float ax = xs[k] * e[0] + ys[k] * e[1];
                        const float ay = xs[k] * e[4] + ys[k] * e[5];
                        const float az = xs[k] * e[8] + ys[k] * e[9];
                        const float xc = (ax + zs[k] * e[2]) + e[3];
                        const float yc = (ay + zs[k] * e[6]) + e[7];
                        const float zc = (az + zs[k] * e[10]) + e[11];
                        bad |= (__float_as_uint(zc) - 0x2D800000u) > 0x30000000u;
                        const float inv_z = rcp_m(zc);
                        const float u = g.fx * xc * inv_z + g.cx;
                        const float v = g.fy * yc * inv_z + g.cy;
                        const bool in = (__float_as_uint(v) <= hb) && (__float_as_uint(u) <= wb);
                        const uint32_t off = in ? __umul24((uint32_t)(int)v, W4) + ((uint32_t)(int)u << 2) : bytes;
                        qv[k] = __builtin_amdgcn_raw_buffer_load_b64(rs, off & ~7u, 0, 0);
                        shv[k] = off << 3;
                        if ((k + 1) % 2 == 0) __builtin_amdgcn_sched_barrier(0);
                    }
                } else {
                    lean_gather_w<ZPER, 2, 8>(dv, bad, fps[f], frame_rsrc(depths + depth_frame[f] * HW, bytes), xs, ys,
                                              zs, W4, bytes, hb, wb);
                }
                const FrameParams& fp = fps[f];
                const float e8 = fp.ext[8], e9 = fp.ext[9], e10 = fp.ext[10], e11 = fp.ext[11];
#pragma unroll
                for (int k = 0; k < ZPER; ++k) {
                    const float az = xs[k] * e8 + ys[k] * e9;
                    const float zc = (az + zs[k] * e10) + e11;
                    float d;
                    if constexpr ((OPT & 2) != 0) {
                        uint64_t r;
                        const uint64_t q64 = ((uint64_t)qv[k].y << 32) | qv[k].x;
                        asm("v_lshrrev_b64 %0, %1, %2" : "=v"(r) : "v"(shv[k]), "v"(q64));
                        d = __uint_as_float((uint32_t)r);
                    } else {
                        d = dv[k];
                    }
                    const float sdf = d - zc;
                    if (!(d <= 0) && !(d > depth_max) && !(sdf < -sdf_trunc)) {
                        // the entry read first: its LDS latency overlaps the quotient
                        float2 e;  // (w, 1 / (w + 1))
                        if constexpr ((OPT & 1) != 0) {
                            lds_float2* px = (lds_float2*)(uintptr_t)wa[k];
                            e = make_float2(px->x, px->y);
                        } else {
                            e = *reinterpret_cast<const float2*>(tbase + wa[k]);
                        }
                        float s;
                        asm("v_min_f32 %0, %1, %2" : "=v"(s) : "s"(sdf_trunc), "v"(sdf));
                        const float q0 = s * y1t;
                        const float q1 = __builtin_fmaf(__builtin_fmaf(-sdf_trunc, q0, s), y1t, q0);
                        const float sn = DIV1 ? q1 : __builtin_fmaf(__builtin_fmaf(-sdf_trunc, q1, s), y1t, q1);
                        ts[k] = (e.x * ts[k] + sn) * e.y;
                        wa[k] += 8u;
                    }
                    if ((k + 1) % 2 == 0) __builtin_amdgcn_sched_barrier(0);
                }
            }
            if (__syncthreads_or(bad)) {  // block-uniform: the exact fix-up launch redoes it from the pool
                if (tid == 0) hand_off(bad_out, counters, list_cap, slot, mask);
            } else {
#pragma unroll
                for (int k = 0; k < ZPER; ++k)
                    pool_store(vox, voff, (R * win_dy<NT>(k) + R2 * win_dz<NT>(k)) * (int)sizeof(float2),
                               make_float2(ts[k], (float)((wa[k] - lbase) >> 3)));
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

// One-correction quotient s / t of lean_update_v<DIV1 = 1> against IEEE division for every float s
// with bits in [lo_bits, lo_bits + count) (the host passes [+0, t]).
__global__ void k_check_strunc(float t, uint32_t lo_bits, uint64_t count, uint32_t* mismatches) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    const float s = __uint_as_float(lo_bits + (uint32_t)i);
    const float y0t = __builtin_amdgcn_rcpf(t);
    const float y1t = __builtin_fmaf(__builtin_fmaf(-t, y0t, 1.0f), y0t, y0t);
    const float q0 = s * y1t;
    const float q1 = __builtin_fmaf(__builtin_fmaf(-t, q0, s), y1t, q0);
    if (__float_as_uint(q1) != __float_as_uint(s / t)) atomicAdd(mismatches, 1u);
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

// Gate of a speculatively launched integrate (the first batch of a call is integrated right behind
// its touch, before the host has read the touch's counters): copy the batch counters into the shadow
// set the integrate and its fix-up read, with the list emptied when the touch needs the host (pool
// overflow, full table, list overflow, key range, or a frame that touched nothing) -- the integrate
// then does nothing and the host redoes the batch the ordinary way -- and the fix-up count zeroed.
__global__ void k_gate(const int* __restrict__ ctr, int* __restrict__ shadow, int nframes) {
    const int lane = threadIdx.x;  // one wave
    bool empty = false;
    for (int f = lane; f < nframes; f += 64) empty |= ctr[kFrameCounterBase + f] == 0;
    gate_counters(ctr, shadow, __ballot(empty) != 0 || ctr[kOverflow] != 0);
}

// Empty table: keys empty, values -1, both parities' slot masks 0; and the counter segments `segs` selects
// zeroed (bit 0 / 1: parity 0 / 1, bit 2: the pool counter and its spare ints, bit 3 / 4: the parities'
// shadow sets -- a reset that swapped the volume's sets leaves an in-flight integrate's parity alone).
__global__ void k_reset_table(Table t, bmask_t* mask1, int* counters, uint32_t segs) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < t.cap) {
        t.keys[i] = kEmpty;
        t.vals[i] = -1;
        t.mask[i] = 0;
        mask1[i] = 0;
    }
    if (i < kCounterInts) {
        const int seg = i < kCountersTotal ? 0 : i < 2 * kCountersTotal ? 1 : i < 2 * kCountersTotal + 8 ? 2
                      : i < 3 * kCountersTotal + 8 ? 3 : 4;
        if ((segs >> seg) & 1u) counters[i] = 0;
    }
}

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

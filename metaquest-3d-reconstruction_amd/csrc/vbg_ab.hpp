// A/B integrate machinery kept out of the shipped library (built only into tools/_ab/libmqr_ab.so,
// MQR_AB = 1; see the Makefile target `ab`): the XCD-grouped list order (variant bit 0x8000) and the
// LDS-tiled integrate kernel (variant 5) with its timing-only MQR_DIAG 3 / 4 / 5 builds.  Both are
// bit-identical to the generic kernel (tests/test_gpu_ab_variants.py) and slower than the default
// (DESIGN.md §4.1).  Included by vbg.hip after vbg_kernels.hpp.
#pragma once

namespace mqr {

// XCD-grouped longest-first order (variant bit 0x8000, A/B; not the default).  Workgroups are
// dispatched round-robin over the 8 XCDs (blockIdx % 8 labels the workgroups that share an XCD and
// its L2; cdna_hip_programming.md T1), so a list in plain LPT order hands every XCD blocks from the
// whole volume and each XCD's L2 fetches nearly every depth line of every frame of the batch
// (traffic 2.7x the algorithmic bytes).  Here the batch's blocks are cut into 8 spatially compact
// groups of equal work (popcount of the frame mask): Morton order of a 16^3 grid of cells over the
// batch's bounding box, cut at the work octiles (a cell on a cut is split by arrival order).  Group
// g is written to [off[g], off[g+1]) of `out` in longest-first order, and the integrate kernel runs
// group g on the workgroups with blockIdx % 8 == g.  Traffic falls to 1.35x, but the launch is 13 %
// slower: the kernel is bound by the gather address path, not by HBM, and the XCDs' shares of the
// time do not balance.  One workgroup; `gbyte` is n bytes of scratch.
__global__ __launch_bounds__(1024) void k_xcd_order(const int32_t* __restrict__ list, int* __restrict__ counters,
                                                    int64_t list_cap, Table t, int32_t* __restrict__ out,
                                                    bmask_t* __restrict__ out_mask, uint8_t* __restrict__ gbyte) {
    constexpr int kCells = 4096;
    __shared__ int cellw[kCells];   // work per cell, then the work before the cell in Morton order
    __shared__ int cellrun[kCells]; // work of the cell's blocks placed so far
    __shared__ int ghist[kNumGroups][kMaxBatch + 1];
    __shared__ int bb[6];
    __shared__ int wsum[1024 / 64];
    const int n = (int)min((int64_t)counters[kListCount], list_cap);
    const int tid = threadIdx.x;
    for (int c = tid; c < kCells; c += blockDim.x) cellw[c] = cellrun[c] = 0;
    for (int c = tid; c < kNumGroups * (kMaxBatch + 1); c += blockDim.x) (&ghist[0][0])[c] = 0;
    if (tid < 3) bb[tid] = INT_MAX;
    else if (tid < 6) bb[tid] = INT_MIN;
    __syncthreads();
    for (int i = tid; i < n; i += blockDim.x) {
        int x, y, z;
        unpack_key(t.keys[list[i]], x, y, z);
        atomicMin(&bb[0], x), atomicMin(&bb[1], y), atomicMin(&bb[2], z);
        atomicMax(&bb[3], x), atomicMax(&bb[4], y), atomicMax(&bb[5], z);
    }
    __syncthreads();
    auto cell_of = [&](uint64_t key) {
        int x, y, z;
        unpack_key(key, x, y, z);
        const int c[3] = {((x - bb[0]) * 16) / (bb[3] - bb[0] + 1), ((y - bb[1]) * 16) / (bb[4] - bb[1] + 1),
                          ((z - bb[2]) * 16) / (bb[5] - bb[2] + 1)};
        int code = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
            for (int a = 0; a < 3; ++a) code |= ((c[a] >> b) & 1) << (3 * b + a);
        return code;
    };
    for (int i = tid; i < n; i += blockDim.x) {
        const int32_t s = list[i];
        atomicAdd(&cellw[cell_of(t.keys[s])], bm_popc(bm_frames(t.mask[s])));
    }
    __syncthreads();
    // exclusive scan of the 4096 cell weights: 4 per thread, wave shuffles, then the 16 wave totals
    int v4[4], acc = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        v4[k] = cellw[4 * tid + k];
        acc += v4[k];
    }
    int incl = acc;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int u = __shfl_up(incl, o, 64);
        if ((tid & 63) >= o) incl += u;
    }
    if ((tid & 63) == 63) wsum[tid >> 6] = incl;
    __syncthreads();
    int before = incl - acc;
    for (int w = 0; w < (tid >> 6); ++w) before += wsum[w];
    int total = 0;
    for (int w = 0; w < 1024 / 64; ++w) total += wsum[w];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        cellw[4 * tid + k] = before;
        before += v4[k];
    }
    __syncthreads();
    for (int i = tid; i < n; i += blockDim.x) {
        const int32_t s = list[i];
        const int w = bm_popc(bm_frames(t.mask[s]));
        const int c = cell_of(t.keys[s]);
        const int64_t start = (int64_t)cellw[c] + atomicAdd(&cellrun[c], w);
        const int g = total > 0 ? (int)min<int64_t>(kNumGroups - 1, ((2 * start + w) * kNumGroups) / (2 * (int64_t)total)) : 0;
        gbyte[i] = (uint8_t)g;
        atomicAdd(&ghist[g][w], 1);
    }
    __syncthreads();
    if (tid == 0) {  // group offsets, and within each group the longest-first positions
        int pos = 0;
        for (int g = 0; g < kNumGroups; ++g) {
            counters[kGroupBase + g] = pos;
            for (int c = kMaxBatch; c >= 0; --c) {
                const int h = ghist[g][c];
                ghist[g][c] = pos;
                pos += h;
            }
        }
        counters[kGroupBase + kNumGroups] = pos;
    }
    __syncthreads();
    for (int i = tid; i < n; i += blockDim.x) {
        const int32_t s = list[i];
        const bmask_t m = bm_frames(t.mask[s]);
        const int pos = atomicAdd(&ghist[gbyte[i]][bm_popc(m)], 1);
        out[pos] = s;
        out_mask[pos] = m;
    }
}

// ---- helpers of the tiled kernel ------------------------------------------------------------------
typedef __attribute__((address_space(1))) void gvoid_t;
typedef __attribute__((address_space(3))) void lvoid_t;

// Index of the j-th (from 0) set bit of m (m has more than j set bits).
__device__ __forceinline__ int nth_bit(bmask_t m, int j) {
    uint64_t q = (uint64_t)m;
    int base = 0;
    const int c64 = __popcll(q);
    if (j >= c64) {
        j -= c64;
        base = 64;
        q = (uint64_t)(m >> 64);
    }
    uint32_t w = (uint32_t)q;
    const int c = __popc(w);
    if (j >= c) {
        j -= c;
        base += 32;
        w = (uint32_t)(q >> 32);
    }
#pragma unroll
    for (int s = 16; s >= 1; s >>= 1) {
        const int cl = __popc(w & ((1u << s) - 1));
        if (j >= cl) {
            j -= cl;
            w >>= s;
            base += s;
        }
    }
    return base;
}

// ---- tiled integrate (A/B, variant 5): depth read from LDS tiles instead of gathered from HBM ---------
// The lean kernel is co-limited by the vector-memory address path (TA busy ~0.74 of the launch,
// ~45 TCP tag lookups per 64-lane dword gather) and by VALU issue (~0.57).  Here the pixel rectangle
// a block projects to in each frame -- its 8 corners projected with the kernel's own operations
// (all voxels lie in their hull when every corner is in front of the camera), padded by 2 px,
// clamped to the image, the left edge aligned down to 4 px -- is copied into LDS with 16-byte
// LDS-DMA loads and the voxels read their depth from there.  Each rectangle gets only the LDS it
// needs (pitch = its width rounded up to 4 px, size rounded up to one 64-lane copy instruction =
// 256 floats; a 16^3 block of 5 mm voxels at 2 m covers ~22 x 22 px), and consecutive frames (bit
// order) are packed into one half of a double buffer until it is full: one workgroup barrier per
// group of frames, group g + 1 copied while group g is integrated.  Rectangles come from 8 waves at
// once (frame j: wave j / 8, lanes (j % 8, corner)); the grouping is a greedy scan over a wave-wide
// prefix sum of the tile sizes.  A frame whose rectangle exceeds 68 x 64 px, or whose corners leave
// 2^-30 <= zc <= 2^50, uses the lean kernel's direct gathers; one outside the image is skipped.
// Measured: TA busy 0.74 -> 0.12, but VALU +15 % (rectangles, the in-image test
// where a rectangle touches the border) and 0.39 vs 0.34 ms per launch.  Earlier forms -- one tile
// per frame with a barrier each (k_integrate_tb), packed f32 math at 6 waves / SIMD (k_integrate_tg)
// -- were 0.40 ms and are gone.
constexpr int kTBP = 68;                 // widest rectangle (px; 17 chunks of 4 px)
constexpr int kTBH = 64;                 // tallest rectangle (rows)
constexpr int kTGHalf = kTBP * kTBH;     // floats per half of the double buffer (17 KB): one worst-case tile
constexpr int kTGSlots = kTGHalf / 256;  // 64-lane copy instructions per half

struct TileShared {
    __attribute__((aligned(16))) float tile[2][kTGHalf];
    int4 rect[kMaxBatch];  // frame j of the block (bit order): u0, v0, width (0: outside the image,
                           // -1: direct gathers), height | inner << 16 (1 px off every image edge)
    int off[kMaxBatch];    // its tile's offset in its group's half (floats)
    int fidx[kMaxBatch];   // its bit (batch frame)
    int gstart[kMaxBatch + 1], gq[kMaxBatch];  // group g: first frame, copy instructions
    uint8_t qf[kMaxBatch * kTGSlots];          // group g, instruction q -> frame
    int ng;
};

// Rectangles and groups of one block's frames (call with the whole workgroup; ends on a barrier).
__device__ __forceinline__ void tile_plan(TileShared& sh, bmask_t mask, int nf, int xb, int yb, int zb, int R,
                                          float voxel_size, const FrameParams* __restrict__ fps, int H, int W) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    {
        const int c = lane & 7, j = 8 * wave + (lane >> 3);
        if (8 * wave < nf) {  // wave-uniform
            const bool have = j < nf;
            const int fb = have ? nth_bit(mask, j) : 0;
            const FrameParams& fp = fps[fb];
            const float cxs = (float)(xb * R + (c & 1) * (R - 1)) * voxel_size;
            const float cys = (float)(yb * R + ((c >> 1) & 1) * (R - 1)) * voxel_size;
            const float czs = (float)(zb * R + (c >> 2) * (R - 1)) * voxel_size;
            const float xc = ((cxs * fp.ext[0] + cys * fp.ext[1]) + czs * fp.ext[2]) + fp.ext[3];
            const float yc = ((cxs * fp.ext[4] + cys * fp.ext[5]) + czs * fp.ext[6]) + fp.ext[7];
            const float zc = ((cxs * fp.ext[8] + cys * fp.ext[9]) + czs * fp.ext[10]) + fp.ext[11];
            const float inv = rcp_m(zc);
            const float u = fp.fx * xc * inv + fp.cx;
            const float v = fp.fy * yc * inv + fp.cy;
            int ok = zc >= 0x1p-30f && zc <= 0x1p50f && fabsf(u) < 1e6f && fabsf(v) < 1e6f;
            float umin = u, umax = u, vmin = v, vmax = v;
#pragma unroll
            for (int o = 1; o <= 4; o <<= 1) {
                umin = fminf(umin, __shfl_xor(umin, o, 64));
                umax = fmaxf(umax, __shfl_xor(umax, o, 64));
                vmin = fminf(vmin, __shfl_xor(vmin, o, 64));
                vmax = fmaxf(vmax, __shfl_xor(vmax, o, 64));
                ok &= __shfl_xor(ok, o, 64);
            }
            if (have && c == 0) {
                int4 r = make_int4(0, 0, -1, 0);
                if (ok) {
                    const int u0 = max(0, (int)floorf(umin) - 2) & ~3, u1 = min(W - 1, (int)floorf(umax) + 2);
                    const int v0 = max(0, (int)floorf(vmin) - 2), v1 = min(H - 1, (int)floorf(vmax) + 2);
                    const int w = u1 - u0 + 1, h = v1 - v0 + 1;
                    const bool inner = u0 >= 1 && u1 <= W - 2 && v0 >= 1 && v1 <= H - 2;
                    if (w <= 0 || h <= 0)
                        r = make_int4(0, 0, 0, 0);
                    else if (w <= kTBP && h <= kTBH)
                        r = make_int4(u0, v0, w, h | (inner ? 0x10000 : 0));
                }
                sh.rect[j] = r;
                sh.fidx[j] = fb;
            }
        }
    }
    __syncthreads();
    if (wave == 0) {  // lane = frame; greedy groups over the prefix sum of tile sizes
        const int4 r = lane < nf ? sh.rect[lane] : make_int4(0, 0, 0, 0);
        const int A = r.z > 0 ? ((((r.w & 0xffff) * ((r.z + 3) >> 2)) + 63) >> 6) << 8 : 0;  // <= kTGHalf
        int P = A;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int u = __shfl_up(P, o, 64);
            if (lane >= o) P += u;
        }
        int s = 0, base = 0, g = 0, grp = 0, off = 0;
        while (s < nf) {  // wave-uniform; every group takes at least frame s (A_s <= kTGHalf)
            const uint64_t b = __ballot(lane >= s && lane < nf && P - base <= kTGHalf);
            const int e = 64 - __builtin_clzll(b);
            if (lane >= s && lane < e) {
                grp = g;
                off = P - A - base;
            }
            const int end = __shfl(P, e - 1, 64);
            if (lane == 0) {
                sh.gstart[g] = s;
                sh.gq[g] = (end - base) >> 8;
            }
            base = end;
            s = e;
            ++g;
        }
        if (lane == 0) {
            sh.gstart[g] = nf;
            sh.ng = g;
        }
        if (lane < nf) {
            sh.off[lane] = off;
            for (int q = 0; q < (A >> 8); ++q) sh.qf[grp * kTGSlots + (off >> 8) + q] = (uint8_t)lane;
        }
    }
    __syncthreads();
}

// Copy of group g into half g & 1: instruction q (wave-uniform) covers 64 consecutive 4-px chunks of
// one frame's tile; chunks past the tile's last row re-read its row 0 into the unused tail.
__device__ __forceinline__ void tile_stage(TileShared& sh, int g, const float* __restrict__ depths, int64_t HW, int W,
                                           const int64_t* __restrict__ depth_frame) {
#if MQR_DIAG == 4 || MQR_DIAG == 5  // timing diagnostics only: no tile copies
    return;
#endif
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, nwaves = blockDim.x >> 6;
    const int Q = __builtin_amdgcn_readfirstlane(sh.gq[g]);
    float* half = sh.tile[g & 1];
    for (int q = wave; q < Q; q += nwaves) {
        const int j = __builtin_amdgcn_readfirstlane(sh.qf[g * kTGSlots + q]);
        const int4 r = sh.rect[j];
        const int u0 = __builtin_amdgcn_readfirstlane(r.x), v0 = __builtin_amdgcn_readfirstlane(r.y);
        const int pq = (__builtin_amdgcn_readfirstlane(r.z) + 3) >> 2;
        const int h = __builtin_amdgcn_readfirstlane(r.w) & 0xffff;
        const int fb = __builtin_amdgcn_readfirstlane(sh.fidx[j]);
        const int c = (q - (__builtin_amdgcn_readfirstlane(sh.off[j]) >> 8)) * 64 + lane;
        int row = (int)(((float)c + 0.5f) * __builtin_amdgcn_rcpf((float)pq));  // c / pq (c < 1088)
        const int col = c - row * pq;
        row = row < h ? row : 0;
        const float* dep = depths + depth_frame[fb] * HW;
        const int gc = min(u0 + 4 * col, W - 4);
        __builtin_amdgcn_global_load_lds((gvoid_t*)(dep + (int64_t)(v0 + row) * W + gc), (lvoid_t*)(half + 256 * q),
                                         16, 0, 0);
    }
}

// Per voxel: Open3D's projection (the same operations as lean_gather), then the tile read; a voxel
// in the image but outside its frame's rectangle sets `bad` (the block is redone exactly), one
// outside the image reads 0 (as lean_gather's past-the-end read).  Every corner of the block has
// 2^-30 <= zc <= 2^50 when a frame has a rectangle, so the voxels' 1 / zc by rcp_m is exact without
// lean_gather's per-voxel range check.  INNER: the rectangle keeps 1 px off every image edge, so a
// voxel inside it is inside the image (no bound test).
template <int ZPER, int ILP, bool INNER>
__device__ __forceinline__ void lean_gather_tile(float (&dv)[ZPER], bool& bad, const FrameParams& fp,
                                                 const float* tile, int rx, int ry, uint32_t tw, uint32_t th,
                                                 uint32_t pitch, const float (&xs)[ZPER], const float (&ys)[ZPER],
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
        const float inv_z = rcp_m(zc);
        const float u = fx * xc * inv_z + cx;
        const float v = fy * yc * inv_z + cy;
        const uint32_t tu = (uint32_t)((int)u - rx), tv = (uint32_t)((int)v - ry);
        const bool hit = (tu < tw) & (tv < th);
#if MQR_DIAG == 3 || MQR_DIAG == 5
        const float d = zc + (float)((hit ? __umul24(tv, pitch) + tu : 0) & 1u) * 1e-30f;
#else
        const float d = tile[hit ? __umul24(tv, pitch) + tu : 0];
#endif
        if (INNER) {
            bad |= !hit;
            dv[k] = d;
        } else {
            const bool in = (v >= 0) & (u >= 0) & (v <= hm1) & (u <= wm1);
            bad |= in & !hit;
            dv[k] = in ? d : 0.f;
        }
        if ((k + 1) % ILP == 0) __builtin_amdgcn_sched_barrier(0);
    }
}

template <int ILP>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_integrate_lt(
    const int32_t* __restrict__ list, const bmask_t* __restrict__ lmask, int32_t* __restrict__ bad_out,
    int* __restrict__ counters, int64_t list_cap, Table t, float2* __restrict__ pool, float voxel_size,
    const float* __restrict__ depths, int64_t HW, int H, int W, const FrameParams* __restrict__ fps,
    const int64_t* __restrict__ depth_frame, float depth_max, float sdf_trunc, int first_new) {
    constexpr int R = 16, R2 = R * R, R3 = R2 * R, NT = 512, ZPER = R3 / NT, MAP = 1;
    __shared__ TileShared sh;
    const int64_t n = min((int64_t)counters[kListCount], list_cap);
    const float hf = (float)H, hm1 = (float)H - 1.0f, wm1 = (float)W - 1.0f;
    const uint32_t W4 = 4u * (uint32_t)W, bytes = 4u * (uint32_t)HW;
    const float y0t = __builtin_amdgcn_rcpf(sdf_trunc);
    const float y1t = __builtin_fmaf(__builtin_fmaf(-sdf_trunc, y0t, 1.0f), y0t, y0t);
    const int tid = threadIdx.x;
    int vx, vy, vz;
    lean_map<R, NT, MAP>(tid, vx, vy, vz);
    const uint32_t voff = 8u * (uint32_t)(vx + R * vy + R2 * vz);
    for (int64_t i = blockIdx.x; i < n; i += gridDim.x) {
        const int32_t slot = list[i];
        const int buf = __builtin_amdgcn_readfirstlane(t.vals[slot]);
        const bmask_t mask = readfirstlane_mask(lmask ? lmask[i] : bm_frames(t.mask[slot]));
        int xb, yb, zb;
        unpack_key(t.keys[slot], xb, yb, zb);
        if (buf < 0 || !mask) {  // block-uniform
            __syncthreads();
            if (tid == 0) t.mask[slot] = 0;
            continue;
        }
        const __amdgpu_buffer_rsrc_t vox = __builtin_amdgcn_make_buffer_rsrc(
            pool + (int64_t)buf * R3, (short)0, (int)(R3 * sizeof(float2)), 0x00020000);
        float2 tw[ZPER];
        float xs[ZPER], ys[ZPER], zs[ZPER];
        bool bad = false;
        const float xs0 = (float)(xb * R + vx) * voxel_size;
#pragma unroll
        for (int k = 0; k < ZPER; ++k) {
            const int dy = lean_dy<R, NT, MAP>(k), dz = lean_dz<R, NT, MAP>(k);
            tw[k] = buf >= first_new ? make_float2(0.f, 0.f)
                                     : pool_load(vox, voff, (R * dy + R2 * dz) * (int)sizeof(float2));
            xs[k] = xs0;
            ys[k] = (float)(yb * R + vy + dy) * voxel_size;
            zs[k] = (float)(zb * R + vz + dz) * voxel_size;
            const float w = tw[k].y;  // rcp_m(w + 1) is exact for integer w <= 2^23 + 64: a batch adds <= 127
            bad |= !(w >= 0.0f && w <= 0x1p23f - 64.0f && w == __builtin_truncf(w));
        }
        tile_plan(sh, mask, bm_popc(mask), xb, yb, zb, R, voxel_size, fps, H, W);
        const int ng = __builtin_amdgcn_readfirstlane(sh.ng);
        tile_stage(sh, 0, depths, HW, W, depth_frame);
        bmask_t m = mask;
        for (int g = 0; g < ng; ++g) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's copies of group g have landed
            __syncthreads();  // ... every wave's; and every wave is done with group g - 1's half
            if (g + 1 < ng) tile_stage(sh, g + 1, depths, HW, W, depth_frame);
            const float* half = sh.tile[g & 1];
            const int j1 = __builtin_amdgcn_readfirstlane(sh.gstart[g + 1]);
            for (int j = __builtin_amdgcn_readfirstlane(sh.gstart[g]); j < j1; ++j) {
                const int f = bm_ctz(m);
                m &= m - 1;
                int4 r = sh.rect[j];
                r = make_int4(__builtin_amdgcn_readfirstlane(r.x), __builtin_amdgcn_readfirstlane(r.y),
                              __builtin_amdgcn_readfirstlane(r.z), __builtin_amdgcn_readfirstlane(r.w));
                if (r.z == 0) continue;  // the block is outside this frame's image
                float dv[ZPER];
                if (r.z > 0) {
                    const float* tile = half + __builtin_amdgcn_readfirstlane(sh.off[j]);
                    const uint32_t pitch = (uint32_t)((r.z + 3) & ~3);
                    if (r.w >> 16)
                        lean_gather_tile<ZPER, ILP, true>(dv, bad, fps[f], tile, r.x, r.y, (uint32_t)r.z,
                                                          (uint32_t)(r.w & 0xffff), pitch, xs, ys, zs, hm1, wm1);
                    else
                        lean_gather_tile<ZPER, ILP, false>(dv, bad, fps[f], tile, r.x, r.y, (uint32_t)r.z,
                                                           (uint32_t)(r.w & 0xffff), pitch, xs, ys, zs, hm1, wm1);
                } else {
                    lean_gather<ZPER, ILP>(dv, bad, fps[f], frame_rsrc(depths + depth_frame[f] * HW, bytes), xs, ys,
                                           zs, W4, hf, hm1, wm1);
                }
                lean_update<ZPER, ILP>(tw, dv, fps[f], xs, ys, zs, depth_max, sdf_trunc, y1t);
            }
        }
        if (__syncthreads_or(bad)) {  // block-uniform: the exact fix-up launch redoes it from the pool
            if (tid == 0) hand_off(bad_out, counters, list_cap, slot, mask);
        } else {
#pragma unroll
            for (int k = 0; k < ZPER; ++k)
                pool_store(vox, voff, (R * lean_dy<R, NT, MAP>(k) + R2 * lean_dz<R, NT, MAP>(k)) * (int)sizeof(float2),
                           tw[k]);
        }
        __syncthreads();
        if (tid == 0) t.mask[slot] = 0;
    }
}

// ---- paired-lane gather (A/B, variant 6) ----------------------------------------------------------
// Lanes l and l ^ 1 of the brick map hold x-adjacent voxels, which mostly project into the same
// image row within 4 pixels (80 % of pairs on the C2 walk, tools/integrate_work_stats.py).  The even
// lane loads the 16-byte-aligned window holding its own pixel and hands the odd lane its dword (DPP
// quad swap) when that dword lies in the window; every other lane issues its own dword gather.  Two gather instructions per
// voxel (x4 by even lanes, x1 by the rest) in place of one x1 by all 64 lanes: fewer addresses for
// the texture addresser and the L1 tag lookups, ~10 more VALU per voxel-frame.  Same values as
// lean_gather: a served lane reads the same dword; a 16-byte load that would leave the frame is not
// used (out-of-range dwords read as 0).
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
template <int ZPER, int ILP>
__device__ void lean_gather_pair(float (&dv)[ZPER], bool& bad, const FrameParams& fp, __amdgpu_buffer_rsrc_t rs,
                                 const float (&xs)[ZPER], const float (&ys)[ZPER], const float (&zs)[ZPER], uint32_t W4,
                                 float hf, float hm1, float wm1, uint32_t bytes) {
    constexpr int kSwap = 0xB1;  // DPP quad_perm [1, 0, 3, 2]: the partner lane
    float e[12];
#pragma unroll
    for (int j = 0; j < 12; ++j) e[j] = fp.ext[j];
    const float fx = fp.fx, fy = fp.fy, cx = fp.cx, cy = fp.cy;
    const bool odd = threadIdx.x & 1;
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
        const float u = fx * xc * inv_z + cx;
        const float v = fy * yc * inv_z + cy;
        const bool in = (v >= 0) & (u >= 0) & (v <= hm1) & (u <= wm1);
        const uint32_t off = in ? __umul24((uint32_t)(int)v, W4) + ((uint32_t)(int)u << 2) : __umul24((uint32_t)hf, W4);
        const uint32_t poff = (uint32_t)__builtin_amdgcn_mov_dpp((int)off, kSwap, 0xF, 0xF, false);
        // even lane: the 16-byte-aligned window holding its own dword; it serves the odd partner when
        // the partner's dword lies in the same window
        const uint32_t a = off & ~15u;
        const uint32_t pd = poff - a, od = off - a;
        const bool wide = !odd && a + 16u <= bytes;
        const bool serves = wide && pd < 16u;
        // the DPP reads run with every lane active (under `odd && ...` they would run for the odd
        // lanes only, reading disabled even lanes)
        const int pserves = __builtin_amdgcn_mov_dpp((int)serves, kSwap, 0xF, 0xF, false);
        const bool served = odd && pserves;
        float mine = 0.f, partner = 0.f;
        if (wide) {
            const u32x4 q = __builtin_amdgcn_raw_buffer_load_b128(rs, a, 0, 0);
            mine = __uint_as_float(od == 0 ? q.x : od == 4 ? q.y : od == 8 ? q.z : q.w);
            partner = __uint_as_float(pd == 0 ? q.x : pd == 4 ? q.y : pd == 8 ? q.z : q.w);
        }
        const float got = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(partner), kSwap, 0xF, 0xF, false));
        if (!wide && !served) mine = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0));
        dv[k] = served ? got : mine;
        if ((k + 1) % ILP == 0) __builtin_amdgcn_sched_barrier(0);
    }
}

// ---- VALU-lean projection / update (PAIR = 2, 3) ---------------------------------------------------
// The same float operations as lean_gather / lean_update with fewer instructions around them:
//  * in-image test as two unsigned compares of the float bits: 0 <= u <= W - 1 holds exactly when
//    bits(u) <= bits(W - 1) for every u but -0.0 (sign bit) -- the host replaces a -0.0 principal
//    point by +0.0, which changes no u and no pixel (x + -0 = x + +0 unless x = -0, and (int)-0 =
//    (int)+0), so u = -0.0 cannot occur; NaN and negative values compare above the bound;
//  * min(sdf, trunc) as one v_min_f32: sdf comes out of a subtraction, so it is never a signalling
//    NaN and IEEE-mode v_min_f32 returns trunc for a NaN sdf, as fminf does (the compiler's fminf adds
//    a canonicalising v_max_f32 in front);
//  * (PAIR = 3) the zc range checked once per block and batch (block_zc_unsafe), not per voxel-frame.
// The depth read stays a gather by every lane through the raw view (out-of-image lanes read 0 past
// the end): reading under the in-image exec mask kept 8 lane masks live across the gathers, which
// the compiler spilled to VGPR booleans (3 VALU per voxel-frame) and made the update wait for all 8
// gathers.
template <int ZPER, int ILP = 1, bool ZCHK = true>
__device__ __forceinline__ void lean_gather_v(float (&dv)[ZPER], bool& bad, const FrameParams& fp,
                                              __amdgpu_buffer_rsrc_t rs, const float (&xs)[ZPER],
                                              const float (&ys)[ZPER], const float (&zs)[ZPER], uint32_t W4,
                                              uint32_t past_end, uint32_t hm1_bits, uint32_t wm1_bits) {
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
        if (ZCHK) bad |= (__float_as_uint(zc) - 0x2D800000u) > 0x30000000u;  // not 2^-36 <= zc <= 2^60
        const float inv_z = rcp_m(zc);
        const float u = fx * xc * inv_z + cx;
        const float v = fy * yc * inv_z + cy;
        const bool in = (__float_as_uint(v) <= hm1_bits) && (__float_as_uint(u) <= wm1_bits);
        const uint32_t off = in ? __umul24((uint32_t)(int)v, W4) + ((uint32_t)(int)u << 2) : past_end;
        dv[k] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0));
        if ((k + 1) % ILP == 0) __builtin_amdgcn_sched_barrier(0);
    }
}


// The zc range check of lean_gather (2^-36 <= zc <= 2^60, where rcp_m is exact) once per block and
// batch instead of per voxel-frame (PAIR = 3): thread (frame j = tid / 8, corner c = tid % 8) bounds
// zc at one corner of the block's voxel-coordinate box.  The voxel coordinates are the float values
// fl((float)i * voxel_size), monotone in i, so every voxel lies in the box of the corner values; the
// exact affine Z = x e8 + y e9 + z e10 + e11 takes its extremes over the box at the corners; the
// float32 evaluation (three products, three sums) differs from Z by at most gamma_4 A < 2^-21 A,
// A = max|x| |e8| + max|y| |e9| + max|z| |e10| + |e11| over the box.  A corner with Z - 2^-20 A <
// 2^-36 or Z + 2^-20 A > 2^60 (or NaN) marks the block bad: the exact fix-up launch redoes it.
template <int R>
__device__ __forceinline__ bool block_zc_unsafe_frame(int j, int c, const FrameParams* __restrict__ fps, int xb, int yb,
                                                      int zb, float voxel_size) {
    const FrameParams& fp = fps[j];
    const float xl = (float)(xb * R) * voxel_size, xh = (float)(xb * R + R - 1) * voxel_size;
    const float yl = (float)(yb * R) * voxel_size, yh = (float)(yb * R + R - 1) * voxel_size;
    const float zl = (float)(zb * R) * voxel_size, zh = (float)(zb * R + R - 1) * voxel_size;
    const double e8 = fp.ext[8], e9 = fp.ext[9], e10 = fp.ext[10], e11 = fp.ext[11];
    const double x = (c & 1) ? xh : xl, y = (c & 2) ? yh : yl, z = (c & 4) ? zh : zl;
    const double Z = x * e8 + y * e9 + z * e10 + e11;
    const double A = fmax(fabs((double)xl), fabs((double)xh)) * fabs(e8) +
                     fmax(fabs((double)yl), fabs((double)yh)) * fabs(e9) +
                     fmax(fabs((double)zl), fabs((double)zh)) * fabs(e10) + fabs(e11);
    const double err = A * 0x1p-20;
    return !(Z - err >= 0x1p-36 && Z + err <= 0x1p60);
}

template <int R>
__device__ __forceinline__ bool block_zc_unsafe(int tid, bmask_t mask, const FrameParams* __restrict__ fps, int xb,
                                                int yb, int zb, float voxel_size) {
    const int c = tid & 7;
    bool unsafe = false;
    for (int j = tid >> 3; j < kMaxBatch; j += 64)  // 512 threads: 64 frames x 8 corners per round
        if ((mask >> j) & 1) unsafe |= block_zc_unsafe_frame<R>(j, c, fps, xb, yb, zb, voxel_size);
    return unsafe;
}


// A/B: the round-2..4 lean integrate with all its measured variants (the product keeps k_integrate_lean with
// dword gathers and k_integrate_win).  Lean integrate, unit depth scale only (host: sdf_trunc in the division core's range).  Block per
// workgroup, voxels per lean_map<MAP>; every voxel of a block not handed off is written back.
// WPE: minimum waves per SIMD the register allocation must allow; ILP: voxel chains the scheduler
// may interleave (lean_gather / lean_update).

// PAIR (A/B library only, variant 6): the paired-lane gather of vbg_ab.hpp.
// FIXIN: a block whose operands leave the proven ranges is redone by the workgroup itself through the
// exact path (exact_block, not inlined: its registers stay out of the frame loop's allocation) instead of
// being handed to the fix-up launch -- no second launch behind every integrate.
template <int R, int NT>
__device__ __attribute__((noinline)) void exact_block_call(float2* __restrict__ vox, bool fresh, bmask_t mask, int xb,
                                                           int yb, int zb, float voxel_size,
                                                           const float* __restrict__ depths, int64_t HW, int W,
                                                           float hm1, float wm1, const FrameParams* __restrict__ fps,
                                                           const int64_t* __restrict__ depth_frame, float depth_max,
                                                           float sdf_trunc);
template <int R, int NT, int MAP = 0, int WPE = 1, int ILP = 1, int PAIR = 0, int DIV1 = 0, bool ZBLK = false,
          bool FIXIN = false>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(WPE, 8))) void k_integrate_lean_ab(
    const int32_t* __restrict__ list, const bmask_t* __restrict__ lmask, int32_t* __restrict__ bad_out,
    int* __restrict__ counters, int64_t list_cap, Table t, float2* __restrict__ pool, float voxel_size,
    const float* __restrict__ depths, int64_t HW, int H, int W, const FrameParams* __restrict__ fps,
    const int64_t* __restrict__ depth_frame, float depth_max, float sdf_trunc, int first_new, int grouped) {
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
    // grouped (k_xcd_order): the workgroups with blockIdx % 8 == g run group g (grid % 8 == 0)
    int64_t i = blockIdx.x, iend = n, step = gridDim.x;
    if (grouped) {
        const int g = blockIdx.x % kNumGroups;
        i = counters[kGroupBase + g] + blockIdx.x / kNumGroups;
        iend = counters[kGroupBase + g + 1];
        step = gridDim.x / kNumGroups;
    }
    for (; i < iend; i += step) {
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
            if constexpr (PAIR == 3 || ZBLK) {  // block-level zc range check (block_zc_unsafe): skip the frame loop
                static_assert(NT == 512, "one (frame, corner) per thread");
                if (__syncthreads_or(block_zc_unsafe<R>(tid, mask, fps, xb, yb, zb, voxel_size))) bad = true, m = 0;
            }
            while (m) {
                const int f = bm_ctz(m);
                m &= m - 1;
                float dv[ZPER];
                if constexpr (PAIR == 6 || PAIR == 7) {  // windows in two halves: <= 4 window loads in flight
                    constexpr int H2 = ZPER / 2;
                    const __amdgpu_buffer_rsrc_t rsf = frame_rsrc(depths + depth_frame[f] * HW, bytes);
                    constexpr int WB = PAIR == 6 ? 16 : 8;
                    lean_gather_w<ZPER, ILP, WB, true, 0, H2>(dv, bad, fps[f], rsf, xs, ys, zs, W4, bytes,
                                                              __float_as_uint(hm1), __float_as_uint(wm1));
                    __builtin_amdgcn_sched_barrier(0);
                    lean_update_v<ZPER, ILP, DIV1, 0, H2>(tw, dv, fps[f], xs, ys, zs, depth_max, sdf_trunc, y1t);
                    __builtin_amdgcn_sched_barrier(0);
                    lean_gather_w<ZPER, ILP, WB, true, H2, ZPER>(dv, bad, fps[f], rsf, xs, ys, zs, W4, bytes,
                                                                 __float_as_uint(hm1), __float_as_uint(wm1));
                    __builtin_amdgcn_sched_barrier(0);
                    lean_update_v<ZPER, ILP, DIV1, H2, ZPER>(tw, dv, fps[f], xs, ys, zs, depth_max, sdf_trunc, y1t);
                    continue;
                } else if constexpr (PAIR == 4 || PAIR == 5) {
                    lean_gather_w<ZPER, ILP, PAIR == 4 ? 16 : 8, !ZBLK>(dv, bad, fps[f], frame_rsrc(depths + depth_frame[f] * HW, bytes),
                                                                  xs, ys, zs, W4, bytes, __float_as_uint(hm1),
                                                                  __float_as_uint(wm1));
                    lean_update_v<ZPER, ILP, DIV1>(tw, dv, fps[f], xs, ys, zs, depth_max, sdf_trunc, y1t);
                    continue;
                } else if constexpr (PAIR == 2 || PAIR == 3) {
                    lean_gather_v<ZPER, ILP, PAIR == 2>(dv, bad, fps[f], frame_rsrc(depths + depth_frame[f] * HW, bytes),
                                                         xs, ys, zs, W4, bytes, __float_as_uint(hm1), __float_as_uint(wm1));
                    lean_update_v<ZPER, ILP, DIV1>(tw, dv, fps[f], xs, ys, zs, depth_max, sdf_trunc, y1t);
                    continue;
                } else if constexpr (PAIR) {
                    static_assert(MAP == 1, "pairs are the x-adjacent lanes of the brick map");
                    lean_gather_pair<ZPER, ILP>(dv, bad, fps[f], frame_rsrc(depths + depth_frame[f] * HW, bytes), xs,
                                                ys, zs, W4, hf, hm1, wm1, bytes);
                } else {
                    lean_gather<ZPER, ILP>(dv, bad, fps[f], frame_rsrc(depths + depth_frame[f] * HW, bytes), xs, ys,
                                           zs, W4, hf, hm1, wm1);
                }
                lean_update<ZPER, ILP>(tw, dv, fps[f], xs, ys, zs, depth_max, sdf_trunc, y1t);
            }
            if (__syncthreads_or(bad)) {  // block-uniform: the exact path redoes it from the pool
                if constexpr (FIXIN)
                    exact_block_call<R, NT>(pool + (int64_t)buf * R3, buf >= first_new, mask, xb, yb, zb, voxel_size,
                                            depths, HW, W, hm1, wm1, fps, depth_frame, depth_max, sdf_trunc);
                else if (tid == 0)
                    hand_off(bad_out, counters, list_cap, slot, mask);
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

// ---- A/B: k_integrate_win with a software-pipelined frame loop, 1024-thread workgroups, timing diagnostics -------------------------------
// k_integrate_lean<16, 512, brick, WPE, 2, 8-byte windows, FIXIN>'s arithmetic (lean_gather_w /
// lean_update_v: bit-identical), with the brick map generalised to NT threads and, for PIPE, the frame
// loop unrolled by two with the roles of two depth-register sets alternating: frame f_next's projection
// and window loads are issued BEFORE frame f's running-average update, so a wave keeps one frame's loads
// in flight while it updates the previous one (the plain loop issues frame f's loads and at once waits
// for them in frame f's update: nothing of f + 1 is in flight).  The per-voxel update order stays frame
// order.  NT = 512: 8 voxels per thread (+8 VGPRs for the second set); NT = 1024: 4 voxels per thread.
// Map: lane l of wave w owns x = l % 8 + 8 (w % 2), y = (l / 8) % 2 + 2 (w / 2), z = l / 16 (a wave's
// voxels k form an 8 x 2 x 4 brick); voxel k sits at (x, y + 8 (k / 4), z + 4 (k % 4)) for NT = 512
// and at (x, y, z + 4 k) for NT = 1024.

// DIAG (A/B library timing diagnostics, wrong results): 1 = the bare v_rcp for 1 / zc and 1 / (w + 1) and
// one product for s / sdf_trunc (about a third of the frame loop's VALU work gone); 2 = every frame's depth
// read from the batch's first frame (a 1.2 MB working set that stays in L2: the refetch of each XCD's
// frames from the MALL taken away).
// BF: bit 0 = branch-free window offsets, bit 1 = branch-free updates (lean_gather_w / lean_update_v DIAGV
// bits 1 / 2).
template <int NT, int WPE, int PIPE, int DIAG = 0, int BF = 0>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(WPE, 8))) void k_integrate_win_ab(
    const int32_t* __restrict__ list, const bmask_t* __restrict__ lmask, int* __restrict__ counters, int64_t list_cap,
    Table t, float2* __restrict__ pool, float voxel_size, const float* __restrict__ depths, int64_t HW, int H, int W,
    const FrameParams* __restrict__ fps, const int64_t* __restrict__ depth_frame, float depth_max, float sdf_trunc,
    int first_new) {
    constexpr int R = 16, R2 = R * R, R3 = R2 * R;
    constexpr int ZPER = R3 / NT;
    static_assert(NT == 512 || NT == 1024, "brick map for 512 or 1024 threads");
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
                // a block allocated by this batch (buffer >= first_new) starts at (0, 0)
                tw[k] = buf >= first_new ? make_float2(0.f, 0.f)
                                         : pool_load(vox, voff, (R * dy + R2 * dz) * (int)sizeof(float2));
                xs[k] = xs0;
                ys[k] = (float)(yb * R + vy + dy) * voxel_size;
                zs[k] = (float)(zb * R + vz + dz) * voxel_size;
                const float wv = tw[k].y;  // rcp_m(w + 1) is exact for integer w <= 2^23 + 64
                bad |= !(wv >= 0.0f && wv <= 0x1p23f - 64.0f && wv == __builtin_truncf(wv));
            }
            const int64_t f0 = depth_frame[bm_ctz(mask)];
            auto dframe = [&](int f) { return DIAG == 2 ? f0 : depth_frame[f]; };
            auto gather = [&](float (&dv)[ZPER], int f) {
                lean_gather_w<ZPER, 2, 8, true, 0, ZPER, (DIAG == 1 ? 1 : 0) | (BF << 1)>(dv, bad, fps[f],
                                                                   frame_rsrc(depths + dframe(f) * HW, bytes), xs, ys,
                                                                   zs, W4, bytes, hb, wb);
            };
            auto update = [&](const float (&dv)[ZPER], int f) {
                lean_update_v<ZPER, 2, 0, 0, ZPER, (DIAG == 1 ? 1 : 0) | (BF << 1)>(tw, dv, fps[f], xs, ys, zs, depth_max, sdf_trunc, y1t);
            };
            bmask_t m = mask;
            float da[ZPER];
            if constexpr (PIPE == 2) {
                // half-frame pipeline: the voxels in two halves h0 / h1 and one depth-register set; steady
                // state per frame f: gather h0(f), update h1(f_prev), gather h1(f), update h0(f) -- each
                // half's update runs while the other half's loads are in flight
                constexpr int H2 = ZPER / 2;
                auto g0 = [&](int f) {
                    lean_gather_w<ZPER, 2, 8, true, 0, H2, (DIAG == 1 ? 1 : 0) | (BF << 1)>(da, bad, fps[f],
                                                                     frame_rsrc(depths + dframe(f) * HW, bytes), xs, ys,
                                                                     zs, W4, bytes, hb, wb);
                };
                auto g1 = [&](int f) {
                    lean_gather_w<ZPER, 2, 8, true, H2, ZPER, (DIAG == 1 ? 1 : 0) | (BF << 1)>(da, bad, fps[f],
                                                                        frame_rsrc(depths + dframe(f) * HW, bytes), xs,
                                                                        ys, zs, W4, bytes, hb, wb);
                };
                auto u0 = [&](int f) {
                    lean_update_v<ZPER, 2, 0, 0, H2, (DIAG == 1 ? 1 : 0) | (BF << 1)>(tw, da, fps[f], xs, ys, zs, depth_max, sdf_trunc, y1t);
                };
                auto u1 = [&](int f) {
                    lean_update_v<ZPER, 2, 0, H2, ZPER, (DIAG == 1 ? 1 : 0) | (BF << 1)>(tw, da, fps[f], xs, ys, zs, depth_max, sdf_trunc, y1t);
                };
                int fp = bm_ctz(m);
                m &= m - 1;
                g0(fp);
                __builtin_amdgcn_sched_barrier(0);
                g1(fp);
                __builtin_amdgcn_sched_barrier(0);
                u0(fp);
                while (m) {
                    const int f = bm_ctz(m);
                    m &= m - 1;
                    __builtin_amdgcn_sched_barrier(0);
                    g0(f);
                    __builtin_amdgcn_sched_barrier(0);
                    u1(fp);
                    __builtin_amdgcn_sched_barrier(0);
                    g1(f);
                    __builtin_amdgcn_sched_barrier(0);
                    u0(f);
                    fp = f;
                }
                __builtin_amdgcn_sched_barrier(0);
                u1(fp);
            } else if constexpr (PIPE) {
                float db[ZPER];
                int fa = bm_ctz(m);
                m &= m - 1;
                gather(da, fa);
                for (;;) {
                    if (!m) {
                        update(da, fa);
                        break;
                    }
                    const int fb = bm_ctz(m);
                    m &= m - 1;
                    gather(db, fb);  // frame fb's loads in flight ...
                    __builtin_amdgcn_sched_barrier(0);
                    update(da, fa);  // ... while frame fa is applied
                    if (!m) {
                        update(db, fb);
                        break;
                    }
                    fa = bm_ctz(m);
                    m &= m - 1;
                    gather(da, fa);
                    __builtin_amdgcn_sched_barrier(0);
                    update(db, fb);
                }
            } else {
                while (m) {
                    const int f = bm_ctz(m);
                    m &= m - 1;
                    gather(da, f);
                    update(da, f);
                }
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

// ---- packed-FP32 integrate (R = 16, NT = 512) --------------------------------------------------------------
// k_integrate_win's float operations two voxels at a time: voxels (2p, 2p + 1) of a thread share x and y and
// differ in z, so their transform, projection, reciprocal corrections and running-average update map onto
// gfx950's packed FP32 instructions (v_pk_mul_f32 / v_pk_add_f32 / v_pk_fma_f32: two IEEE round-to-nearest
// results, exactly the scalar instructions' -- no contraction is introduced, the fma calls are the scalar
// code's own).  v_rcp, the float -> int conversions, the in-image tests and the window addressing stay scalar.
// Voxel state as pairs: tt[p] = (tsdf 2p, tsdf 2p+1), ww[p] = (weight 2p, weight 2p+1).
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 splat2(float a) { return (f32x2){a, a}; }
__device__ __forceinline__ f32x2 fma2(f32x2 a, f32x2 b, f32x2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f32x2 rcp_m2(f32x2 b) {  // rcp_m elementwise: v_rcp x 2, Markstein correction packed
    const f32x2 y0 = {__builtin_amdgcn_rcpf(b.x), __builtin_amdgcn_rcpf(b.y)};
    return fma2(fma2(-b, y0, splat2(1.0f)), y0, y0);
}

// Pairs [P0, P1): projection + 8-byte window read of both voxels of each pair (lean_gather_w's operations).
template <int NP, int P0, int P1>
__device__ __forceinline__ void pk_gather(float (&dv)[2 * NP], bool& bad, const FrameParams& fp,
                                          __amdgpu_buffer_rsrc_t rs, float xs0, const float (&ysp)[NP],
                                          const f32x2 (&zz)[NP], uint32_t W4, uint32_t past_end, uint32_t hb,
                                          uint32_t wb) {
    float e[12];
#pragma unroll
    for (int j = 0; j < 12; ++j) e[j] = fp.ext[j];
#pragma unroll
    for (int p = P0; p < P1; ++p) {
        const float ax = xs0 * e[0] + ysp[p] * e[1];  // shared by the pairs of one y (merged)
        const float ay = xs0 * e[4] + ysp[p] * e[5];
        const float az = xs0 * e[8] + ysp[p] * e[9];
        const f32x2 xc = (splat2(ax) + zz[p] * splat2(e[2])) + splat2(e[3]);
        const f32x2 yc = (splat2(ay) + zz[p] * splat2(e[6])) + splat2(e[7]);
        const f32x2 zc = (splat2(az) + zz[p] * splat2(e[10])) + splat2(e[11]);
        bad |= (__float_as_uint(zc.x) - 0x2D800000u) > 0x30000000u;  // not 2^-36 <= zc <= 2^60
        bad |= (__float_as_uint(zc.y) - 0x2D800000u) > 0x30000000u;
        const f32x2 inv_z = rcp_m2(zc);
        const f32x2 u = (splat2(fp.fx) * xc) * inv_z + splat2(fp.cx);
        const f32x2 v = (splat2(fp.fy) * yc) * inv_z + splat2(fp.cy);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const float uh = h ? u.y : u.x, vh = h ? v.y : v.x;
            const bool in = (__float_as_uint(vh) <= hb) && (__float_as_uint(uh) <= wb);
            const uint32_t off = in ? __umul24((uint32_t)(int)vh, W4) + ((uint32_t)(int)uh << 2) : past_end;
            const u32x2 q = __builtin_amdgcn_raw_buffer_load_b64(rs, off & ~7u, 0, 0);
            dv[2 * p + h] = __uint_as_float((off & 4u) ? q.y : q.x);
        }
        __builtin_amdgcn_sched_barrier(0);  // one pair's chain at a time (registers)
    }
}

// Pairs [P0, P1): lean_update_v's running-average update, both voxels of a pair in packed form; a pair is
// skipped when no lane updates either voxel (the scalar code's per-voxel branch, per pair).
template <int NP, int P0, int P1>
__device__ __forceinline__ void pk_update(f32x2 (&tt)[NP], f32x2 (&ww)[NP], const float (&dv)[2 * NP],
                                          const FrameParams& fp, float xs0, const float (&ysp)[NP],
                                          const f32x2 (&zz)[NP], float depth_max, float sdf_trunc, float y1t) {
    const float e8 = fp.ext[8], e9 = fp.ext[9], e10 = fp.ext[10], e11 = fp.ext[11];
#pragma unroll
    for (int p = P0; p < P1; ++p) {
        const float az = xs0 * e8 + ysp[p] * e9;
        const f32x2 zc = (splat2(az) + zz[p] * splat2(e10)) + splat2(e11);
        const f32x2 d = {dv[2 * p], dv[2 * p + 1]};
        const f32x2 sdf = d - zc;
        const bool up0 = !(d.x <= 0) && !(d.x > depth_max) && !(sdf.x < -sdf_trunc);
        const bool up1 = !(d.y <= 0) && !(d.y > depth_max) && !(sdf.y < -sdf_trunc);
        if (up0 || up1) {
            f32x2 s;
            asm("v_min_f32 %0, %1, %2" : "=v"(s.x) : "s"(sdf_trunc), "v"(sdf.x));
            asm("v_min_f32 %0, %1, %2" : "=v"(s.y) : "s"(sdf_trunc), "v"(sdf.y));
            const f32x2 T = splat2(sdf_trunc), Y = splat2(y1t);
            const f32x2 q0 = s * Y;
            const f32x2 q1 = fma2(fma2(-T, q0, s), Y, q0);
            const f32x2 sn = fma2(fma2(-T, q1, s), Y, q1);
            const f32x2 wgt = ww[p], wp = wgt + splat2(1.0f);
            const f32x2 nt = (wgt * tt[p] + sn) * rcp_m2(wp);
            tt[p].x = up0 ? nt.x : tt[p].x;
            tt[p].y = up1 ? nt.y : tt[p].y;
            ww[p].x = up0 ? wp.x : ww[p].x;
            ww[p].y = up1 ? wp.y : ww[p].y;
        }
        __builtin_amdgcn_sched_barrier(0);
    }
}

// The packed-FP32 kernel: k_integrate_win<512, WPE, PIPE in {0, 2}>'s structure over pk_gather / pk_update.
template <int WPE, int PIPE>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(WPE, 8))) void k_integrate_pk(
    const int32_t* __restrict__ list, const bmask_t* __restrict__ lmask, int* __restrict__ counters, int64_t list_cap,
    Table t, float2* __restrict__ pool, float voxel_size, const float* __restrict__ depths, int64_t HW, int H, int W,
    const FrameParams* __restrict__ fps, const int64_t* __restrict__ depth_frame, float depth_max, float sdf_trunc,
    int first_new) {
    constexpr int NT = 512, R = 16, R2 = R * R, R3 = R2 * R;
    constexpr int ZPER = R3 / NT, NP = ZPER / 2;
    const int64_t n = min((int64_t)counters[kListCount], list_cap);
    const float hm1 = (float)H - 1.0f, wm1 = (float)W - 1.0f;
    const uint32_t W4 = 4u * (uint32_t)W, bytes = 4u * (uint32_t)HW;
    const uint32_t hb = __float_as_uint(hm1), wb = __float_as_uint(wm1);
    const float y0t = __builtin_amdgcn_rcpf(sdf_trunc);
    const float y1t = __builtin_fmaf(__builtin_fmaf(-sdf_trunc, y0t, 1.0f), y0t, y0t);
    const int tid = threadIdx.x;
    const int l = tid & 63, w = tid >> 6;
    const int vx = (l & 7) + 8 * (w & 1), vy = ((l >> 3) & 1) + 2 * (w >> 1), vz = l >> 4;
    const uint32_t voff = 8u * (uint32_t)(vx + R * vy + R2 * vz);
    for (int64_t i = blockIdx.x; i < n; i += gridDim.x) {
        const int32_t slot = list[i];
        const int buf = __builtin_amdgcn_readfirstlane(t.vals[slot]);
        const bmask_t mask = readfirstlane_mask(lmask ? lmask[i] : bm_frames(t.mask[slot]));
        int xb, yb, zb;
        unpack_key(t.keys[slot], xb, yb, zb);
        if (buf >= 0 && mask) {
            const __amdgpu_buffer_rsrc_t vox = __builtin_amdgcn_make_buffer_rsrc(
                pool + (int64_t)buf * R3, (short)0, (int)(R3 * sizeof(float2)), 0x00020000);
            f32x2 tt[NP], ww[NP], zz[NP];
            float ysp[NP];
            bool bad = false;
            const float xs0 = (float)(xb * R + vx) * voxel_size;
#pragma unroll
            for (int p = 0; p < NP; ++p) {
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int k = 2 * p + h;
                    const int dy = win_dy<NT>(k), dz = win_dz<NT>(k);
                    const float2 v = buf >= first_new ? make_float2(0.f, 0.f)
                                                      : pool_load(vox, voff, (R * dy + R2 * dz) * (int)sizeof(float2));
                    if (h) tt[p].y = v.x, ww[p].y = v.y, zz[p].y = (float)(zb * R + vz + dz) * voxel_size;
                    else tt[p].x = v.x, ww[p].x = v.y, zz[p].x = (float)(zb * R + vz + dz) * voxel_size;
                    bad |= !(v.y >= 0.0f && v.y <= 0x1p23f - 64.0f && v.y == __builtin_truncf(v.y));
                }
                ysp[p] = (float)(yb * R + vy + win_dy<NT>(2 * p)) * voxel_size;
            }
            auto frs = [&](int f) { return frame_rsrc(depths + depth_frame[f] * HW, bytes); };
            bmask_t m = mask;
            float da[ZPER];
            if constexpr (PIPE == 2) {
                constexpr int H2 = NP / 2;
                int fp = bm_ctz(m);
                m &= m - 1;
                pk_gather<NP, 0, H2>(da, bad, fps[fp], frs(fp), xs0, ysp, zz, W4, bytes, hb, wb);
                pk_gather<NP, H2, NP>(da, bad, fps[fp], frs(fp), xs0, ysp, zz, W4, bytes, hb, wb);
                pk_update<NP, 0, H2>(tt, ww, da, fps[fp], xs0, ysp, zz, depth_max, sdf_trunc, y1t);
                while (m) {
                    const int f = bm_ctz(m);
                    m &= m - 1;
                    pk_gather<NP, 0, H2>(da, bad, fps[f], frs(f), xs0, ysp, zz, W4, bytes, hb, wb);
                    pk_update<NP, H2, NP>(tt, ww, da, fps[fp], xs0, ysp, zz, depth_max, sdf_trunc, y1t);
                    pk_gather<NP, H2, NP>(da, bad, fps[f], frs(f), xs0, ysp, zz, W4, bytes, hb, wb);
                    pk_update<NP, 0, H2>(tt, ww, da, fps[f], xs0, ysp, zz, depth_max, sdf_trunc, y1t);
                    fp = f;
                }
                pk_update<NP, H2, NP>(tt, ww, da, fps[fp], xs0, ysp, zz, depth_max, sdf_trunc, y1t);
            } else {
                while (m) {
                    const int f = bm_ctz(m);
                    m &= m - 1;
                    pk_gather<NP, 0, NP>(da, bad, fps[f], frs(f), xs0, ysp, zz, W4, bytes, hb, wb);
                    pk_update<NP, 0, NP>(tt, ww, da, fps[f], xs0, ysp, zz, depth_max, sdf_trunc, y1t);
                }
            }
            if (__syncthreads_or(bad)) {
                exact_block_call<R, NT>(pool + (int64_t)buf * R3, buf >= first_new, mask, xb, yb, zb, voxel_size, depths,
                                        HW, W, hm1, wm1, fps, depth_frame, depth_max, sdf_trunc);
            } else {
#pragma unroll
                for (int k = 0; k < ZPER; ++k) {
                    const f32x2 a = tt[k >> 1], b = ww[k >> 1];
                    pool_store(vox, voff, (R * win_dy<NT>(k) + R2 * win_dz<NT>(k)) * (int)sizeof(float2),
                               (k & 1) ? make_float2(a.y, b.y) : make_float2(a.x, b.x));
                }
            }
        }
        __syncthreads();
        if (tid == 0) t.mask[slot] = 0;
    }
}

// ---- A/B: the round-4 default's exact source (lean_gather_w / lean_update_v as of round 4, before the
// round-5 restructuring of the window offset and update), for the same-process comparison (variant 44)
template <int ZPER, int ILP = 1, int WIN = 16, bool ZCHK = true, int K0 = 0, int K1 = ZPER>
__device__ __forceinline__ void lean_gather_w_r4(float (&dv)[ZPER], bool& bad, const FrameParams& fp,
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
        const float inv_z = rcp_m(zc);
        const float u = fx * xc * inv_z + cx;
        const float v = fy * yc * inv_z + cy;
        const bool in = (__float_as_uint(v) <= hm1_bits) && (__float_as_uint(u) <= wm1_bits);
        const uint32_t off = in ? __umul24((uint32_t)(int)v, W4) + ((uint32_t)(int)u << 2) : past_end;
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
template <int ZPER, int ILP = 1, int DIV1 = 0, int K0 = 0, int K1 = ZPER>
__device__ __forceinline__ void lean_update_v_r4(float2 (&tw)[ZPER], const float (&dv)[ZPER], const FrameParams& fp,
                                              const float (&xs)[ZPER], const float (&ys)[ZPER],
                                              const float (&zs)[ZPER], float depth_max, float sdf_trunc, float y1t) {
    const float e8 = fp.ext[8], e9 = fp.ext[9], e10 = fp.ext[10], e11 = fp.ext[11];
#pragma unroll
    for (int k = K0; k < K1; ++k) {
        const float az = xs[k] * e8 + ys[k] * e9;
        const float zc = (az + zs[k] * e10) + e11;
        const float d = dv[k];
        const float sdf = d - zc;
        if (!(d <= 0) && !(d > depth_max) && !(sdf < -sdf_trunc)) {
            float s;
            asm("v_min_f32 %0, %1, %2" : "=v"(s) : "s"(sdf_trunc), "v"(sdf));
            const float q0 = s * y1t;
            const float q1 = __builtin_fmaf(__builtin_fmaf(-sdf_trunc, q0, s), y1t, q0);
            const float sn = DIV1 ? q1 : __builtin_fmaf(__builtin_fmaf(-sdf_trunc, q1, s), y1t, q1);
            const float wgt = tw[k].y, wp = wgt + 1;
            tw[k].x = (wgt * tw[k].x + sn) * rcp_m(wp);
            tw[k].y = wp;
        }
        if ((k + 1) % ILP == 0) __builtin_amdgcn_sched_barrier(0);
    }
}


template <int WPE>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(WPE, 8))) void k_integrate_win_r4(
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
                lean_gather_w_r4<ZPER, 2, 8>(dv, bad, fps[f], frame_rsrc(depths + depth_frame[f] * HW, bytes), xs, ys, zs,
                                          W4, bytes, hb, wb);
                lean_update_v_r4<ZPER, 2, 0>(tw, dv, fps[f], xs, ys, zs, depth_max, sdf_trunc, y1t);
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


// ---- A/B: lane-level tile proofs (verdict r05 item 3) ------------------------------------------------------
// Per 8 x 4 pixel tile of every batch frame, an 8-byte record (k_tile_records): bit p of word 0 = pixel
// (p % 8, p / 8) of the tile passes the update's depth test !(d <= 0) && !(d > depth_max) (NaN passes it),
// word 1 = lo | hi << 16: binary16 bounds, lo <= every valid non-NaN depth of the tile (rounded down; +inf
// if none), hi >= every one of them (rounded up; -inf if none, +inf if the tile holds a NaN).  In the frame
// loop a lane reads its tile's record first (lanes of a wave mostly share one or two tiles) and is decided
// without its pixel when
//   bit 0                     -> no update (the update's own depth test fails): depth 0 stands in;
//   fl(lo - zc) >= sdf_trunc  -> sdf >= sdf_trunc for every valid pixel of the tile (monotone rounding), so
//                                s = sdf_trunc: a NaN depth stands in, which takes exactly that update;
//   fl(hi - zc) < -sdf_trunc  -> sdf < -sdf_trunc: no update (depth 0).
// Only the other lanes issue the 8-byte window read (exec-masked: a wave with none skips the load).  The
// running-average update is lean_update_v unchanged, so the volume is bit-identical to k_integrate_win's.
// tools/tile_proof_stats.py estimated 36 % of in-image lane-frames decided, 21 % of wave slots without a
// pixel read, 0.66x the distinct windows, at the cost of one more (mostly one-address) load per voxel-frame.
__device__ __forceinline__ uint32_t half_bits_down(float x) {  // binary16 bits of the largest half <= x (x >= 0 or +-inf)
    if (!(x < 65504.0f)) return x == __builtin_inff() ? 0x7C00u : 0x7BFFu;
    const _Float16 h = (_Float16)x;
    uint32_t b = (uint32_t)__builtin_bit_cast(uint16_t, h);
    if ((float)h > x) b = b == 0 ? 0x8001u : b - 1;  // x >= 0: only finite positive values round up
    return b;
}
__device__ __forceinline__ uint32_t half_bits_up(float x) {  // binary16 bits of the smallest half >= x (x >= 0 or +-inf)
    if (x == -__builtin_inff()) return 0xFC00u;
    if (!(x <= 65504.0f)) return 0x7C00u;
    const _Float16 h = (_Float16)x;
    uint32_t b = (uint32_t)__builtin_bit_cast(uint16_t, h);
    if ((float)h < x) b = b + 1;  // x >= 0 here: the next half up (65504 rounds to itself)
    return b;
}
__device__ __forceinline__ float half_from_bits(uint32_t b) {
    return (float)__builtin_bit_cast(_Float16, (uint16_t)b);
}

// One wave per two tiles (lanes 0-31 / 32-63), 8 tiles per 256-thread workgroup; blockIdx.y = batch frame.
__global__ __launch_bounds__(256) void k_tile_records(const float* __restrict__ depths, int64_t HW, int H, int W,
                                                      const int64_t* __restrict__ depth_frame, float depth_max,
                                                      int TW, int TH, uint2* __restrict__ rec) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int tile = (blockIdx.x * 4 + wave) * 2 + (lane >> 5);
    const int p = lane & 31;
    const int ntiles = TW * TH;
    const int tx = tile % TW, ty = tile / TW;
    const int px = tx * 8 + (p & 7), py = ty * 4 + (p >> 3);
    const bool in = tile < ntiles && px < W && py < H;
    const float d = in ? depths[depth_frame[blockIdx.y] * HW + (int64_t)py * W + px] : 0.0f;
    const bool valid = in && !(d <= 0.0f) && !(d > depth_max);
    const bool fin = valid && d == d;
    const uint64_t vb = __ballot(valid), nb = __ballot(valid && d != d);
    float lo = fin ? d : __builtin_inff(), hi = fin ? d : -__builtin_inff();
#pragma unroll
    for (int o = 1; o < 32; o <<= 1) {
        lo = __builtin_fminf(lo, __shfl_xor(lo, o));
        hi = __builtin_fmaxf(hi, __shfl_xor(hi, o));
    }
    if (p == 0 && tile < ntiles) {
        const uint32_t half = lane >> 5;
        const uint32_t m = (uint32_t)(vb >> (32 * half));
        if ((uint32_t)(nb >> (32 * half))) hi = __builtin_inff();
        rec[(int64_t)blockIdx.y * ntiles + tile] = make_uint2(m, half_bits_down(lo) | (half_bits_up(hi) << 16));
    }
}

// lean_gather_w<ZPER, 2, 8> with the tile proofs in front of the window read.
template <int ZPER, int BF = 0>
__device__ __forceinline__ void tp_gather(float (&dv)[ZPER], bool& bad, const FrameParams& fp,
                                          __amdgpu_buffer_rsrc_t rs, __amdgpu_buffer_rsrc_t rr,
                                          const float (&xs)[ZPER], const float (&ys)[ZPER], const float (&zs)[ZPER],
                                          uint32_t W4, uint32_t past_end, uint32_t rec_end, uint32_t TW8,
                                          uint32_t hm1_bits, uint32_t wm1_bits, float sdf_trunc) {
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
        bad |= (__float_as_uint(zc) - 0x2D800000u) > 0x30000000u;
        const float inv_z = rcp_m(zc);
        const float u = fx * xc * inv_z + cx;
        const float v = fy * yc * inv_z + cy;
        const bool in = (__float_as_uint(v) <= hm1_bits) && (__float_as_uint(u) <= wm1_bits);
        const uint32_t ui = (uint32_t)(int)u, vi = (uint32_t)(int)v;
        const uint32_t roff = in ? __umul24(vi >> 2, TW8) + ((ui >> 3) << 3) : rec_end;
        const u32x2 r = __builtin_amdgcn_raw_buffer_load_b64(rr, roff, 0, 0);
        const bool valid = (r.x >> (((vi & 3u) << 3) | (ui & 7u))) & 1u;  // out of the image: r = 0
        const bool clamp = valid && (half_from_bits(r.y & 0xFFFFu) - zc >= sdf_trunc);
        const bool behind = valid && (half_from_bits(r.y >> 16) - zc < -sdf_trunc);
        float d = clamp ? __builtin_nanf("") : 0.0f;
        if constexpr (BF) {  // every lane issues the read; decided lanes read past the end (one address)
            const bool need = valid && !clamp && !behind;
            const uint32_t off = need ? __umul24(vi, W4) + (ui << 2) : past_end;
            const u32x2 q = __builtin_amdgcn_raw_buffer_load_b64(rs, off & ~7u, 0, 0);
            d = need ? __uint_as_float((off & 4u) ? q.y : q.x) : d;
        } else if (valid && !clamp && !behind) {
            const uint32_t off = __umul24(vi, W4) + (ui << 2);
            const u32x2 q = __builtin_amdgcn_raw_buffer_load_b64(rs, off & ~7u, 0, 0);
            d = __uint_as_float((off & 4u) ? q.y : q.x);
        }
        dv[k] = d;
        if ((k + 1) % 2 == 0) __builtin_amdgcn_sched_barrier(0);
    }
}

// TWO_PHASE: the 8 voxels' record loads issued together first (one memory round trip for all of them),
// then the projection recomputed (an empty asm hides its operands, so the compiler does not keep the first
// pass's values live) for the decisions and the window reads.
template <int ZPER, int BF = 0>
__device__ __forceinline__ void tp_gather2(float (&dv)[ZPER], bool& bad, const FrameParams& fp,
                                           __amdgpu_buffer_rsrc_t rs, __amdgpu_buffer_rsrc_t rr,
                                           const float (&xs)[ZPER], const float (&ys)[ZPER], const float (&zs)[ZPER],
                                           uint32_t W4, uint32_t past_end, uint32_t rec_end, uint32_t TW8,
                                           uint32_t hm1_bits, uint32_t wm1_bits, float sdf_trunc) {
    float e[12];
#pragma unroll
    for (int j = 0; j < 12; ++j) e[j] = fp.ext[j];
    const float fx = fp.fx, fy = fp.fy, cx = fp.cx, cy = fp.cy;
    u32x2 r[ZPER];
#pragma unroll
    for (int k = 0; k < ZPER; ++k) {
        const float xc = ((xs[k] * e[0] + ys[k] * e[1]) + zs[k] * e[2]) + e[3];
        const float yc = ((xs[k] * e[4] + ys[k] * e[5]) + zs[k] * e[6]) + e[7];
        const float zc = ((xs[k] * e[8] + ys[k] * e[9]) + zs[k] * e[10]) + e[11];
        const float inv_z = rcp_m(zc);
        const float u = fx * xc * inv_z + cx;
        const float v = fy * yc * inv_z + cy;
        const bool in = (__float_as_uint(v) <= hm1_bits) && (__float_as_uint(u) <= wm1_bits);
        const uint32_t roff = in ? __umul24((uint32_t)(int)v >> 2, TW8) + (((uint32_t)(int)u >> 3) << 3) : rec_end;
        r[k] = __builtin_amdgcn_raw_buffer_load_b64(rr, roff, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int k = 0; k < ZPER; ++k) {
        float x = xs[k], y = ys[k], z = zs[k];
        asm volatile("" : "+v"(x), "+v"(y), "+v"(z));
        const float ax = x * e[0] + y * e[1];
        const float ay = x * e[4] + y * e[5];
        const float az = x * e[8] + y * e[9];
        const float xc = (ax + z * e[2]) + e[3];
        const float yc = (ay + z * e[6]) + e[7];
        const float zc = (az + z * e[10]) + e[11];
        bad |= (__float_as_uint(zc) - 0x2D800000u) > 0x30000000u;
        const float inv_z = rcp_m(zc);
        const float u = fx * xc * inv_z + cx;
        const float v = fy * yc * inv_z + cy;
        const uint32_t ui = (uint32_t)(int)u, vi = (uint32_t)(int)v;
        const bool valid = (r[k].x >> (((vi & 3u) << 3) | (ui & 7u))) & 1u;  // out of the image: r = 0
        const bool clamp = valid && (half_from_bits(r[k].y & 0xFFFFu) - zc >= sdf_trunc);
        const bool behind = valid && (half_from_bits(r[k].y >> 16) - zc < -sdf_trunc);
        float d = clamp ? __builtin_nanf("") : 0.0f;
        if constexpr (BF) {
            const bool need = valid && !clamp && !behind;
            const uint32_t off = need ? __umul24(vi, W4) + (ui << 2) : past_end;
            const u32x2 q = __builtin_amdgcn_raw_buffer_load_b64(rs, off & ~7u, 0, 0);
            d = need ? __uint_as_float((off & 4u) ? q.y : q.x) : d;
        } else if (valid && !clamp && !behind) {
            const uint32_t off = __umul24(vi, W4) + (ui << 2);
            const u32x2 q = __builtin_amdgcn_raw_buffer_load_b64(rs, off & ~7u, 0, 0);
            d = __uint_as_float((off & 4u) ? q.y : q.x);
        }
        dv[k] = d;
        if ((k + 1) % 2 == 0) __builtin_amdgcn_sched_barrier(0);
    }
}

template <int WPE, int TWO_PHASE = 0, int BF = 0>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(WPE, 8))) void k_integrate_tp(
    const int32_t* __restrict__ list, const bmask_t* __restrict__ lmask, int* __restrict__ counters, int64_t list_cap,
    Table t, float2* __restrict__ pool, float voxel_size, const float* __restrict__ depths, int64_t HW, int H, int W,
    const FrameParams* __restrict__ fps, const int64_t* __restrict__ depth_frame, float depth_max, float sdf_trunc,
    int first_new, const uint2* __restrict__ recs, int TW, int TH) {
    constexpr int NT = 512, R = 16, R2 = R * R, R3 = R2 * R;
    constexpr int ZPER = R3 / NT;
    const int64_t n = min((int64_t)counters[kListCount], list_cap);
    const float hm1 = (float)H - 1.0f, wm1 = (float)W - 1.0f;
    const uint32_t W4 = 4u * (uint32_t)W, bytes = 4u * (uint32_t)HW;
    const uint32_t rec_bytes = 8u * (uint32_t)(TW * TH), TW8 = 8u * (uint32_t)TW;
    const uint32_t hb = __float_as_uint(hm1), wb = __float_as_uint(wm1);
    const float y0t = __builtin_amdgcn_rcpf(sdf_trunc);
    const float y1t = __builtin_fmaf(__builtin_fmaf(-sdf_trunc, y0t, 1.0f), y0t, y0t);
    const int tid = threadIdx.x;
    const int l = tid & 63, w = tid >> 6;
    const int vx = (l & 7) + 8 * (w & 1), vy = ((l >> 3) & 1) + 2 * (w >> 1), vz = l >> 4;
    const uint32_t voff = 8u * (uint32_t)(vx + R * vy + R2 * vz);
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
                tw[k] = buf >= first_new ? make_float2(0.f, 0.f)
                                         : pool_load(vox, voff, (R * dy + R2 * dz) * (int)sizeof(float2));
                xs[k] = xs0;
                ys[k] = (float)(yb * R + vy + dy) * voxel_size;
                zs[k] = (float)(zb * R + vz + dz) * voxel_size;
                const float wv = tw[k].y;
                bad |= !(wv >= 0.0f && wv <= 0x1p23f - 64.0f && wv == __builtin_truncf(wv));
            }
            bmask_t m = mask;
            while (m) {
                const int f = bm_ctz(m);
                m &= m - 1;
                float dv[ZPER];
                const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
                    const_cast<uint2*>(recs + (int64_t)f * TW * TH), (short)0, (int)rec_bytes, 0x00020000);
                if constexpr (TWO_PHASE)
                    tp_gather2<ZPER, BF>(dv, bad, fps[f], frame_rsrc(depths + depth_frame[f] * HW, bytes), rr, xs, ys,
                                         zs, W4, bytes, rec_bytes, TW8, hb, wb, sdf_trunc);
                else
                    tp_gather<ZPER, BF>(dv, bad, fps[f], frame_rsrc(depths + depth_frame[f] * HW, bytes), rr, xs, ys, zs,
                                        W4, bytes, rec_bytes, TW8, hb, wb, sdf_trunc);
                lean_update_v<ZPER, 2, 0>(tw, dv, fps[f], xs, ys, zs, depth_max, sdf_trunc, y1t);
            }
            if (__syncthreads_or(bad)) {
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

// ---- round 6: register-pressure forms of k_integrate_win (A/B variants 51-58) ---------------------------------
// The shipped kernel at 72 VGPRs keeps 7 of its 8 voxels' (tsdf, weight) pairs in scratch inside the frame
// loop (14 scratch loads / stores per wave-frame beside the 8 window reads), and a 512-thread workgroup gets 3
// workgroups per CU -- 6 waves per SIMD -- whether the budget allows 6 or 7.  MODE bit 0: the frame's 8 voxels
// in two halves (gather 0-3, update 0-3, gather 4-7, update 4-7: half the window reads in flight, half the
// registers for them); bit 1: no in-kernel exact path (a block outside the proven ranges is handed to the exact
// fix-up launch, hand_off, like k_integrate_lean) -- no call, so no registers saved across one; bit 2: a
// workgroup barrier after every frame.
template <int WPE, int MODE>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(WPE, 8))) void k_integrate_wx(
    const int32_t* __restrict__ list, const bmask_t* __restrict__ lmask, int32_t* __restrict__ bad_out,
    int* __restrict__ counters, int64_t list_cap, Table t, float2* __restrict__ pool, float voxel_size,
    const float* __restrict__ depths, int64_t HW, int H, int W, const FrameParams* __restrict__ fps,
    const int64_t* __restrict__ depth_frame, float depth_max, float sdf_trunc, int first_new) {
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
    const uint32_t voff = 8u * (uint32_t)(vx + R * vy + R2 * vz);
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
                tw[k] = buf >= first_new ? make_float2(0.f, 0.f)
                                         : pool_load(vox, voff, (R * dy + R2 * dz) * (int)sizeof(float2));
                xs[k] = xs0;
                ys[k] = (float)(yb * R + vy + dy) * voxel_size;
                zs[k] = (float)(zb * R + vz + dz) * voxel_size;
                const float wv = tw[k].y;
                bad |= !(wv >= 0.0f && wv <= 0x1p23f - 64.0f && wv == __builtin_truncf(wv));
            }
            bmask_t m = mask;
            while (m) {
                const int f = bm_ctz(m);
                m &= m - 1;
                float dv[ZPER];
                const __amdgpu_buffer_rsrc_t rs = frame_rsrc(depths + depth_frame[f] * HW, bytes);
                if constexpr ((MODE & 1) != 0) {
                    lean_gather_w<ZPER, 2, 8, true, 0, ZPER / 2>(dv, bad, fps[f], rs, xs, ys, zs, W4, bytes, hb, wb);
                    lean_update_v<ZPER, 2, 0, 0, ZPER / 2>(tw, dv, fps[f], xs, ys, zs, depth_max, sdf_trunc, y1t);
                    lean_gather_w<ZPER, 2, 8, true, ZPER / 2, ZPER>(dv, bad, fps[f], rs, xs, ys, zs, W4, bytes, hb, wb);
                    lean_update_v<ZPER, 2, 0, ZPER / 2, ZPER>(tw, dv, fps[f], xs, ys, zs, depth_max, sdf_trunc, y1t);
                } else {
                    lean_gather_w<ZPER, 2, 8>(dv, bad, fps[f], rs, xs, ys, zs, W4, bytes, hb, wb);
                    lean_update_v<ZPER, 2, 0>(tw, dv, fps[f], xs, ys, zs, depth_max, sdf_trunc, y1t);
                }
                // MODE bit 2: the workgroup's 8 waves kept in step frame by frame (they read the same image
                // region of the same frame, so the L1 can serve one wave's windows to the next)
                if constexpr ((MODE & 4) != 0) __syncthreads();
            }
            if (__syncthreads_or(bad)) {
                if constexpr ((MODE & 2) != 0) {
                    if (tid == 0) hand_off(bad_out, counters, list_cap, slot, mask);
                } else {
                    exact_block_call<R, NT>(pool + (int64_t)buf * R3, buf >= first_new, mask, xb, yb, zb, voxel_size,
                                            depths, HW, W, hm1, wm1, fps, depth_frame, depth_max, sdf_trunc);
                }
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


}  // namespace mqr

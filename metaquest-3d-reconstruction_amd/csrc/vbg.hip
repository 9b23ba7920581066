// vbg.hip -- host side of the HBM-resident voxel-block TSDF volume: block hash, touch,
// integrate, export/import and the multi-GPU pack/unpack.  Replaces Open3D 0.19's
// VoxelBlockGrid (reference call sites: scripts/processing/reconstruction/utils/o3d_utils.py:170-229).
//
// Data layout in HBM (one volume):
//   pool   [pool_cap][R^3] float2 (tsdf, weight), voxel [z][y][x] inside a block -> 32 KiB/block at R=16
//   bkeys  [pool_cap] packed block key of each buffer (for extraction / export)
//   table  keys u64 / vals i32 / mask u64 x2 (batch parity), open addressing, capacity >= 2x live keys
//   lists  slots touched by the current batch (appended once per batch, on first touch), x2
//
// Per batch of <= 127 frames (the first of a call a full batch too; variant bits 21-23 shorten it for A/Bs): k_touch
// (two stride-4 pixels per thread per frame, 4 ray samples,
// hash insert, per-slot frame bitmask) -> host reads the batch counters (pool growth, empty-frame
// error) -> k_integrate (one workgroup per touched block, every voxel applies that block's frames
// in frame order = bit-identical to sequential per-frame integration).
// touch(b+1) runs on a second stream while integrate(b) runs (double-buffered batch state).
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <unordered_map>

#include "mqr_common.hpp"
#include "vbg_kernels.hpp"
#if MQR_AB
#include "vbg_ab.hpp"
#endif

namespace mqr {

static thread_local std::string g_err;
void set_error(const std::string& msg) { g_err = msg; }
const char* get_error() { return g_err.c_str(); }

// mqr_set_stream: the calling thread's caller stream (nullptr = the null stream) and one ordering
// event per device.  The event is recorded with a device-scope release: the producer (a kernel or a
// copy the caller enqueued) and the consumer (a library kernel) are on the same device, and the
// consumer's dispatch acquires as every kernel launch does.  The events are never destroyed: a
// thread-exit destructor could run after the HIP runtime has been torn down.
static constexpr int kOrderDevices = 64;
static thread_local hipStream_t t_caller_stream = nullptr;
static thread_local hipEvent_t t_order_ev[kOrderDevices] = {};

hipStream_t caller_stream() { return t_caller_stream; }

int order_after_caller(int device, hipStream_t a, hipStream_t b) {
    MQR_REQUIRE(device >= 0 && device < kOrderDevices, "device index out of range");
    if (t_caller_stream) {
        hipDevice_t sd = -1;
        if (hipStreamGetDevice(t_caller_stream, &sd) != hipSuccess) {
            (void)hipGetLastError();
            set_error("the caller stream given to mqr_set_stream is not a valid stream (destroyed?)");
            return 2;
        }
        if (sd != device) {
            // a stream of another device (e.g. torch's current stream on cuda:0 while the call works on a
            // volume on device 1): no device-side wait across devices -- drain it on the host instead
            MQR_CHECK_HIP(hipStreamSynchronize(t_caller_stream));
            return 0;
        }
    }
    hipEvent_t& e = t_order_ev[device];
    if (!e) MQR_CHECK_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventDisableSystemFence));
    if (hipEventRecord(e, t_caller_stream) != hipSuccess) {
        (void)hipGetLastError();  // not left behind for a later launch check
        set_error("the caller stream given to mqr_set_stream cannot be waited on from device " +
                  std::to_string(device) + " (a stream of another device, or destroyed)");
        return 2;
    }
    MQR_CHECK_HIP(hipStreamWaitEvent(a, e, 0));
    if (b) MQR_CHECK_HIP(hipStreamWaitEvent(b, e, 0));
    return 0;
}

void make_frame_params(const double* K, const double* T, FrameParams* fp) {
    fp->fx = (float)K[0];
    fp->fy = (float)K[4];
    fp->cx = (float)K[2];
    fp->cy = (float)K[5];
    // a -0.0 principal point becomes +0.0: u = p + c is the same for both unless p = -0, where it is
    // -0 or +0, the same pixel; then no u or v is -0.0 (lean_gather_v's in-image test on float bits)
    if (fp->cx == 0.0f) fp->cx = 0.0f;
    if (fp->cy == 0.0f) fp->cy = 0.0f;
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

// ------------------------------------------------------------------ host helpers
static int64_t next_pow2(int64_t x) {
    int64_t p = 1024;
    while (p < x) p <<= 1;
    return p;
}

static int alloc_table(Table& t, int64_t cap, hipStream_t s) {
    MQR_CHECK_HIP(hipMalloc(&t.keys, sizeof(uint64_t) * cap));
    MQR_CHECK_HIP(hipMalloc(&t.vals, sizeof(int32_t) * cap));
    MQR_CHECK_HIP(hipMalloc(&t.mask, sizeof(bmask_t) * cap));
    MQR_CHECK_HIP(hipMemsetAsync(t.keys, 0xff, sizeof(uint64_t) * cap, s));
    MQR_CHECK_HIP(hipMemsetAsync(t.vals, 0xff, sizeof(int32_t) * cap, s));
    MQR_CHECK_HIP(hipMemsetAsync(t.mask, 0, sizeof(bmask_t) * cap, s));
    t.cap = cap;
    return 0;
}

static void free_table(Table& t) {
    if (t.keys) (void)hipFree(t.keys);
    if (t.vals) (void)hipFree(t.vals);
    if (t.mask) (void)hipFree(t.mask);
    t = Table{};
}

int sync_all(mqr_vbg* v) {
    MQR_CHECK_HIP(hipStreamSynchronize(v->stream2));
    MQR_CHECK_HIP(hipStreamSynchronize(v->stream));
    v->int_pending[0] = v->int_pending[1] = false;
    return 0;
}

int order_after_integrate(mqr_vbg* v) {
    for (int p = 0; p < 2; ++p)
        if (v->int_pending[p]) MQR_CHECK_HIP(hipStreamWaitEvent(v->stream, v->int_done[p], 0));
    return 0;
}

int order_caller_after_integrate(mqr_vbg* v) {
    hipStream_t cs = t_caller_stream;
    if (cs) {
        hipDevice_t sd = -1;
        if (hipStreamGetDevice(cs, &sd) != hipSuccess || sd != v->device) {
            (void)hipGetLastError();
            return sync_all(v);  // a stream of another device (or none valid): no device-side wait -- drain
        }
    }
    // both parities: integrates run in order on their stream, but a call of one batch leaves only its
    // own parity pending and an earlier call may have left the other
    for (int p = 0; p < 2; ++p)
        if (v->int_pending[p]) MQR_CHECK_HIP(hipStreamWaitEvent(cs, v->int_done[p], 0));
    return 0;
}

static int ensure_lists(mqr_vbg* v, int64_t cap) {
    if (v->list_cap >= cap) return 0;
    if (sync_all(v)) return 1;
    for (int p = 0; p < 2; ++p) {
        if (v->lists[p]) MQR_CHECK_HIP(hipFree(v->lists[p]));
        if (v->lpt[p]) MQR_CHECK_HIP(hipFree(v->lpt[p]));
        v->lists[p] = v->lpt[p] = nullptr;
        MQR_CHECK_HIP(hipMalloc(&v->lists[p], sizeof(int32_t) * cap));
        // slots, then their masks, then k_xcd_order's group byte per entry
        MQR_CHECK_HIP(hipMalloc(&v->lpt[p], (sizeof(int32_t) + sizeof(bmask_t) + 1) * cap));
        if (v->bad[p]) MQR_CHECK_HIP(hipFree(v->bad[p]));
        v->bad[p] = nullptr;
        MQR_CHECK_HIP(hipMalloc(&v->bad[p], (sizeof(int32_t) + sizeof(bmask_t)) * cap));  // slots, then masks
    }
    v->list_cap = cap;
    return 0;
}

// Grow the main table to hold `live` keys at <= 50 % load.  Only between batches: waits for any
// in-flight integrate (its lists hold slot indices of the old table) and all masks are zero then.
static int ensure_table(mqr_vbg* v, int64_t live) {
    const int64_t want = next_pow2(2 * live);
    if (v->tab.cap >= want) return ensure_lists(v, v->tab.cap);
    if (sync_all(v)) return 1;
    Table nt{};
    if (alloc_table(nt, want, v->stream)) return 1;
    bmask_t* nm1 = nullptr;
    MQR_CHECK_HIP(hipMalloc(&nm1, sizeof(bmask_t) * want));
    MQR_CHECK_HIP(hipMemsetAsync(nm1, 0, sizeof(bmask_t) * want, v->stream));
    if (v->tab.cap) {
        const int64_t blocks = (v->tab.cap + 255) / 256;
        hipLaunchKernelGGL(k_rehash, dim3((unsigned)blocks), dim3(256), 0, v->stream, v->tab, nt);
        MQR_CHECK_HIP(hipGetLastError());
        MQR_CHECK_HIP(hipStreamSynchronize(v->stream));
        free_table(v->tab);
    }
    if (v->mask1) MQR_CHECK_HIP(hipFree(v->mask1));
    v->tab = nt;
    v->mask1 = nm1;
    return ensure_lists(v, v->tab.cap);
}

int grow_pool(mqr_vbg* v, int64_t need) {
    if (need <= v->pool_cap) return 0;
    if (sync_all(v)) return 1;
    int64_t ncap = std::max<int64_t>(need, v->pool_cap + v->pool_cap / 2);
    float2* np = nullptr;
    uint64_t* nk = nullptr;
    MQR_CHECK_HIP(hipMalloc(&np, sizeof(float2) * ncap * v->R3));
    MQR_CHECK_HIP(hipMalloc(&nk, sizeof(uint64_t) * ncap));
    if (v->pool_cap) {  // buffers past the old capacity are not cleared (see mqr_vbg_reset)
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

static int ensure_fp(mqr_vbg* v, int n) {
    if (v->fp_cap >= n) return 0;
    if (sync_all(v)) return 1;
    const int cap = std::max(n, kMaxBatch);
    for (int p = 0; p < 2; ++p) {
        if (v->d_fp[p]) MQR_CHECK_HIP(hipFree(v->d_fp[p]));
        if (v->h_fp[p]) MQR_CHECK_HIP(hipHostFree(v->h_fp[p]));
        // FrameParams followed by the int64 depth-frame index array
        MQR_CHECK_HIP(hipMalloc(&v->d_fp[p], (sizeof(FrameParams) + sizeof(int64_t)) * cap));
        MQR_CHECK_HIP(hipHostMalloc(&v->h_fp[p], (sizeof(FrameParams) + sizeof(int64_t)) * cap, hipHostMallocDefault));
    }
    v->fp_cap = cap;
    return 0;
}

static int ensure_depth(mqr_vbg* v, int64_t floats) {
    if (v->depth_cap >= floats) return 0;
    if (sync_all(v)) return 1;
    for (int p = 0; p < 2; ++p) {
        if (v->d_depth[p]) MQR_CHECK_HIP(hipFree(v->d_depth[p]));
        MQR_CHECK_HIP(hipMalloc(&v->d_depth[p], sizeof(float) * floats));
    }
    v->depth_cap = floats;
    return 0;
}

// Whether one Markstein correction gives IEEE s / t for every s in [-t, t] (k_integrate_wt<.., 1>, lean_update_v<DIV1>):
// k_check_strunc over the ~1e9 floats of [+0, t] once per t per process (a few ms; the sequence is
// odd in s).  Cached; on any error the answer is false (two corrections stay).
static bool strunc_one_correction_ok(float t) {
    static std::mutex mu;
    static std::unordered_map<uint32_t, bool> cache;
    const uint32_t tb = __builtin_bit_cast(uint32_t, t);
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find(tb);
    if (it != cache.end()) return it->second;
    bool ok = false;
    uint32_t* d = nullptr;
    if (t > 0.0f && std::isfinite(t) && hipMalloc(&d, sizeof(uint32_t)) == hipSuccess) {
        hipStream_t s = nullptr;
        bool run = hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess &&
                   hipMemsetAsync(d, 0, sizeof(uint32_t), s) == hipSuccess;
        const uint64_t count = (uint64_t)tb + 1, chunk = 1ull << 28;
        for (uint64_t off = 0; run && off < count; off += chunk) {
            const uint64_t c = std::min<uint64_t>(chunk, count - off);
            hipLaunchKernelGGL(k_check_strunc, dim3((unsigned)((c + 255) / 256)), dim3(256), 0, s, t, (uint32_t)off, c, d);
            run = hipGetLastError() == hipSuccess;
        }
        uint32_t mism = 1;
        if (run && hipMemcpyAsync(&mism, d, sizeof(uint32_t), hipMemcpyDeviceToHost, s) == hipSuccess &&
            hipStreamSynchronize(s) == hipSuccess)
            ok = mism == 0;
        if (s) (void)hipStreamDestroy(s);
        (void)hipFree(d);
    }
    cache[tb] = ok;
    return ok;
}

#if MQR_AB
// The A/B library's integrate variants (launch_integrate's variant list; kernels in vbg_ab.hpp).  *fixup: the
// caller runs the exact fix-up launch behind the kernel (the kernels that hand blocks back).
static int launch_integrate_ab(mqr_vbg* v, int var, hipStream_t s, unsigned grid, unsigned lean_grid, int grouped,
                               const int32_t* list, const bmask_t* lmask, int* counters, const Table& t,
                               const float* depths, int64_t HW, int H, int W, const FrameParams* fp,
                               const int64_t* depth_frame, float depth_max, float sdf_trunc, int first_new,
                               int32_t* bad_out, bool* fixup, int nframes) {
    // k_integrate_lean_ab<16, 512, MAP, WPE, ILP, PAIR, DIV1, ZBLK, FIXIN>
    auto lean = [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3(lean_grid), dim3(512), 0, s, list, lmask, bad_out, counters, v->list_cap, t,
                           v->pool, v->voxel_size, depths, HW, H, W, fp, depth_frame, depth_max, sdf_trunc, first_new,
                           grouped);
    };
    auto win = [&](auto kern, unsigned nt) {
        hipLaunchKernelGGL(kern, dim3(grid), dim3(nt), 0, s, list, lmask, counters, v->list_cap, t, v->pool,
                           v->voxel_size, depths, HW, H, W, fp, depth_frame, depth_max, sdf_trunc, first_new);
    };
    auto wx = [&](auto kern) {  // k_integrate_wx: the window kernel's arguments plus the fix-up list
        hipLaunchKernelGGL(kern, dim3(grid), dim3(512), 0, s, list, lmask, bad_out, counters, v->list_cap, t, v->pool,
                           v->voxel_size, depths, HW, H, W, fp, depth_frame, depth_max, sdf_trunc, first_new);
    };
    *fixup = var <= 22;
    switch (var) {
        case 3: lean(k_integrate_lean_ab<16, 512>); break;  // plate map
        case 5:
            hipLaunchKernelGGL((k_integrate_lt<1>), dim3(grid), dim3(512), 0, s, list, lmask, bad_out, counters, v->list_cap, t, v->pool, v->voxel_size, depths, HW, H, W, fp, depth_frame,
                               depth_max, sdf_trunc, first_new);
            break;
        case 6: lean(k_integrate_lean_ab<16, 512, 1, 8, 1, 1>); break;  // paired gathers, 8 waves (spills)
        case 7: lean(k_integrate_lean_ab<16, 512, 1, 6, 1, 1>); break;  // paired gathers, 6 waves
        case 8: lean(k_integrate_lean_ab<16, 512, 1, 8, 2, 2>); break;  // VALU-lean projection / update
        case 9: lean(k_integrate_lean_ab<16, 512, 1, 8, 2, 3>); break;  // + zc checked per block
        case 10:                                                         // + one-correction s / trunc
            if (strunc_one_correction_ok(sdf_trunc)) lean(k_integrate_lean_ab<16, 512, 1, 8, 2, 3, 1>);
            else lean(k_integrate_lean_ab<16, 512, 1, 8, 2, 3>);
            break;
        case 11: lean(k_integrate_lean_ab<16, 512, 1, 5, 2, 4>); break;  // 16-byte windows, >= 5 waves
        case 12: lean(k_integrate_lean_ab<16, 512, 1, 4, 2, 4>); break;  // 16-byte windows, >= 4 waves
        case 13: lean(k_integrate_lean_ab<16, 512, 1, 6, 2, 5>); break;  // 8-byte windows, >= 6 waves
        case 14: lean(k_integrate_lean_ab<16, 512, 1, 5, 1, 4>); break;  // 16-byte windows, ILP 1
        case 15: lean(k_integrate_lean_ab<16, 512, 1, 7, 2, 5>); break;  // the round-3 default (fix-up launch)
        case 16: lean(k_integrate_lean_ab<16, 512, 1, 6, 2, 5, 0, true>); break;  // zc checked per block
        case 17:                                                                  // 16 + one-correction
            if (strunc_one_correction_ok(sdf_trunc)) lean(k_integrate_lean_ab<16, 512, 1, 6, 2, 5, 1, true>);
            else lean(k_integrate_lean_ab<16, 512, 1, 6, 2, 5, 0, true>);
            break;
        case 18: lean(k_integrate_lean_ab<16, 512, 1, 6, 4, 5>); break;  // 4 interleaved voxel chains
        case 19: lean(k_integrate_lean_ab<16, 512, 1, 6, 2, 6>); break;  // 16-byte windows in two halves
        case 20: lean(k_integrate_lean_ab<16, 512, 1, 7, 2, 7>); break;  // 8-byte windows in two halves
        case 21:                                                          // default + one-correction
            if (strunc_one_correction_ok(sdf_trunc)) lean(k_integrate_lean_ab<16, 512, 1, 6, 2, 5, 1>);
            else lean(k_integrate_lean_ab<16, 512, 1, 7, 2, 5>);
            break;
        case 22:  // 21 + zc checked per block, >= 5 waves
            if (strunc_one_correction_ok(sdf_trunc)) lean(k_integrate_lean_ab<16, 512, 1, 5, 2, 5, 1, true>);
            else lean(k_integrate_lean_ab<16, 512, 1, 7, 2, 5>);
            break;
        case 23: lean(k_integrate_lean_ab<16, 512, 1, 7, 2, 5, 0, false, true>); break;  // the round-4 default
        case 24: win(k_integrate_win_ab<512, 7, 0>, 512); break;    // plain frame loop
        case 25: win(k_integrate_win_ab<512, 6, 1>, 512); break;    // frames pipelined, >= 6 waves
        case 26: win(k_integrate_win_ab<1024, 8, 1>, 1024); break;  // 1024 threads, frames pipelined
        case 27: win(k_integrate_win_ab<1024, 8, 0>, 1024); break;  // 1024 threads, plain
        case 28: win(k_integrate_win_ab<512, 7, 1>, 512); break;    // frames pipelined, >= 7 waves
        case 29: win(k_integrate_win_ab<512, 7, 2>, 512); break;    // half-frame pipeline, >= 7 waves
        case 30: win(k_integrate_win_ab<1024, 8, 2>, 1024); break;  // half-frame pipeline, 1024 threads
        case 31: win(k_integrate_win_ab<512, 6, 2>, 512); break;    // half-frame pipeline, >= 6 waves
        case 32: win(k_integrate_win_ab<512, 7, 0, 1>, 512); break;  // timing diagnostics (wrong results)
        case 33: win(k_integrate_win_ab<512, 7, 0, 2>, 512); break;
        case 34: win(k_integrate_win_ab<512, 6, 2, 1>, 512); break;
        case 35: win(k_integrate_win_ab<512, 6, 2, 2>, 512); break;
        case 36: win(k_integrate_pk<7, 0>, 512); break;  // packed FP32
        case 37: win(k_integrate_pk<7, 2>, 512); break;
        case 38: win(k_integrate_pk<6, 2>, 512); break;
        case 39: win(k_integrate_pk<6, 0>, 512); break;
        // branch-free forms: 40 window offsets selected, 41 updates selected, 42 both, 43 both at >= 6 waves
        case 40: win(k_integrate_win_ab<512, 7, 0, 0, 1>, 512); break;
        case 41: win(k_integrate_win_ab<512, 7, 0, 0, 2>, 512); break;
        case 42: win(k_integrate_win_ab<512, 7, 0, 0, 3>, 512); break;
        case 43: win(k_integrate_win_ab<512, 6, 0, 0, 3>, 512); break;
        case 44: win(k_integrate_win_r4<7>, 512); break;  // the round-4 default's source
        case 45:    // lane-level tile proofs (k_tile_records + k_integrate_tp), >= 7 waves
        case 46:    // the same at >= 6 waves
        case 47:    // record loads of all 8 voxels first, >= 7 waves
        case 48:    // the same at >= 5 waves
        case 49:    // 45 branch-free: every lane issues the window read, decided lanes past the end
        case 50: {  // 47 branch-free
            // per device, grow-only (A/B library only): the batch's 8 x 4 tile records, 8 B each
            static void* rec_buf[64] = {};
            static size_t rec_cap[64] = {};
            const int TW = (W + 7) / 8, TH = (H + 3) / 4;
            const size_t need = sizeof(uint2) * (size_t)TW * TH * (size_t)std::max(nframes, 1);
            MQR_REQUIRE(v->device >= 0 && v->device < 64, "device index out of range");
            if (rec_cap[v->device] < need) {
                if (rec_buf[v->device]) MQR_CHECK_HIP(hipFree(rec_buf[v->device]));
                rec_buf[v->device] = nullptr;
                rec_cap[v->device] = 0;
                MQR_CHECK_HIP(hipMalloc(&rec_buf[v->device], need));
                rec_cap[v->device] = need;
            }
            uint2* recs = static_cast<uint2*>(rec_buf[v->device]);
            hipLaunchKernelGGL(k_tile_records, dim3((unsigned)((TW * TH + 7) / 8), (unsigned)nframes), dim3(256), 0, s,
                               depths, HW, H, W, depth_frame, depth_max, TW, TH, recs);
            auto tp = [&](auto kern) {
                hipLaunchKernelGGL(kern, dim3(grid), dim3(512), 0, s, list, lmask, counters, v->list_cap, t, v->pool,
                                   v->voxel_size, depths, HW, H, W, fp, depth_frame, depth_max, sdf_trunc, first_new,
                                   recs, TW, TH);
            };
            if (var == 45) tp(k_integrate_tp<7>);
            else if (var == 46) tp(k_integrate_tp<6>);
            else if (var == 47) tp(k_integrate_tp<7, 1>);
            else if (var == 48) tp(k_integrate_tp<5, 1>);
            else if (var == 49) tp(k_integrate_tp<7, 0, 1>);
            else tp(k_integrate_tp<7, 1, 1>);
            break;
        }
        // round 6: register-pressure forms of the default (k_integrate_wx<WPE, MODE>: MODE 1 halves, 2 fix-up launch)
        case 51: wx(k_integrate_wx<6, 0>); break;
        case 52: wx(k_integrate_wx<7, 1>); break;
        case 53: wx(k_integrate_wx<8, 1>); break;
        case 54: wx(k_integrate_wx<6, 1>); break;
        case 55: *fixup = true; wx(k_integrate_wx<7, 2>); break;
        case 56: *fixup = true; wx(k_integrate_wx<6, 2>); break;
        case 57: *fixup = true; wx(k_integrate_wx<8, 3>); break;
        case 58: *fixup = true; wx(k_integrate_wx<7, 3>); break;
        case 59: *fixup = true; wx(k_integrate_wx<8, 2>); break;
        case 60: wx(k_integrate_wx<7, 4>); break;  // the default + a workgroup barrier per frame
        case 61: wx(k_integrate_wx<6, 4>); break;
        case 62: *fixup = true; wx(k_integrate_wx<8, 6>); break;
        case 65: case 66: case 67: {  // the default's kernel with OPT 1 / 2 / 3 (k_integrate_wt<7, DIV1, OPT>)
            const int tcount = (int)v->launch_wbound;
            const bool one = v->div1 && strunc_one_correction_ok(sdf_trunc);
            auto kern = var == 65 ? (one ? k_integrate_wt<7, 1, 1> : k_integrate_wt<7, 0, 1>)
                      : var == 66 ? (one ? k_integrate_wt<7, 1, 2> : k_integrate_wt<7, 0, 2>)
                                  : (one ? k_integrate_wt<7, 1, 3> : k_integrate_wt<7, 0, 3>);
            hipLaunchKernelGGL(kern, dim3(grid), dim3(512), sizeof(float2) * (size_t)tcount, s, list, lmask, bad_out,
                               counters, v->list_cap, t, v->pool, v->voxel_size, depths, HW, H, W, fp, depth_frame,
                               depth_max, sdf_trunc, first_new, tcount);
            *fixup = true;
            break;
        }
        case 64: {  // the default's LDS-table kernel at >= 6 waves per SIMD (k_integrate_wt<6>)
            const int tcount = (int)v->launch_wbound;
            hipLaunchKernelGGL(k_integrate_wt<6>, dim3(grid), dim3(512), sizeof(float2) * (size_t)tcount, s, list, lmask,
                               bad_out, counters, v->list_cap, t, v->pool, v->voxel_size, depths, HW, H, W, fp,
                               depth_frame, depth_max, sdf_trunc, first_new, tcount);
            *fixup = true;
            break;
        }
        default: set_error("integrate variant " + std::to_string(var) + " unknown"); return 2;
    }
    return 0;
}
#endif

// Host twin of den_unsafe(): true unless 2^-60 <= |x| <= 2^60.
static bool div_unsafe_host(float x) {
    const float m = std::fabs(x);
    return !(m >= 0x1p-60f && m <= 0x1p60f);
}

static const int64_t* dframe_dev(const mqr_vbg* v, int p) {
    return reinterpret_cast<const int64_t*>(v->d_fp[p] + v->fp_cap);
}

// Stage B frames' parameters into parity p (on `stream`; the caller made sure batch p is free).
static int upload_frames(mqr_vbg* v, int p, const double* K, const double* T, const int* idx, int b,
                         const int64_t* dframe) {
    if (ensure_fp(v, b)) return 1;
    int64_t* h_dframe = reinterpret_cast<int64_t*>(v->h_fp[p] + v->fp_cap);
    for (int f = 0; f < b; ++f) {
        make_frame_params(K + 9 * idx[f], T + 16 * idx[f], &v->h_fp[p][f]);
        h_dframe[f] = dframe[f];
    }
    // one command when the two arrays are close (the parameters' unused tail travels along)
    if (v->fp_cap <= 2 * kMaxBatch) {
        MQR_CHECK_HIP(hipMemcpyAsync(v->d_fp[p], v->h_fp[p], sizeof(FrameParams) * v->fp_cap + sizeof(int64_t) * b,
                                     hipMemcpyHostToDevice, v->stream));
    } else {
        MQR_CHECK_HIP(hipMemcpyAsync(v->d_fp[p], v->h_fp[p], sizeof(FrameParams) * b, hipMemcpyHostToDevice, v->stream));
        MQR_CHECK_HIP(hipMemcpyAsync(v->d_fp[p] + v->fp_cap, h_dframe, sizeof(int64_t) * b, hipMemcpyHostToDevice,
                                     v->stream));
    }
    return 0;
}

// Counters of parity p: zero (pool counter untouched).
static int reset_batch_counters(mqr_vbg* v, int p) {
    v->lpt_ready[p] = false;
    if (!v->ctr_clean[p])  // (a volume reset already zeroed them: one queued command fewer at the step head)
        MQR_CHECK_HIP(hipMemsetAsync(v->ctr(p), 0, sizeof(int) * kCountersTotal, v->stream));
    v->ctr_clean[p] = false;
    return 0;
}

// Copy parity p's counters and the pool counter to the pinned mirror and wait (on `stream`).
static int read_counters(mqr_vbg* v, int p) {
    MQR_CHECK_HIP(hipMemcpyAsync(v->hctr(p), v->ctr(p), sizeof(int) * kCountersTotal, hipMemcpyDeviceToHost,
                                 v->stream));
    MQR_CHECK_HIP(hipMemcpyAsync(v->h_counters + 2 * kCountersTotal, v->pool_ctr(), sizeof(int),
                                 hipMemcpyDeviceToHost, v->stream));
    MQR_CHECK_HIP(hipEventRecord(v->ev_host[p], v->stream));
    MQR_CHECK_HIP(hipEventSynchronize(v->ev_host[p]));
    return 0;
}

// After a touch/activate of parity p: allocate pool buffers that did not fit, if any.
// table_full: when given, a full table is reported there (the caller undoes the touch and retries on
// a grown table) instead of as an error.
static int resolve_pool_overflow(mqr_vbg* v, int p, bool* table_full = nullptr) {
    if (read_counters(v, p)) return 1;
    int* c = v->hctr(p);
    if (c[kOverflow] & 2) {
        if (table_full) {
            *table_full = true;
            return 0;
        }
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
    int64_t pc = v->h_counters[2 * kCountersTotal];
    if (c[kOverflow] & 1) {
        const int64_t old_cap = v->pool_cap;
        if (grow_pool(v, std::max<int64_t>(pc, old_cap * 2))) return 1;  // waits for in-flight work
        // every allocation < old_cap succeeded; those >= old_cap are retried on the new pool
        hipLaunchKernelGGL(k_set_counter, dim3(1), dim3(1), 0, v->stream, v->pool_ctr(), (int)old_cap);
        MQR_CHECK_HIP(hipMemsetAsync(v->ctr(p) + kOverflow, 0, sizeof(int), v->stream));
        const int64_t blocks = (v->tab.cap + 255) / 256;
        hipLaunchKernelGGL(k_fixup_alloc, dim3((unsigned)blocks), dim3(256), 0, v->stream, v->tab, v->ctr(p),
                           v->pool_ctr(), v->pool_cap, v->bkeys);
        MQR_CHECK_HIP(hipGetLastError());
        if (read_counters(v, p)) return 1;
        if (c[kOverflow] & 1) {
            set_error("internal: pool growth failed");
            return 1;
        }
        pc = v->h_counters[2 * kCountersTotal];
    }
    v->pool_count = pc;
    return 0;
}

// Longest-first order of parity p's batch list (k_lpt_order reads the list length on the device, so
// the batch touch enqueues it before the host has read the counters).
// nframes: the batch's frame count -- the order kernel also fills the shadow counters a speculative
// integrate of the batch reads (k_gate's work; launch_integrate then launches no gate).
static int enqueue_lpt(mqr_vbg* v, int p, int nframes) {
    bmask_t* om = reinterpret_cast<bmask_t*>(v->lpt[p] + v->list_cap);
#if MQR_AB
    if (v->xcd_order)
        hipLaunchKernelGGL(k_xcd_order, dim3(1), dim3(1024), 0, v->stream, v->lists[p], v->ctr(p), v->list_cap,
                           v->table(p), v->lpt[p], om, reinterpret_cast<uint8_t*>(om + v->list_cap));
    else
#endif
        hipLaunchKernelGGL(k_lpt_order, dim3(1), dim3(1024), 0, v->stream, v->lists[p], v->ctr(p), v->list_cap,
                           v->table(p).mask, v->lpt[p], om, v->shadow(p), nframes);
    MQR_CHECK_HIP(hipGetLastError());
    v->lpt_ready[p] = true;
    return 0;
}

// Launch the integrate kernel for parity p on `stream2`, after touch(p) (event) completed.
// first_new: the pool size before this batch's allocations (its blocks start at (0, 0)).
// spec > 0: speculative launch (first batch of a call, counters not read yet): the kernels read the
// shadow counters k_gate fills, the grid is `spec` workgroups (they loop over the list), and the
// caller (mqr_integrate_frames) accounts the launch in the stats once the counters confirm it.
static int launch_integrate(mqr_vbg* v, int p, const float* depths, int64_t HW, int H, int W, int nframes,
                            float depth_scale, float depth_max, float sdf_trunc, int first_new, int64_t spec = 0) {
    const int64_t n = spec > 0 ? spec : std::min<int64_t>(v->hctr(p)[kListCount], v->list_cap);
    if (n == 0) return 0;
    hipStream_t s = v->pipelined ? v->stream2 : v->stream;
    const unsigned grid = (unsigned)std::min<int64_t>(n, 8192);
    const int64_t* depth_frame = dframe_dev(v, p);
    const Table t = v->table(p);
    int* counters = spec > 0 ? v->shadow(p) : v->ctr(p);
    const int32_t* list = v->lists[p];
    const bmask_t* lmask = nullptr;
    // The host has just read this batch's counters (resolve_pool_overflow waits for them), so the
    // touch -- and an order enqueued behind it -- completed: integrate needs no device-side wait on
    // the touch stream, only for an order enqueued here, after that read.
    bool touch_wait = v->touch_wait;
    bool gated_by_order = false;  // k_lpt_order filled the shadow counters (no k_gate launch)
    if (v->lpt_order && n > 1) {  // on the touch stream: overlaps the previous integrate
        if (!v->lpt_ready[p]) {
            if (enqueue_lpt(v, p, nframes)) return 1;
            touch_wait = true;
        }
        list = v->lpt[p];
        lmask = reinterpret_cast<bmask_t*>(v->lpt[p] + v->list_cap);
        gated_by_order = !v->xcd_order;
    }
    v->lpt_ready[p] = false;
    // the lean kernels run k_xcd_order's groups on the workgroups that share an XCD
    [[maybe_unused]] const int grouped = (v->xcd_order && lmask) ? 1 : 0;
    [[maybe_unused]] const unsigned lean_grid =
        grouped ? (unsigned)(kNumGroups * std::min<int64_t>((3 * n / 2 + kNumGroups - 1) / kNumGroups, 1024)) : grid;
    if (v->pipelined && (touch_wait || spec > 0)) {
        MQR_CHECK_HIP(hipEventRecord(v->touch_ev(p), v->stream));
        MQR_CHECK_HIP(hipStreamWaitEvent(s, v->touch_ev(p), 0));
    }
    if (spec > 0 && !gated_by_order) {
        hipLaunchKernelGGL(k_gate, dim3(1), dim3(64), 0, s, v->ctr(p), v->shadow(p), nframes);
        MQR_CHECK_HIP(hipGetLastError());
    }
    const FrameParams* fp = v->d_fp[p];
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (v->profile) {
        e0 = v->pooled_event();
        e1 = v->pooled_event();
        MQR_REQUIRE(e0 && e1, "profiling: event creation failed");
        MQR_CHECK_HIP(hipEventRecord(e0, s));
    }
    // The fast kernels (k_integrate_win, k_integrate_lean) evaluate s / sdf_trunc through the division
    // core (div_rn_core: exact while the denominator is in [2^-60, 2^60]), take depth in metres
    // (depth_scale 1: Open3D's d / 1 is d), and address the frame with 32-bit byte offsets that
    // must stay past 4HW for out-of-image voxels.  Otherwise the exact k_integrate_t runs alone.
    const bool lean_ok = !div_unsafe_host(sdf_trunc) && depth_scale == 1.0f && 4 * (HW + W) <= (int64_t{1} << 31);
    // Variants (mqr_vbg_set_variant, low byte; all bit-identical, tests/test_gpu_numerics.py):
    //   0 default -- R = 16: k_integrate_win (brick map, 8-byte window depth reads, >= 7 waves per SIMD,
    //     blocks outside the proven ranges redone in-kernel) when the frames allow the window reads (even
    //     H W, 8-byte aligned stack), else variant 4;  R = 8: k_integrate_lean, plate map, dword gathers;
    //   1 generic k_integrate (runtime R);  2 exact k_integrate_t;  4 k_integrate_lean with dword gathers
    //     at >= 8 waves per SIMD (the round-2 default) + the exact fix-up launch;
    //   A/B library only (MQR_AB, vbg_ab.hpp; DESIGN.md §4.1 has the measurements): 3 plate map;  5 packed
    //     LDS tiles (k_integrate_lt);  6 / 7 paired-lane gathers;  8 VALU-lean projection / update, 9 + zc
    //     checked per block, 10 + one-correction s / trunc;  11 / 12 / 14 / 19 16-byte windows;  13 / 16 /
    //     17 / 18 / 20 / 21 / 22 8-byte windows at 6 waves / SIMD, with the block zc check, one-correction
    //     division, ILP 4, in two halves;  15 = the round-3 default (the exact path in a fix-up launch);
    //     23 = the round-4 default (k_integrate_lean_ab with the same arithmetic as 0);  24-31 the frame
    //     loop software-pipelined / 1024-thread workgroups (k_integrate_win_ab);  32-35 timing diagnostics
    //     (wrong results);  36-39 packed FP32 (k_integrate_pk);  40-43 branch-free window offsets / updates;  44 the
    //     round-4 source;  45 / 46 lane-level tile proofs (k_tile_records + k_integrate_tp, >= 7 / 6 waves), 47 / 48 with
    //     the eight record loads issued first (>= 7 / 5 waves), 49 / 50 = 45 / 47 branch-free.  (24 of round 4, a ballot skip of
    //     out-of-image wave slots, ran 0.70 vs 0.48 ms per launch: removed.)
    int var = v->kernel_variant;
    if (var < 0 || var > 67 || var == 63) var = 0;
    // the LDS-table kernels (default, 64) need a known weight bound whose table fits a workgroup's LDS share
    const bool rtab_ok = v->rtab && v->launch_wbound >= 1 && v->launch_wbound <= kRtabMax;
    if (var >= 64 && !rtab_ok) var = 0;
    if (!MQR_AB && var != 1 && var != 2 && var != 4) var = 0;
    if (var != 1 && var != 2 && !lean_ok) var = 2;
    if (var == 5 && (v->R != 16 || W % 4 != 0 || W < 4 || (reinterpret_cast<uintptr_t>(depths) & 15))) var = 0;
    if (var >= 5 && v->R != 16) var = 0;
    // window reads: 4HW a multiple of the window and a frame base aligned to it, so an in-image
    // window never crosses the end of a frame and an out-of-image one (at 4HW) lies wholly past it
    const bool win8_ok = (HW % 2) == 0 && (reinterpret_cast<uintptr_t>(depths) & 7) == 0;
    const bool win16_ok = (HW % 4) == 0 && (reinterpret_cast<uintptr_t>(depths) & 15) == 0;
    if ((var == 11 || var == 12 || var == 14 || var == 19) && !win16_ok) var = 0;
    if (var == 0 && !(v->R == 16 && win8_ok)) var = 4;
    if (var >= 13 && !win8_ok) var = 4;
    if (v->R != 16 && v->R != 8) var = 1;
    v->last_var = var;
    v->last_kname = var == 1 ? "k_integrate" : var == 2 ? "k_integrate_t" : var == 4 || v->R == 8 ? "k_integrate_lean"
                                                                                                   : "k_integrate_ab";
    const int32_t* bad_list = v->bad[p];
    const bmask_t* bad_mask = reinterpret_cast<const bmask_t*>(v->bad[p] + v->list_cap);
    int* bad_count = counters + kBadCount;
    bool fixup = false;  // the exact fix-up launch over the blocks a fast kernel handed back
    if (var == 1) {
        hipLaunchKernelGGL(k_integrate, dim3(grid), dim3(256), 0, s, list, counters, v->list_cap, t, v->pool, v->R,
                           v->voxel_size, depths, HW, H, W, fp, depth_frame, depth_scale, depth_max, sdf_trunc, first_new);
    } else if (v->R == 16) {
        if (var == 2) {
            hipLaunchKernelGGL((k_integrate_t<16, 4, 512>), dim3(grid), dim3(512), 0, s, list, lmask,
                               counters + kListCount, v->list_cap, t, v->pool, v->voxel_size, depths, HW, H, W, fp,
                               depth_frame, depth_scale, depth_max, sdf_trunc, first_new);
        } else if (var == 4) {  // dword gathers (frames the window reads cannot take)
            hipLaunchKernelGGL((k_integrate_lean<16, 512, 1, 8, 2>), dim3(grid), dim3(512), 0, s, list, lmask,
                               v->bad[p], counters, v->list_cap, t, v->pool, v->voxel_size, depths, HW, H, W, fp,
                               depth_frame, depth_max, sdf_trunc, first_new);
            fixup = true;
        } else if (var == 0 && rtab_ok) {  // the update through the (w, 1 / (w + 1)) table
            const int tcount = (int)v->launch_wbound;
            // s / sdf_trunc with one correction where that is verified exact for this sdf_trunc (bit 27: never)
            const bool one = v->div1 && strunc_one_correction_ok(sdf_trunc);
            auto kern = one ? k_integrate_wt<7, 1> : k_integrate_wt<7, 0>;
            v->last_kname = one ? "k_integrate_wt<7, 1>" : "k_integrate_wt<7, 0>";
            hipLaunchKernelGGL(kern, dim3(grid), dim3(512), sizeof(float2) * (size_t)tcount, s, list, lmask, v->bad[p],
                               counters, v->list_cap, t, v->pool, v->voxel_size, depths, HW, H, W, fp, depth_frame,
                               depth_max, sdf_trunc, first_new, tcount);
            fixup = true;
        } else if (var == 0) {
            v->last_kname = "k_integrate_win<7>";
            hipLaunchKernelGGL(k_integrate_win<7>, dim3(grid), dim3(512), 0, s, list, lmask, counters, v->list_cap, t,
                               v->pool, v->voxel_size, depths, HW, H, W, fp, depth_frame, depth_max, sdf_trunc,
                               first_new);
        } else {
#if MQR_AB
            if (launch_integrate_ab(v, var, s, grid, lean_grid, grouped, list, lmask, counters, t, depths, HW, H, W, fp,
                                    depth_frame, depth_max, sdf_trunc, first_new, v->bad[p], &fixup, nframes))
                return 1;
#endif
        }
    } else {  // R == 8
        if (var == 2) {
            hipLaunchKernelGGL((k_integrate_t<8, 2, 256>), dim3(grid), dim3(256), 0, s, list, lmask,
                               counters + kListCount, v->list_cap, t, v->pool, v->voxel_size, depths, HW, H, W, fp,
                               depth_frame, depth_scale, depth_max, sdf_trunc, first_new);
        } else {
            hipLaunchKernelGGL((k_integrate_lean<8, 256>), dim3(grid), dim3(256), 0, s, list, lmask, v->bad[p],
                               counters, v->list_cap, t, v->pool, v->voxel_size, depths, HW, H, W, fp, depth_frame,
                               depth_max, sdf_trunc, first_new);
            hipLaunchKernelGGL((k_integrate_t<8, 2, 256>), dim3(8), dim3(256), 0, s, bad_list, bad_mask, bad_count,
                               v->list_cap, t, v->pool, v->voxel_size, depths, HW, H, W, fp, depth_frame, depth_scale,
                               depth_max, sdf_trunc, first_new);
        }
    }
    if (fixup)  // (usually no block: reads a zero count)
        hipLaunchKernelGGL((k_integrate_t<16, 4, 512>), dim3(8), dim3(512), 0, s, bad_list, bad_mask, bad_count,
                           v->list_cap, t, v->pool, v->voxel_size, depths, HW, H, W, fp, depth_frame, depth_scale,
                           depth_max, sdf_trunc, first_new);
    MQR_CHECK_HIP(hipGetLastError());
    if (v->profile) {
        MQR_CHECK_HIP(hipEventRecord(e1, s));
        v->int_done[p] = e1;
        v->int_events.emplace_back(e0, e1);
        if (spec == 0) {
            v->stats.integrate_launches += 1;
            v->stats.union_blocks += n;
            for (int f = 0; f < kMaxBatch; ++f) v->stats.frame_blocks += v->hctr(p)[kFreshBase + f];
            v->stats.frames += nframes;
        }
    }
    if (!v->profile) {
        MQR_CHECK_HIP(hipEventRecord(v->int_ev(p), s));
        v->int_done[p] = v->int_ev(p);
    }
    v->int_pending[p] = true;
    return 0;
}

// Before reusing parity p's batch state on `stream`: the integrate that last used it must be done.
static int wait_parity_free(mqr_vbg* v, int p) {
    if (v->int_pending[p]) {
        MQR_CHECK_HIP(hipStreamWaitEvent(v->stream, v->int_done[p], 0));
        v->int_pending[p] = false;  // ordered behind it on `stream` from here on
    }
    return 0;
}

static void drain_events(mqr_vbg* v) {
    for (auto& e : v->int_events) {
        float ms = 0.f;
        if (hipEventSynchronize(e.second) == hipSuccess && hipEventElapsedTime(&ms, e.first, e.second) == hipSuccess)
            v->stats.integrate_ms += ms;
    }
    v->int_events.clear();
    for (auto& e : v->touch_events) {
        float ms = 0.f;
        if (hipEventSynchronize(e.second) == hipSuccess && hipEventElapsedTime(&ms, e.first, e.second) == hipSuccess)
            v->stats.touch_ms += ms;
    }
    v->touch_events.clear();
    v->ev_used = 0;
}

// Fill an EMPTY volume with `n` distinct packed keys (device), buffer i = keys[i], pool counter n.
// merge_writes_all: the caller's merge writes every voxel of the n buffers (k_merge_fused) -- the pool is
// not zeroed first, and the table-full check is deferred: the counters are copied to the host behind the
// activation and activate_ordered_check reads them after the caller's final synchronize, so the host
// does not wait here.  Otherwise the buffers start at (0, 0) (k_merge_blocks accumulates into them) and
// the check is made before returning.
int activate_ordered(mqr_vbg* v, const uint64_t* dkeys, int64_t n, bool merge_writes_all) {
    if (v->pool_count != 0) {
        set_error("internal: ordered activation needs an empty volume");
        return 1;
    }
    v->act_check = false;
    if (n == 0) return 0;
    // (ensure_table / grow_pool drain the volume's streams before they reallocate; everything else is
    // ordered on `stream` behind the reset)
    if (ensure_table(v, n) || grow_pool(v, n) || reset_batch_counters(v, 0)) return 1;
    if (!merge_writes_all) MQR_CHECK_HIP(hipMemsetAsync(v->pool, 0, sizeof(float2) * n * v->R3, v->stream));
    hipLaunchKernelGGL(k_activate_ordered, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, v->stream, dkeys, n,
                       v->tab, v->bkeys, v->ctr(0));
    hipLaunchKernelGGL(k_set_counter, dim3(1), dim3(1), 0, v->stream, v->pool_ctr(), (int)n);
    MQR_CHECK_HIP(hipGetLastError());
    v->pool_count = n;
    if (merge_writes_all) {
        MQR_CHECK_HIP(hipMemcpyAsync(v->hctr(0), v->ctr(0), sizeof(int) * kCountersTotal, hipMemcpyDeviceToHost,
                                     v->stream));
        MQR_CHECK_HIP(hipEventRecord(v->ev_host[0], v->stream));
        v->act_check = true;
        return 0;
    }
    if (read_counters(v, 0)) return 1;
    if (v->hctr(0)[kOverflow] & 2) {
        set_error("internal: block table full");
        return 1;
    }
    return 0;
}

int activate_ordered_check(mqr_vbg* v) {
    if (!v->act_check) return 0;  // checked by activate_ordered itself, or nothing activated
    v->act_check = false;
    MQR_CHECK_HIP(hipEventSynchronize(v->ev_host[0]));
    if (v->hctr(0)[kOverflow] & 2) {
        set_error("internal: block table full");
        return 1;
    }
    return 0;
}

// max_probe: slots a new key may probe before the touch reports a full table (Table.cap = no limit).
static int touch_launch(mqr_vbg* v, int p, const float* dbase, int64_t HW, int H, int W, int b, float depth_scale,
                        float depth_max, float sdf_trunc, float block_size, const Table& t, int alloc,
                        int64_t max_probe) {
    const int n = (H / 4) * (W / 4);
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (v->profile_touch) {
        e0 = v->pooled_event();
        e1 = v->pooled_event();
        MQR_REQUIRE(e0 && e1, "profiling: event creation failed");
        MQR_CHECK_HIP(hipEventRecord(e0, v->stream));
    }
    // (measured and removed, profiles/r04_ab_integrate.json and DESIGN.md §4.1: a frame per workgroup
    // (k_touch_frame), a two-phase collect / claim touch, 8 frames per strip workgroup with one claim per
    // (block, frame group))
    hipStream_t ts = v->stream;
    if (n > 0) {
        if (v->touch_ppt == 1)
            hipLaunchKernelGGL(k_touch<1>, dim3((n + 255) / 256, b), dim3(256), 0, ts, dbase, HW, H, W,
                               v->d_fp[p], dframe_dev(v, p), depth_scale, depth_max, sdf_trunc, block_size, t, max_probe,
                               alloc, v->ctr(p), v->pool_ctr(), v->pool_cap, v->bkeys, v->lists[p], v->list_cap);
        else
            hipLaunchKernelGGL(k_touch<2>, dim3((n + 511) / 512, b), dim3(256), 0, ts, dbase, HW, H, W,
                               v->d_fp[p], dframe_dev(v, p), depth_scale, depth_max, sdf_trunc, block_size, t, max_probe,
                               alloc, v->ctr(p), v->pool_ctr(), v->pool_cap, v->bkeys, v->lists[p], v->list_cap);
    }
    MQR_CHECK_HIP(hipGetLastError());
    if (v->profile_touch) {
        MQR_CHECK_HIP(hipEventRecord(e1, v->stream));
        v->touch_events.emplace_back(e0, e1);
        v->stats.touch_launches += 1;
        v->stats.pixels += (int64_t)b * HW;
    }
    return 0;
}

// Undo the touch of parity p: clear its slot marks, remove the keys it inserted (buffer index >=
// pool_before, or -2 when the pool overflowed) and give their pool buffers back.
static int undo_touch(mqr_vbg* v, int p, int64_t pool_before) {
    const int64_t n = std::min<int64_t>(v->hctr(p)[kListCount], v->list_cap);
    if (n > 0)
        hipLaunchKernelGGL(k_clear_slots, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, v->stream, v->lists[p], n,
                           v->table(p), 0);
    hipLaunchKernelGGL(k_rollback, dim3((unsigned)((v->tab.cap + 255) / 256)), dim3(256), 0, v->stream, v->table(p),
                       (int)pool_before);
    hipLaunchKernelGGL(k_set_counter, dim3(1), dim3(1), 0, v->stream, v->pool_ctr(), (int)pool_before);
    MQR_CHECK_HIP(hipGetLastError());
    v->pool_count = pool_before;
    v->lpt_ready[p] = false;
    return 0;
}

// Table keys the touch of a batch may need room for.  The worst case (every sample of every frame a
// new block: 4 * (H/4) * (W/4) keys per frame) would size the table at ~2^24 slots for 64 VGA frames
// -- 470 MB that every reset clears and that the touch probes far outside the L2s -- while a batch of
// the C2 sequence allocates ~3 000 blocks.  The table is sized for the live blocks plus a headroom of
// 4x the largest batch seen (at least 32768), the touch probes at most kProbeLimit slots per key, and
// a batch that overflows that is undone and touched again on a table grown to the worst case.
// The table keeps >= 2^20 slots: the touch's mask atomics serialise per cache line, and a table of
// 2^17 slots (16 masks per 128-byte line, ~3 of them active in a batch) made the touch 10 % and the
// overlapped integrate 4 % slower than sparse lines did (profiles/r02_table_sizing.json).
constexpr int64_t kMinHeadroom = 1 << 15;
constexpr int64_t kMinTableLive = 1 << 19;  // ensure_table sizes for 2x live keys: 2^20 slots
constexpr int64_t kProbeLimit = 128;

// Touch (and allocate) frames [0, b) of the staged parity-p batch, in two phases: the launch (table
// sized, touch and longest-first order enqueued) and the resolution (counters read, pool overflow
// resolved, a probe-limited table that filled up undone, grown and touched again).
struct TouchState {
    int64_t pool_before = 0, worst = 0;
    bool limited = false;
};
static int touch_batch_launch(mqr_vbg* v, int p, const float* dbase, int64_t HW, int H, int W, int b,
                              float depth_scale, float depth_max, float sdf_trunc, float block_size, int64_t max_touch,
                              TouchState& ts) {
    ts.worst = v->pool_count + b * max_touch;
    const int64_t headroom = v->table_worst ? b * max_touch
                                            : std::min<int64_t>(b * max_touch,
                                                                std::max<int64_t>(kMinHeadroom, 4 * v->batch_new_max));
    if (ensure_table(v, std::max(kMinTableLive, v->pool_count + headroom))) return 1;
    ts.limited = v->probe_one || v->tab.cap < next_pow2(2 * ts.worst);
    ts.pool_before = v->pool_count;
    if (touch_launch(v, p, dbase, HW, H, W, b, depth_scale, depth_max, sdf_trunc, block_size, v->table(p), 1,
                     ts.limited ? (v->probe_one ? 1 : std::min(kProbeLimit, v->tab.cap)) : v->tab.cap))
        return 1;
    // the batch order is computed while the host waits for the counters (pool growth below only
    // rewrites buffer indices, which the order does not read)
    if (v->lpt_order && enqueue_lpt(v, p, b)) return 1;
    return 0;
}

static int touch_batch_resolve(mqr_vbg* v, int p, const float* dbase, int64_t HW, int H, int W, int b,
                               float depth_scale, float depth_max, float sdf_trunc, float block_size,
                               const TouchState& ts) {
    bool full = false;
    if (resolve_pool_overflow(v, p, ts.limited ? &full : nullptr)) return 1;
    if (full) {
        if (undo_touch(v, p, ts.pool_before) || ensure_table(v, ts.worst) || reset_batch_counters(v, p)) return 1;
        if (touch_launch(v, p, dbase, HW, H, W, b, depth_scale, depth_max, sdf_trunc, block_size, v->table(p), 1,
                         v->tab.cap))
            return 1;
        if (v->lpt_order && enqueue_lpt(v, p, b)) return 1;
        if (resolve_pool_overflow(v, p)) return 1;
        v->stats.table_retries += 1;
    }
    v->batch_new_max = std::max(v->batch_new_max, v->pool_count - ts.pool_before);
    return 0;
}

static int touch_batch(mqr_vbg* v, int p, const float* dbase, int64_t HW, int H, int W, int b, float depth_scale,
                       float depth_max, float sdf_trunc, float block_size, int64_t max_touch) {
    TouchState ts;
    return touch_batch_launch(v, p, dbase, HW, H, W, b, depth_scale, depth_max, sdf_trunc, block_size, max_touch, ts) ||
           touch_batch_resolve(v, p, dbase, HW, H, W, b, depth_scale, depth_max, sdf_trunc, block_size, ts);
}

const char* confidence_src_tag();  // confidence.hip

static const char* kNoBlock =
    "No block is touched in TSDF volume, abort integration. Please check specified parameters, especially "
    "depth_scale and voxel_size";

}  // namespace mqr

using namespace mqr;

// ====================================================================== C ABI
extern "C" {

int mqr_version(void) { return 100; }

#ifndef MQR_SRC_TAG
#define MQR_SRC_TAG "untagged"
#endif
int mqr_build_tag(int which, char* buf, int cap) {
    MQR_REQUIRE(buf && cap > 0, "null argument");
    MQR_REQUIRE(which == 0 || which == 1, "which: 0 = integrate sources, 1 = confidence sources");
    const std::string t = which == 0 ? std::string(MQR_AB ? "ab-" : "") + MQR_SRC_TAG : std::string(confidence_src_tag());
    std::snprintf(buf, (size_t)cap, "%s", t.c_str());
    return 0;
}

int mqr_vbg_last_kernel(mqr_vbg* v, int* variant) {
    MQR_REQUIRE(v && variant, "null argument");
    *variant = v->last_var;
    return 0;
}

int mqr_vbg_last_kernel_name(mqr_vbg* v, char* buf, int cap) {
    MQR_REQUIRE(v && buf && cap > 0, "null argument");
    std::snprintf(buf, (size_t)cap, "%s", v->last_kname);
    return 0;
}
const char* mqr_last_error(void) { return get_error(); }

int mqr_set_stream(void* stream) {
    t_caller_stream = static_cast<hipStream_t>(stream);
    return 0;
}

int mqr_get_stream(void** stream) {
    MQR_REQUIRE(stream, "null argument");
    *stream = t_caller_stream;
    return 0;
}

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
    // the buffer may still be read by work in flight on the library's streams (an integrate_frames on
    // device frames returns before its last integrate ends): the whole device first
    MQR_CHECK_HIP(hipDeviceSynchronize());
    MQR_CHECK_HIP(hipFree(ptr));
    return 0;
}

int mqr_memcpy(void* dst, int dst_loc, const void* src, int src_loc, int64_t bytes, int device) {
    MQR_CHECK_HIP(hipSetDevice(device));
    // hipMemcpy orders after the null stream only: wait for the caller stream's work on the buffers
    if ((dst_loc == MQR_DEVICE || src_loc == MQR_DEVICE) && t_caller_stream)
        MQR_CHECK_HIP(hipStreamSynchronize(t_caller_stream));
    hipMemcpyKind kind = dst_loc == MQR_DEVICE ? (src_loc == MQR_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice)
                                               : (src_loc == MQR_DEVICE ? hipMemcpyDeviceToHost : hipMemcpyHostToHost);
    if (kind == hipMemcpyDeviceToHost && bytes >= (int64_t)kD2HParallelMin) return d2h_parallel(device, dst, src, (size_t)bytes);
    MQR_CHECK_HIP(hipMemcpy(dst, src, (size_t)bytes, kind));
    return 0;
}

int mqr_device_mem_info(int device, int64_t* free_bytes, int64_t* total_bytes) {
    MQR_REQUIRE(free_bytes && total_bytes, "null argument");
    MQR_CHECK_HIP(hipSetDevice(device));
    size_t f = 0, t = 0;
    MQR_CHECK_HIP(hipMemGetInfo(&f, &t));
    *free_bytes = (int64_t)f;
    *total_bytes = (int64_t)t;
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
    const size_t nctr = kCounterInts;
    // The touch stream gets the device's highest priority: touch(b+1) shares the CUs with
    // integrate(b), and integrate(b+1) cannot be enqueued before the host has read touch(b+1)'s
    // counters -- a touch starved by integrate waves would leave the device idle at every batch.
    int prio_least = 0, prio_greatest = 0;
    (void)hipDeviceGetStreamPriorityRange(&prio_least, &prio_greatest);
    bool ok = hipStreamCreateWithPriority(&v->stream, hipStreamNonBlocking, prio_greatest) == hipSuccess &&
              hipStreamCreateWithFlags(&v->stream2, hipStreamNonBlocking) == hipSuccess &&
              hipMalloc(&v->counters, sizeof(int) * nctr) == hipSuccess &&
              hipHostMalloc(&v->h_counters, sizeof(int) * nctr, hipHostMallocDefault) == hipSuccess &&
              hipMemsetAsync(v->counters, 0, sizeof(int) * nctr, v->stream) == hipSuccess;
    for (int p = 0; p < 2 && ok; ++p)
        ok = hipEventCreateWithFlags(&v->ev_touch[p], hipEventDisableTiming | hipEventDisableSystemFence) ==
                 hipSuccess &&
             hipEventCreateWithFlags(&v->ev_int[p], hipEventDisableTiming | hipEventDisableSystemFence) ==
                 hipSuccess &&
             hipEventCreateWithFlags(&v->ev_touch_sys[p], hipEventDisableTiming) == hipSuccess &&
             hipEventCreateWithFlags(&v->ev_int_sys[p], hipEventDisableTiming) == hipSuccess &&
             hipEventCreateWithFlags(&v->ev_host[p], hipEventDisableTiming) == hipSuccess;
    if (!ok) {
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

static void free_alt(mqr_vbg* v);  // (the second table / pool set, below mqr_vbg_reset's helpers)

int mqr_vbg_destroy(mqr_vbg* v) {
    if (!v) return 0;
    (void)hipSetDevice(v->device);
    if (v->stream) (void)hipStreamSynchronize(v->stream);
    if (v->stream2) (void)hipStreamSynchronize(v->stream2);
    drain_events(v);
    free_table(v->tab);
    free_table(v->ftab);
    free_alt(v);
    for (hipEvent_t e : {v->set_ev, v->alt.ev})
        if (e) (void)hipEventDestroy(e);
    if (v->mask1) (void)hipFree(v->mask1);
    if (v->pool) (void)hipFree(v->pool);
    if (v->bkeys) (void)hipFree(v->bkeys);
    for (int p = 0; p < 2; ++p) {
        if (v->lists[p]) (void)hipFree(v->lists[p]);
        if (v->lpt[p]) (void)hipFree(v->lpt[p]);
        if (v->bad[p]) (void)hipFree(v->bad[p]);
        if (v->d_fp[p]) (void)hipFree(v->d_fp[p]);
        if (v->h_fp[p]) (void)hipHostFree(v->h_fp[p]);
        if (v->d_depth[p]) (void)hipFree(v->d_depth[p]);
        for (hipEvent_t e : {v->ev_touch[p], v->ev_int[p], v->ev_touch_sys[p], v->ev_int_sys[p], v->ev_host[p]})
            if (e) (void)hipEventDestroy(e);
    }
    for (hipEvent_t e : v->ev_pool) (void)hipEventDestroy(e);
    if (v->counters) (void)hipFree(v->counters);
    if (v->h_counters) (void)hipHostFree(v->h_counters);
    if (v->ex_scratch) (void)hipFree(v->ex_scratch);
    if (v->h_ex) (void)hipHostFree(v->h_ex);
    if (v->stream) (void)hipStreamDestroy(v->stream);
    if (v->stream2) (void)hipStreamDestroy(v->stream2);
    delete v;
    return 0;
}

// ---- the second table / pool set (mqr_vbg_reset behind an unfinished integrate) ----
constexpr int64_t kAltMaxBytes = int64_t{2} << 30;  // volumes whose pool is larger wait instead

static void swap_sets(mqr_vbg* v) {
    std::swap(v->tab, v->alt.tab);
    std::swap(v->mask1, v->alt.mask1);
    std::swap(v->pool, v->alt.pool);
    std::swap(v->bkeys, v->alt.bkeys);
    std::swap(v->pool_cap, v->alt.pool_cap);
    std::swap(v->set_ev, v->alt.ev);
    std::swap(v->set_ev_live, v->alt.ev_live);
}

static void free_alt(mqr_vbg* v) {
    free_table(v->alt.tab);
    if (v->alt.mask1) (void)hipFree(v->alt.mask1);
    if (v->alt.pool) (void)hipFree(v->alt.pool);
    if (v->alt.bkeys) (void)hipFree(v->alt.bkeys);
    v->alt.mask1 = nullptr;
    v->alt.pool = nullptr;
    v->alt.bkeys = nullptr;
    v->alt.pool_cap = 0;
}

// The second set at the current set's capacities (fresh allocations: a reset discards contents).  *ok is
// false when the budget does not allow it -- the reset then waits as before.
static int ensure_alt(mqr_vbg* v, bool* ok) {
    *ok = false;
    const bool pool_fits = v->alt.pool && v->alt.pool_cap >= v->pool_cap;
    const bool tab_fits = v->alt.tab.keys && v->alt.tab.cap >= v->tab.cap;
    if (pool_fits && tab_fits) {
        *ok = true;
        return 0;
    }
    const int64_t pool_bytes = (int64_t)sizeof(float2) * v->pool_cap * v->R3 + (int64_t)sizeof(uint64_t) * v->pool_cap;
    const int64_t tab_bytes = (int64_t)(sizeof(uint64_t) + sizeof(int32_t) + 2 * sizeof(bmask_t)) * v->tab.cap;
    if (pool_bytes > kAltMaxBytes) return 0;
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    const int64_t need = (pool_fits ? 0 : pool_bytes) + (tab_fits ? 0 : tab_bytes);
    if ((int64_t)free_b - need < (int64_t)(total_b / 4)) return 0;
    // the set's last readers (an integrate before its event) are done before its memory is replaced
    if (v->alt.ev_live) MQR_CHECK_HIP(hipEventSynchronize(v->alt.ev));
    if (!v->alt.ev) MQR_CHECK_HIP(hipEventCreateWithFlags(&v->alt.ev, hipEventDisableTiming | hipEventDisableSystemFence));
    if (!v->set_ev) MQR_CHECK_HIP(hipEventCreateWithFlags(&v->set_ev, hipEventDisableTiming | hipEventDisableSystemFence));
    v->alt.ev_live = false;
    bool fail = false;
    if (!pool_fits) {
        if (v->alt.pool) (void)hipFree(v->alt.pool);
        if (v->alt.bkeys) (void)hipFree(v->alt.bkeys);
        v->alt.pool = nullptr;
        v->alt.bkeys = nullptr;
        v->alt.pool_cap = 0;
        fail = hipMalloc(&v->alt.pool, sizeof(float2) * v->pool_cap * v->R3) != hipSuccess ||
               hipMalloc(&v->alt.bkeys, sizeof(uint64_t) * v->pool_cap) != hipSuccess;
        if (!fail) v->alt.pool_cap = v->pool_cap;
    }
    if (!fail && !tab_fits) {
        free_table(v->alt.tab);
        if (v->alt.mask1) (void)hipFree(v->alt.mask1);
        v->alt.mask1 = nullptr;
        Table nt{};
        fail = hipMalloc(&nt.keys, sizeof(uint64_t) * v->tab.cap) != hipSuccess ||
               hipMalloc(&nt.vals, sizeof(int32_t) * v->tab.cap) != hipSuccess ||
               hipMalloc(&nt.mask, sizeof(bmask_t) * v->tab.cap) != hipSuccess ||
               hipMalloc(&v->alt.mask1, sizeof(bmask_t) * v->tab.cap) != hipSuccess;
        nt.cap = v->tab.cap;
        v->alt.tab = nt;  // (freed by free_alt on failure; k_reset_table clears it when swapped in)
    }
    if (fail) {
        (void)hipGetLastError();
        free_alt(v);
        return 0;
    }
    *ok = true;
    return 0;
}

int mqr_vbg_reset(mqr_vbg* v) {
    MQR_REQUIRE(v, "null volume");
    MQR_CHECK_HIP(hipSetDevice(v->device));
    uint32_t segs = 0x1f;  // every counter segment (k_reset_table)
    const bool inflight = v->pipelined && (v->int_pending[0] || v->int_pending[1]);
    bool flip = false;
    if (inflight && v->flip_reset && ensure_alt(v, &flip)) return 1;
    if (flip) {
        // an integrate of the current set is still in flight (mqr_integrate_frames on device frames returns
        // before it ends): mark the set's last reader on the integrate stream and swap in the other set,
        // cleared behind the integrate that last read it -- the next touch need not wait for this one
        MQR_CHECK_HIP(hipEventRecord(v->set_ev, v->stream2));
        v->set_ev_live = true;
        swap_sets(v);
        if (v->set_ev_live) MQR_CHECK_HIP(hipStreamWaitEvent(v->stream, v->set_ev, 0));
        // the in-flight parity's counters (and shadows) are still read: cleared by reset_batch_counters,
        // after wait_parity_free, when that parity is next used
        for (int p = 0; p < 2; ++p)
            if (v->int_pending[p]) segs &= ~((1u << p) | (1u << (3 + p)));
        ++v->flips;
    } else {
        // behind an integrate still in flight: a device-side wait on `stream`, no host wait
        if (order_after_integrate(v)) return 1;
    }
    // one launch, ordered on `stream` before anything that uses the volume next; the pool is not
    // cleared: a block starts at (0, 0) in the batch that allocates it (launch_integrate first_new)
    const int64_t cells = std::max<int64_t>(v->tab.cap, kCounterInts);
    hipLaunchKernelGGL(k_reset_table, dim3((unsigned)((cells + 255) / 256)), dim3(256), 0, v->stream, v->tab, v->mask1,
                       v->counters, segs);
    MQR_CHECK_HIP(hipGetLastError());
    v->pool_count = 0;
    v->wbound = 0;
    v->ctr_clean[0] = (segs & 1u) != 0;
    v->ctr_clean[1] = (segs & 2u) != 0;
    return 0;
}

int mqr_vbg_flips(mqr_vbg* v, int64_t* n) {
    MQR_REQUIRE(v && n, "null argument");
    *n = v->flips;
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

int mqr_integrate_frames(mqr_vbg* v, const float* depths, int depth_loc, int B, int H, int W, const double* K,
                         const double* T_wc, const uint8_t* frame_ok, float depth_scale, float depth_max,
                         float trunc_mult) {
    MQR_REQUIRE(v && depths && K && T_wc, "null argument");
    MQR_REQUIRE(B >= 0 && H > 0 && W > 0, "bad frame shape");
    MQR_REQUIRE(depth_loc == MQR_HOST || depth_loc == MQR_DEVICE || depth_loc == MQR_DEVICE_RESIDENT,
                "depth_loc must be MQR_HOST, MQR_DEVICE or MQR_DEVICE_RESIDENT");
    MQR_CHECK_HIP(hipSetDevice(v->device));
    // resident device frames (include/mqr.h): the caller keeps them unchanged until it synchronizes, so its
    // stream is not made to wait for this call's integrates at the return
    const bool resident = depth_loc == MQR_DEVICE_RESIDENT;
    if (resident) depth_loc = MQR_DEVICE;
    // device frames: both streams read them (touch, integrate) -- ordered after the caller's writes, from
    // the first batch's touch on (its frame-parameter upload and counter clear need not wait for them)
    bool caller_ordered = depth_loc != MQR_DEVICE;
    const int64_t HW = (int64_t)H * W;
    const float sdf_trunc = v->voxel_size * trunc_mult;
    const float block_size = v->voxel_size * v->R;
    const int64_t max_touch = 4LL * (H / 4) * (W / 4);
    std::vector<int> valid;
    for (int i = 0; i < B; ++i)
        if (!frame_ok || frame_ok[i]) valid.push_back(i);
    const int64_t wb0 = v->wbound;  // weights before the call: a batch ending at frame e keeps them <= wb0 + e
    if (v->wbound >= 0) v->wbound += (int64_t)valid.size();  // (an upper bound even if the call fails part-way)
    int rc = 0;
    int batch = 0;
    // batches of up to batch_frames frames (127), the first of a call a full batch as well
    // (first_batch_frames; variant bits 21-23 shorten it for A/Bs): its touch runs
    // before any integrate, the later ones behind the previous batch's integrate
    const size_t nb = (size_t)std::max(1, std::min(v->batch_frames, kMaxBatch));
    const size_t nb0 = (size_t)std::max(1, std::min(v->first_batch_frames, (int)nb));
    int b = 0;
    for (size_t s = 0; s < valid.size(); s += (size_t)b, ++batch) {
        const int p = v->pipelined ? (batch & 1) : 0;
        b = (int)std::min<size_t>(batch == 0 ? nb0 : nb, valid.size() - s);
        const int* idx = valid.data() + s;
        if (ensure_fp(v, b)) return 1;
        if (depth_loc != MQR_DEVICE && ensure_depth(v, b * HW)) return 1;
        if (wait_parity_free(v, p)) return 1;
        const float* dbase = depths;
        int64_t dframe[kMaxBatch];
        if (depth_loc == MQR_DEVICE) {
            for (int f = 0; f < b; ++f) dframe[f] = idx[f];
        } else {
            // one copy per run of consecutive source frames (all of them when no frame is skipped): a
            // 150 MB pageable upload runs near the link rate, 127 per-frame ones of 1.2 MB do not
            for (int f = 0; f < b;) {
                int e = f + 1;
                while (e < b && idx[e] == idx[e - 1] + 1) ++e;
                MQR_CHECK_HIP(hipMemcpyAsync(v->d_depth[p] + f * HW, depths + (int64_t)idx[f] * HW,
                                             sizeof(float) * HW * (e - f), hipMemcpyHostToDevice, v->stream));
                for (int g = f; g < e; ++g) dframe[g] = g;
                f = e;
            }
            dbase = v->d_depth[p];
        }
        const int64_t pool_before = v->pool_count;
        if (upload_frames(v, p, K, T_wc, idx, b, dframe) || reset_batch_counters(v, p)) return 1;
        // The first batch of a call: its integrate is enqueued right behind its touch, gated on the
        // device by the touch's own counters (k_gate), so the GPU does not idle while the host reads
        // them.  Later batches' counters are read while the previous integrate runs anyway.
        const bool spec = batch == 0 && v->spec_head && v->pipelined && !v->probe_one && v->batch_n_max > 0;
        if (!caller_ordered) {
            if (order_after_caller(v->device, v->stream, v->stream2)) return 2;
            caller_ordered = true;
        }
        TouchState ts;
        if (touch_batch_launch(v, p, dbase, HW, H, W, b, depth_scale, depth_max, sdf_trunc, block_size, max_touch, ts))
            return 1;
        v->launch_wbound = wb0 >= 0 ? wb0 + (int64_t)s + b : -1;  // this batch's weight bound (the LDS table)
        if (spec) {
            const int64_t grid = std::min<int64_t>(std::max<int64_t>(v->batch_n_max + v->batch_n_max / 4, 256), 8192);
            const size_t ev_before = v->int_events.size();
            if (launch_integrate(v, p, dbase, HW, H, W, b, depth_scale, depth_max, sdf_trunc, (int)pool_before, grid))
                return 1;
            if (read_counters(v, p)) return 1;  // the touch's counters (the integrate keeps running)
            const int* c = v->hctr(p);
            bool gated = c[kOverflow] != 0;
            for (int f = 0; f < b; ++f) gated |= c[kFrameCounterBase + f] == 0;
            if (!gated) {  // the speculative integrate is the batch's integrate (k_gate agreed)
                v->pool_count = v->h_counters[2 * kCountersTotal];
                v->batch_new_max = std::max(v->batch_new_max, v->pool_count - ts.pool_before);
                const int64_t n = std::min<int64_t>(c[kListCount], v->list_cap);
                v->batch_n_max = std::max(v->batch_n_max, n);
                if (v->profile) {
                    v->stats.integrate_launches += 1;
                    v->stats.union_blocks += n;
                    for (int f = 0; f < kMaxBatch; ++f) v->stats.frame_blocks += c[kFreshBase + f];
                    v->stats.frames += b;
                }
                continue;
            }
            // gated: the integrate did nothing (and cleared no slot mark); redo the batch's tail the
            // ordinary way once it has finished
            MQR_CHECK_HIP(hipStreamSynchronize(v->stream2));
            v->int_pending[p] = false;
            if (v->profile && v->int_events.size() > ev_before) v->int_events.resize(ev_before);
        }
        if (touch_batch_resolve(v, p, dbase, HW, H, W, b, depth_scale, depth_max, sdf_trunc, block_size, ts)) return 1;
        v->batch_n_max = std::max<int64_t>(v->batch_n_max, std::min<int64_t>(v->hctr(p)[kListCount], v->list_cap));
        int empty = -1;  // first frame of the batch that touched no block
        for (int f = 0; f < b && empty < 0; ++f)
            if (v->hctr(p)[kFrameCounterBase + f] == 0) empty = f;
        if (empty >= 0) {
            // Open3D raises at frame `empty` (DepthTouch) after integrating the frames
            // before it and before touching anything after it: undo the whole batch's touch (slot marks,
            // blocks it allocated), then integrate the prefix [0, empty) as a batch of its own.
            set_error(kNoBlock);
            rc = 3;
            if (undo_touch(v, p, pool_before)) return 1;
            if (empty > 0) {
                v->launch_wbound = wb0 >= 0 ? wb0 + (int64_t)s + empty : -1;
                if (upload_frames(v, p, K, T_wc, idx, empty, dframe) || reset_batch_counters(v, p)) return 1;
                if (touch_batch(v, p, dbase, HW, H, W, empty, depth_scale, depth_max, sdf_trunc, block_size,
                                max_touch))
                    return 1;
                if (launch_integrate(v, p, dbase, HW, H, W, empty, depth_scale, depth_max, sdf_trunc, (int)pool_before))
                    return 1;
            }
            break;
        }
        if (launch_integrate(v, p, dbase, HW, H, W, b, depth_scale, depth_max, sdf_trunc, (int)pool_before)) return 1;
    }
    if (rc == 0 && depth_loc == MQR_DEVICE && v->async_return) {
        // Device frames, no error: every batch's counters have been read (pool growth, empty frames), so
        // nothing is left to decide on the host -- return with the last integrate queued.  The caller's
        // stream waits for it (its next write to the frames is ordered after the library's reads); the
        // volume's next user orders behind it on the device (order_after_integrate, wait_parity_free) or
        // drains it (sync_all).  Host frames stay synchronous: the caller's array is read by copies.
        // Resident frames: no caller-stream wait -- the caller's next work (the next call's touch included,
        // which orders itself after the caller stream) need not queue behind this call's last integrate.
        return resident ? 0 : order_caller_after_integrate(v);
    }
    if (sync_all(v)) return 1;
    if (rc) set_error(kNoBlock);  // the prefix re-run may have overwritten the message
    return rc;
}

int mqr_touch(mqr_vbg* v, const float* depth, int depth_loc, int H, int W, const double* K, const double* T_wc,
              float depth_scale, float depth_max, float trunc_mult, int32_t* keys_out, int64_t* n_out) {
    MQR_REQUIRE(v && depth && K && T_wc && keys_out && n_out, "null argument");
    MQR_CHECK_HIP(hipSetDevice(v->device));
    if (sync_all(v)) return 1;
    if (depth_loc == MQR_DEVICE && order_after_caller(v->device, v->stream)) return 2;
    const int64_t HW = (int64_t)H * W;
    const int64_t max_touch = 4LL * (H / 4) * (W / 4);
    const int64_t want = next_pow2(2 * std::max<int64_t>(max_touch, 1));
    if (v->ftab.cap < want) {
        free_table(v->ftab);
        if (alloc_table(v->ftab, want, v->stream)) return 1;
    }
    if (ensure_lists(v, std::max(v->tab.cap, v->ftab.cap))) return 1;
    const float* dptr = depth;
    if (depth_loc != MQR_DEVICE) {
        if (ensure_depth(v, HW)) return 1;
        MQR_CHECK_HIP(hipMemcpyAsync(v->d_depth[0], depth, sizeof(float) * HW, hipMemcpyHostToDevice, v->stream));
        dptr = v->d_depth[0];
    }
    const int idx = 0;
    const int64_t dframe = 0;
    if (upload_frames(v, 0, K, T_wc, &idx, 1, &dframe) || reset_batch_counters(v, 0)) return 1;
    if (touch_launch(v, 0, dptr, HW, H, W, 1, depth_scale, depth_max, v->voxel_size * trunc_mult,
                     v->voxel_size * v->R, v->ftab, 0, v->ftab.cap))
        return 1;
    if (read_counters(v, 0)) return 1;
    const int64_t cnt = v->hctr(0)[kListCount];
    int32_t* dkeys = nullptr;
    if (cnt > 0) {
        MQR_CHECK_HIP(hipMalloc(&dkeys, sizeof(int32_t) * 3 * cnt));
        hipLaunchKernelGGL(k_gather_keys, dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0, v->stream, v->lists[0],
                           cnt, v->ftab, dkeys);
        MQR_CHECK_HIP(hipMemcpyAsync(keys_out, dkeys, sizeof(int32_t) * 3 * cnt, hipMemcpyDeviceToHost, v->stream));
        hipLaunchKernelGGL(k_clear_slots, dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0, v->stream, v->lists[0],
                           cnt, v->ftab, 1);
        MQR_CHECK_HIP(hipStreamSynchronize(v->stream));
        MQR_CHECK_HIP(hipFree(dkeys));
    }
    *n_out = cnt;
    if (v->hctr(0)[kFrameCounterBase] == 0) {
        set_error(kNoBlock);
        return 3;
    }
    return 0;
}

int mqr_integrate(mqr_vbg* v, const int32_t* keys, int64_t n, const float* depth, int depth_loc, int H, int W,
                  const double* K, const double* T_wc, float depth_scale, float depth_max, float trunc_mult) {
    MQR_REQUIRE(v && depth && K && T_wc && (keys || n == 0), "null argument");
    MQR_CHECK_HIP(hipSetDevice(v->device));
    if (n == 0) return 0;
    if (v->wbound >= 0) v->wbound += 1;
    if (sync_all(v)) return 1;
    if (depth_loc == MQR_DEVICE && order_after_caller(v->device, v->stream, v->stream2)) return 2;
    const int64_t HW = (int64_t)H * W;
    if (ensure_table(v, v->pool_count + n)) return 1;
    const float* dptr = depth;
    if (depth_loc != MQR_DEVICE) {
        if (ensure_depth(v, HW)) return 1;
        MQR_CHECK_HIP(hipMemcpyAsync(v->d_depth[0], depth, sizeof(float) * HW, hipMemcpyHostToDevice, v->stream));
        dptr = v->d_depth[0];
    }
    int32_t* dkeys = nullptr;
    MQR_CHECK_HIP(hipMalloc(&dkeys, sizeof(int32_t) * 3 * n));
    MQR_CHECK_HIP(hipMemcpyAsync(dkeys, keys, sizeof(int32_t) * 3 * n, hipMemcpyHostToDevice, v->stream));
    const int idx = 0;
    const int64_t dframe = 0;
    const int64_t pool_before = v->pool_count;
    if (upload_frames(v, 0, K, T_wc, &idx, 1, &dframe) || reset_batch_counters(v, 0)) return 1;
    hipLaunchKernelGGL(k_activate, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, v->stream, dkeys, n, v->table(0),
                       v->ctr(0), v->pool_ctr(), v->pool_cap, v->bkeys, v->lists[0], v->list_cap, 1);
    MQR_CHECK_HIP(hipGetLastError());
    if (resolve_pool_overflow(v, 0)) {
        (void)hipFree(dkeys);
        return 1;
    }
    v->launch_wbound = v->wbound;
    int rc = launch_integrate(v, 0, dptr, HW, H, W, 1, depth_scale, depth_max, v->voxel_size * trunc_mult,
                              (int)pool_before);
    if (sync_all(v)) rc = 1;
    MQR_CHECK_HIP(hipFree(dkeys));
    return rc;
}

int mqr_vbg_export(mqr_vbg* v, int32_t* keys, float* tsdf, float* weight, int loc) {
    MQR_REQUIRE(v, "null volume");
    MQR_CHECK_HIP(hipSetDevice(v->device));
    if (sync_all(v)) return 1;
    const int64_t n = v->pool_count;
    if (n == 0) return 0;
    if (loc == MQR_DEVICE && order_after_caller(v->device, v->stream)) return 2;  // the caller may still read them
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
    if (sync_all(v) || ensure_table(v, v->pool_count + U) || reset_batch_counters(v, 0)) return 1;
    if (U > 0)
        hipLaunchKernelGGL(k_activate, dim3((unsigned)((U + 255) / 256)), dim3(256), 0, v->stream, dkeys, U,
                           v->table(0), v->ctr(0), v->pool_ctr(), v->pool_cap, v->bkeys, v->lists[0], v->list_cap, 0);
    MQR_CHECK_HIP(hipGetLastError());
    return resolve_pool_overflow(v, 0);
}

int mqr_vbg_import(mqr_vbg* v, const int32_t* keys, const float* tsdf, const float* weight, int64_t n, int loc) {
    MQR_REQUIRE(v && ((keys && tsdf && weight) || n == 0), "null argument");
    MQR_CHECK_HIP(hipSetDevice(v->device));
    if (n == 0) return 0;
    v->wbound = -1;  // arbitrary weights: the merge keeps them float32
    if (sync_all(v)) return 1;
    if (loc == MQR_DEVICE && order_after_caller(v->device, v->stream)) return 2;
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
    if (sync_all(v)) return 1;
    if (order_after_caller(v->device, v->stream)) return 2;
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
    v->wbound = -1;
    if (sync_all(v)) return 1;
    if (order_after_caller(v->device, v->stream)) return 2;
    if (activate_device_keys(v, union_keys, U)) return 1;
    hipLaunchKernelGGL(k_unpack, dim3((unsigned)U), dim3(256), 0, v->stream, union_keys, U, v->tab, v->pool,
                       (int)v->R3, reinterpret_cast<const float2*>(packed));
    MQR_CHECK_HIP(hipGetLastError());
    MQR_CHECK_HIP(hipStreamSynchronize(v->stream));
    return 0;
}

int mqr_vbg_set_variant(mqr_vbg* v, int variant) {
    MQR_REQUIRE(v, "null volume");
    if (sync_all(v)) return 1;
    if (!MQR_AB && (((variant & 0xff) != 0 && (variant & 0xff) != 1 && (variant & 0xff) != 2 && (variant & 0xff) != 4) || (variant & 0x8000))) {
        set_error("integrate variant " + std::to_string(variant) + " is an A/B kernel: only in tools/_ab/libmqr_ab.so (make ab)");
        return 1;
    }
    v->kernel_variant = variant & 0xff;
    v->pipelined = (variant & 0x100) == 0;  // bit 8: serialise touch and integrate (A/B of the overlap)
    // (the integrate stream rather than the touch stream at the device's highest priority measured
    // 2.592 vs 2.587 ms per step: removed)
    // (the later batches' touches on a stream restricted to 32 / 64 / 128 CUs measured 3.07 / 2.72 /
    // 2.61 vs 2.54-2.58 ms per step -- the overlapped touch barely slows the integrate: removed)
    v->lpt_order = (variant & 0x200) == 0;  // bit 9: integrate in touch order instead of longest-first
    // bit 10: 32-frame batches; bit 20: 64-frame batches (round 3) (A/Bs)
    v->batch_frames = (variant & 0x400) ? 32 : (variant & 0x100000) ? 64 : kMaxBatch;
    // bits 21 / 22 / 23: a first batch of 64 / 32 / 16 frames (A/B of the step head)
    v->first_batch_frames = (variant & 0x200000) ? 64 : (variant & 0x400000) ? 32 : (variant & 0x800000) ? 16 : kFirstBatch;
    v->sys_fence = (variant & 0x800) != 0;  // bit 11: system-scope ordering / timing events (A/B)
    v->probe_one = (variant & 0x1000) != 0; // bit 12: force the full-table retry path (test hook)
    v->table_worst = (variant & 0x2000) != 0; // bit 13: size the table for the worst case (round-2 A/B)
    v->touch_wait = (variant & 0x4000) != 0;  // bit 14: integrate always waits on a touch-stream event (A/B)
    v->xcd_order = (variant & 0x8000) != 0;   // bit 15: spatial per-XCD groups (k_xcd_order, A/B)
    v->touch_ppt = (variant & 0x10000) ? 1 : 2;  // bit 16: one stride-4 pixel per touch thread (A/B)
    v->spec_head = (variant & 0x40000) == 0;     // bit 18: no speculative first-batch integrate (A/B)
    v->async_return = (variant & 0x1000000) == 0; // bit 24: integrate_frames drains its streams before returning (A/B)
    v->flip_reset = (variant & 0x2000000) == 0;   // bit 25: reset waits for an in-flight integrate (no set swap, A/B)
    v->rtab = (variant & 0x4000000) == 0;         // bit 26: k_integrate_win instead of the LDS-table kernel (A/B)
    v->div1 = (variant & 0x8000000) == 0;         // bit 27: the LDS-table kernel keeps two quotient corrections (A/B)
    // (the extraction configuration is set by mqr_vbg_set_extract_mode alone, A/B library only)
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
        if (which == 0 || which == 3 || which == 4)
            hipLaunchKernelGGL(k_check_rcp, dim3(blocks), dim3(256), 0, 0, which == 0 ? 0 : which - 2,
                               lo_bits + (uint32_t)off, c, d, d + 1);
        else
            hipLaunchKernelGGL(k_check_div, dim3(blocks), dim3(256), 0, 0, which == 2 ? 1 : 0, b,
                               lo_bits + (uint32_t)off, c, d, d + 1);
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
    // enable: 1 = integrate launches (2 events per batch), 2 = also the touch launches (4)
    v->profile = enable != 0;
    v->profile_touch = enable >= 2;
    // create the timing events now, outside any timed region (more are created on demand until the
    // next stats read recycles them)
    MQR_CHECK_HIP(hipSetDevice(v->device));
    if (v->profile && v->ev_pool_sys != v->sys_fence) {  // the fence scope changed: rebuild the pool
        if (sync_all(v)) return 1;
        drain_events(v);
        for (hipEvent_t e : v->ev_pool) (void)hipEventDestroy(e);
        v->ev_pool.clear();
        v->ev_pool_sys = v->sys_fence;
    }
    while (v->profile && v->ev_pool.size() < 12288) {
        hipEvent_t e = nullptr;
        MQR_CHECK_HIP(hipEventCreateWithFlags(&e, v->timing_event_flags()));
        v->ev_pool.push_back(e);
    }
    return 0;
}

int mqr_vbg_stats(mqr_vbg* v, mqr_stats* out, int reset) {
    MQR_REQUIRE(v && out, "null argument");
    MQR_CHECK_HIP(hipSetDevice(v->device));
    if (sync_all(v)) return 1;
    drain_events(v);
    *out = v->stats;
    if (reset) v->stats = mqr_stats{};
    return 0;
}

}  // extern "C"

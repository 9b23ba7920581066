// Shared internals of libmqr_hip.so: error plumbing, block-key packing, the HBM-resident
// block hash table and the volume object.  gfx950 only; built with -ffp-contract=off so
// every float op rounds exactly as the Open3D 0.19 reference kernels specify.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "mqr.h"

namespace mqr {

// ---------------------------------------------------------------- errors
void set_error(const std::string& msg);
const char* get_error();

#define MQR_CHECK_HIP(expr)                                                                   \
    do {                                                                                      \
        hipError_t _e = (expr);                                                               \
        if (_e != hipSuccess) {                                                               \
            ::mqr::set_error(std::string(#expr) + ": " + hipGetErrorString(_e));              \
            return 1;                                                                         \
        }                                                                                     \
    } while (0)

#define MQR_REQUIRE(cond, msg)                                                                \
    do {                                                                                      \
        if (!(cond)) {                                                                        \
            ::mqr::set_error(msg);                                                            \
            return 2;                                                                         \
        }                                                                                     \
    } while (0)

// ---------------------------------------------------------------- keys
// A block key (xb, yb, zb) packs into 63 bits (21 per axis, bias 2^20).  EMPTY is all ones.
constexpr uint64_t kEmpty = ~0ull;
constexpr int kBias = 1 << 20;

__host__ __device__ inline uint64_t pack_key(int x, int y, int z) {
    return ((uint64_t)(uint32_t)(x + kBias) << 42) | ((uint64_t)(uint32_t)(y + kBias) << 21) |
           (uint64_t)(uint32_t)(z + kBias);
}
__host__ __device__ inline bool key_in_range(int x, int y, int z) {
    return x >= -kBias && x < kBias && y >= -kBias && y < kBias && z >= -kBias && z < kBias;
}
__host__ __device__ inline void unpack_key(uint64_t k, int& x, int& y, int& z) {
    x = (int)((k >> 42) & 0x1FFFFF) - kBias;
    y = (int)((k >> 21) & 0x1FFFFF) - kBias;
    z = (int)(k & 0x1FFFFF) - kBias;
}
__host__ __device__ inline uint64_t mix64(uint64_t k) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdull;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ull;
    k ^= k >> 33;
    return k;
}

// ---------------------------------------------------------------- hash table (device view)
// Open addressing, linear probing, 64-bit keys claimed by atomicCAS.  vals = pool buffer
// index (-1 none yet, -2 pool overflow), mask = frames of the current batch that touched it.
// Slot mask of a device batch: bit f = frame f of the batch touched the block (f < kMaxBatch = 127);
// bit 127 = the slot is on the batch list (set by whichever frame's mark first found its 64-bit word
// empty and won the flag: two words, so "the whole mask was empty" is not one atomic).  Readers that
// iterate frames strip it (bm_frames).
typedef unsigned __int128 bmask_t;
constexpr unsigned long long kListedBit = 1ull << 63;  // in word 1
__host__ __device__ inline bmask_t bm_frames(bmask_t m) { return m & ~((bmask_t)kListedBit << 64); }
__host__ __device__ inline int bm_popc(bmask_t m) {
    return __builtin_popcountll((unsigned long long)m) + __builtin_popcountll((unsigned long long)(m >> 64));
}
__host__ __device__ inline int bm_ctz(bmask_t m) {  // m != 0
    const unsigned long long lo = (unsigned long long)m;
    return lo ? __builtin_ctzll(lo) : 64 + __builtin_ctzll((unsigned long long)(m >> 64));
}
struct Table {
    uint64_t* keys;
    int32_t* vals;
    bmask_t* mask;
    int64_t cap;  // power of two
};

// Device counters (one int each, zeroed/maintained by the host around each batch).
enum Counter : int {
    kPoolCount = 0,   // allocated pool buffers
    kListCount = 1,   // slots appended to the batch list
    kOverflow = 2,    // bit0 pool overflow, bit1 table full, bit2 list overflow, bit3 key range
    kTouched = 3,     // raw (pre-dedup) touched samples
    kFrameBlocks = 4, // (unused: per-frame new marks live at kFreshBase + f)
    kBadCount = 5,    // blocks the fast integrate kernel handed to the exact fix-up launch
    kNumCounters = 8
};

// Per-frame parameters as Open3D's TransformIndexer holds them: float32 copies of K and the
// 3x4 extrinsic (integrate), and of the float64 rigid inverse (touch).
struct FrameParams {
    float fx, fy, cx, cy;
    float ext[12];
    float pose[12];
};

void make_frame_params(const double* K, const double* T_wc, FrameParams* fp);

constexpr int kMaxBatch = 127;        // frames per device batch (one bit each in the slot mask)
// frames of a call's first batch (its touch runs before any integrate): a full batch -- a 64-frame
// first batch starts the first integrate sooner but adds a launch (2.551 vs 2.499 ms per C2 step,
// profiles/r04_ab_integrate.json)
constexpr int kFirstBatch = kMaxBatch;
constexpr int kFrameCounterBase = 8;  // per-frame raw touch counts live at counters[8 + f]
constexpr int kFreshBase = kFrameCounterBase + kMaxBatch;  // per-frame new (block, frame) marks
constexpr int kNumGroups = 8;                               // workgroup groups that share an XCD
constexpr int kGroupBase = kFreshBase + kMaxBatch;          // k_xcd_order: group g = [off[g], off[g+1])
constexpr int kCountersTotal = kGroupBase + kNumGroups + 1;
// device counter ints: 2 parity sets, the pool counter (+ spare), 2 shadow sets (k_gate: the copies a
// speculatively launched integrate reads)
constexpr int kCounterInts = 4 * kCountersTotal + 8;

// ---------------------------------------------------------------- volume
}  // namespace mqr

struct mqr_vbg {
    int device = 0;
    float voxel_size = 0.f;
    int R = 16;
    int64_t R3 = 4096;
    // Two streams: touch(b+1) on `stream` overlaps integrate(b) on `stream2`.  Per-batch state
    // (slot masks, slot lists, counters, frame parameters, staged depth) is double-buffered by
    // batch parity; the hash table, pool and pool counter are shared.
    hipStream_t stream = nullptr;
    hipStream_t stream2 = nullptr;
    // Ordering events between the two streams are recorded with a DEVICE-scope release
    // (hipEventDisableSystemFence): a default (system-scope) event makes the packet processor write
    // back and invalidate every XCD's L2 at the record -- ~20 us between consecutive integrate
    // launches, and the next kernel starts cold.  Only ev_host (the host's read of the batch
    // counters through pinned memory) keeps the system-scope release.  sys_fence (variant bit
    // 0x800) records the system-scope twins instead, for the A/B.
    hipEvent_t ev_touch[2] = {nullptr, nullptr};
    hipEvent_t ev_int[2] = {nullptr, nullptr};
    hipEvent_t ev_touch_sys[2] = {nullptr, nullptr};
    hipEvent_t ev_int_sys[2] = {nullptr, nullptr};
    hipEvent_t ev_host[2] = {nullptr, nullptr};
    bool sys_fence = false;
    bool int_pending[2] = {false, false};
    bool lpt_ready[2] = {false, false};  // k_lpt_order already enqueued behind this parity's touch
    bool ctr_clean[2] = {true, true};    // the parity's counters are zero (a reset cleared them)
    bool spec_head = true;               // first batch of a call: integrate enqueued behind its touch (k_gate)
    // mqr_integrate_frames on device frames returns once its last integrate is queued (the caller's stream
    // waits for it; the volume's next user orders behind it on the device) instead of draining the streams
    bool async_return = true;
    bool act_check = false;  // activate_ordered's table-full check is still to be read (activate_ordered_check)
    int64_t batch_n_max = 0;             // largest batch list seen (grid of a speculative integrate)
    hipEvent_t touch_ev(int p) const { return sys_fence ? ev_touch_sys[p] : ev_touch[p]; }
    hipEvent_t int_ev(int p) const { return sys_fence ? ev_int_sys[p] : ev_int[p]; }
    // the event that last closed parity p's integrate on its stream: int_ev(p), or, while profiling,
    // that launch's timing end event (one event record between launches instead of two)
    hipEvent_t int_done[2] = {nullptr, nullptr};

    mqr::Table tab{};          // main block table (tab.mask == mask[0])
    mqr::bmask_t* mask1 = nullptr; // parity-1 slot masks
    mqr::Table ftab{};         // frustum table for mqr_touch (Open3D's separate frustum hash map)
    float2* pool = nullptr;    // [pool_cap][R3] (tsdf, weight)
    uint64_t* bkeys = nullptr; // [pool_cap] packed key of each buffer
    int64_t pool_cap = 0;
    int64_t pool_count = 0;    // host mirror (valid after each batch)
    // Upper bound of any voxel's weight (every integrated frame adds at most 1): the merge sends weights as
    // uint16 when every rank's bound is <= 65535.  -1 = unknown (imported or unpacked contents).
    int64_t wbound = 0;
    int64_t batch_new_max = 0; // most blocks one integrate batch has allocated (sizes the table headroom)
    // Weight bound of the next integrate launch (set by its caller: the weights before the call plus the frames
    // up to the batch's end; -1 unknown): the default kernel's LDS table of (w, 1 / (w + 1)) has this many
    // entries (k_integrate_wt; without a bound, or above kRtabMax, k_integrate_win runs).
    int64_t launch_wbound = -1;
    bool rtab = true;  // variant bit 26 clears it (A/B)
    bool div1 = true;  // one-correction s / sdf_trunc where verified (strunc_one_correction_ok); bit 27 clears it

    // Second table / pool set.  mqr_vbg_reset while an integrate is still in flight swaps the sets instead of
    // ordering the clear behind that integrate: the next call's touch then overlaps the previous call's last
    // integrate.  set_ev marks, on stream2, the last integrate that used a set while it was
    // current; a set swapped back in is cleared behind it.  Kept only for volumes within kAltMaxBytes and
    // while the device keeps a quarter of its HBM free; variant bit 25 turns the swap off.
    struct VolSet {
        mqr::Table tab{};
        mqr::bmask_t* mask1 = nullptr;
        float2* pool = nullptr;
        uint64_t* bkeys = nullptr;
        int64_t pool_cap = 0;
        hipEvent_t ev = nullptr;
        bool ev_live = false;
    } alt;
    hipEvent_t set_ev = nullptr;  // the current set's event (swapped with alt.ev)
    bool set_ev_live = false;
    bool flip_reset = true;
    int64_t flips = 0;  // resets that swapped the sets (mqr_vbg_flips)

    int32_t* lists[2] = {nullptr, nullptr};  // batch slot lists, capacity list_cap each
    int32_t* lpt[2] = {nullptr, nullptr};    // the same lists reordered (k_lpt_order / k_xcd_order): slots,
                                             // then their masks, then a group byte per entry (scratch)
    int32_t* bad[2] = {nullptr, nullptr};    // fast-kernel fix-up list: slots, then their masks
    int64_t list_cap = 0;
    int* counters = nullptr;   // device: 2 x kCountersTotal per-parity sets, then the pool counter
    int* h_counters = nullptr; // pinned mirror, same layout

    mqr::FrameParams* d_fp[2] = {nullptr, nullptr};  // frame params (+ int64 depth-frame index array)
    mqr::FrameParams* h_fp[2] = {nullptr, nullptr};  // pinned mirrors
    int fp_cap = 0;
    float* d_depth[2] = {nullptr, nullptr};          // staging for host depth frames
    int64_t depth_cap = 0;                           // floats per parity
    void* ex_scratch = nullptr;                      // extraction scratch (grow-only, extract.hip)
    size_t ex_scratch_bytes = 0;
    int64_t* h_ex = nullptr;                         // pinned totals of the extraction scans
    int64_t ex_hint[3] = {0, 0, 0};  // last extraction's vertex / triangle / point counts (speculative capacity)

    int kernel_variant = 0;    // integrate kernel configuration (launch_integrate in vbg.hip), 1 = generic
    bool pipelined = true;     // overlap touch(b+1) with integrate(b)
    bool lpt_order = true;     // integrate blocks in longest-first order
    bool xcd_order = false;    // spatial groups per XCD (k_xcd_order; variant bit 0x8000, A/B)
    bool touch_wait = false;   // integrate waits on a touch-stream event every batch (variant bit 0x4000, A/B)
    bool table_worst = false;  // table sized for every sample a new block (variant bit 0x2000, A/B)
    bool probe_one = false;    // batch touch probes one slot per new key (variant bit 0x1000, test hook)
    int batch_frames = mqr::kMaxBatch;  // frames per device batch (A/B: 32, variant bit 0x400; 64, bit 20)
    int first_batch_frames = mqr::kFirstBatch;  // frames of a call's first batch
    // profiling
    int touch_ppt = 2;  // stride-4 pixels per k_touch thread (variant bit 16: one)
    int ex_mode = -1;   // extraction configuration under A/B (-1: the library default kExMode; tools/ab_extract.py)
    int last_var = -1;        // integrate variant of the last launch, after fallbacks (mqr_vbg_last_kernel)
    const char* last_kname = "";  // its main kernel (mqr_vbg_last_kernel_name)
    bool profile = false;
    bool profile_touch = false;  // mqr_vbg_profile level 2: also time the touch launches
    std::vector<std::pair<hipEvent_t, hipEvent_t>> int_events, touch_events;
    std::vector<hipEvent_t> ev_pool;  // timing events, created once and reused (hipEventCreate per
    size_t ev_used = 0;               // launch added ~0.1 ms to a 500-frame step); device-scope
    bool ev_pool_sys = false;         // release unless sys_fence (then a pool of default events)
    unsigned timing_event_flags() const { return sys_fence ? hipEventDefault : hipEventDisableSystemFence; }
    hipEvent_t pooled_event() {
        if (ev_used == ev_pool.size()) {
            hipEvent_t e = nullptr;
            if (hipEventCreateWithFlags(&e, timing_event_flags()) != hipSuccess) return nullptr;
            ev_pool.push_back(e);
        }
        return ev_pool[ev_used++];
    }
    mqr_stats stats{};

    mqr::Table table(int parity) const {
        mqr::Table t = tab;
        t.mask = parity ? mask1 : tab.mask;
        return t;
    }
    int* ctr(int parity) const { return counters + parity * mqr::kCountersTotal; }
    int* hctr(int parity) const { return h_counters + parity * mqr::kCountersTotal; }
    int* pool_ctr() const { return counters + 2 * mqr::kCountersTotal; }
    int* shadow(int parity) const { return counters + 2 * mqr::kCountersTotal + 8 + parity * mqr::kCountersTotal; }
};

// Device-resident geometry result (extract.hip, meshfilter.hip); released by mqr_geom_free.
struct mqr_geom {
    int device = 0;
    int64_t nv = 0, nt = 0;
    float* pos = nullptr;
    float* nrm = nullptr;
    int32_t* tri = nullptr;
    void* blk = nullptr;  // when set, pos / nrm / tri are carved from this one allocation
    size_t blk_cap = 0;   // its size (a recycled block may be larger than needed)
};

namespace mqr {
// Device blocks for geometry results, recycled by mqr_geom_free (a few per device) instead of
// hipFree + hipMalloc: hipFree synchronises the device and a fresh multi-10-MB hipMalloc maps new
// pages, together 1-3 ms per extraction of a 2 M-triangle mesh.
void* geom_block_alloc(int device, size_t bytes, size_t* cap);
void geom_block_release(int device, void* p, size_t cap);
int grow_pool(mqr_vbg* v, int64_t need);
int sync_all(mqr_vbg* v);
// Work enqueued on the volume's `stream` from here on runs after any integrate still in flight on its second
// stream (a device-side wait; no host synchronisation when nothing is in flight, the usual case).
int order_after_integrate(mqr_vbg* v);
// Caller-stream ordering (mqr_set_stream, include/mqr.h): the library streams `a` (and `b`) wait for
// every command the calling thread's caller stream holds so far.  Called by each entry point that
// reads or writes caller MQR_DEVICE buffers, before its first command on them (the current device
// must be `device`).  Every entry point but one drains its own streams before it returns, so outputs
// need no ordering in the other direction; mqr_integrate_frames on device frames instead makes the caller
// stream wait for its last integrate (order_caller_after_integrate).
int order_after_caller(int device, hipStream_t a, hipStream_t b = nullptr);
// The caller stream waits (device-side) for every integrate of `v` still in flight: what the caller
// enqueues there next -- e.g. overwriting the frames just integrated -- runs after the library's reads.
int order_caller_after_integrate(mqr_vbg* v);
hipStream_t caller_stream();  // the calling thread's caller stream (nullptr: the null stream)
// Large device -> pageable host copies by several host threads through pinned staging (extract.hip);
// mqr_geom_copy and mqr_memcpy use it from kD2HParallelMin bytes on.
constexpr size_t kD2HParallelMin = size_t(32) << 20;
int d2h_parallel(int device, void* dst, const void* src, size_t bytes);
// Host <-> device copies ordered on stream s, complete on return (the bytes are in place and the host
// buffer is free).  Downloads of kD2HParallelMin bytes or more into pageable memory go through the pinned
// ring, everything else is hipMemcpyAsync + a stream synchronize.  copy_stream(): the caller's stream
// (mqr_set_stream) when it is `device`'s, else null.
int copy_to_host(int device, void* dst, const void* src, size_t bytes, hipStream_t s);
int copy_to_device(int device, void* dst, const void* src, size_t bytes, hipStream_t s);
hipStream_t copy_stream(int device);
int activate_ordered(mqr_vbg* v, const uint64_t* dkeys, int64_t n, bool merge_writes_all);  // empty volume, buffer i = key i
int activate_ordered_check(mqr_vbg* v);  // its table-full check (deferred when merge_writes_all)
}  // namespace mqr

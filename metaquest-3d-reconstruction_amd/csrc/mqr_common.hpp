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
struct Table {
    uint64_t* keys;
    int32_t* vals;
    uint32_t* mask;
    int64_t cap;  // power of two
};

// Device counters (one int each, zeroed/maintained by the host around each batch).
enum Counter : int {
    kPoolCount = 0,   // allocated pool buffers
    kListCount = 1,   // slots appended to the batch list
    kOverflow = 2,    // bit0 pool overflow, bit1 table full, bit2 list overflow, bit3 key range
    kTouched = 3,     // raw (pre-dedup) touched samples
    kFrameBlocks = 4, // sum over frames of touched blocks (per-frame unique)
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

// ---------------------------------------------------------------- volume
}  // namespace mqr

struct mqr_vbg {
    int device = 0;
    float voxel_size = 0.f;
    int R = 16;
    int64_t R3 = 4096;
    hipStream_t stream = nullptr;

    mqr::Table tab{};          // main block table
    mqr::Table ftab{};         // frustum table for mqr_touch (Open3D's separate frustum hash map)
    float2* pool = nullptr;    // [pool_cap][R3] (tsdf, weight)
    uint64_t* bkeys = nullptr; // [pool_cap] packed key of each buffer
    int64_t pool_cap = 0;
    int64_t pool_count = 0;    // host mirror (valid after each batch)

    int32_t* list = nullptr;   // batch slot list, capacity list_cap
    int64_t list_cap = 0;
    int* counters = nullptr;   // device counters
    int* h_counters = nullptr; // pinned mirror

    mqr::FrameParams* d_fp = nullptr;  // per-batch frame parameters (+ int64 depth-frame index array)
    mqr::FrameParams* h_fp = nullptr;  // pinned host mirror of d_fp
    int fp_cap = 0;
    float* d_depth = nullptr;          // staging for host depth frames
    int64_t depth_cap = 0;             // floats

    int kernel_variant = 0;            // 0 = R-specialised integrate, 1 = generic (A/B)
    // profiling
    bool profile = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> int_events, touch_events;
    mqr_stats stats{};
};

namespace mqr {
int ensure_fp(mqr_vbg* v, int n);
int ensure_depth(mqr_vbg* v, int64_t floats);
int grow_pool(mqr_vbg* v, int64_t need);
int sync_counters(mqr_vbg* v);
}  // namespace mqr

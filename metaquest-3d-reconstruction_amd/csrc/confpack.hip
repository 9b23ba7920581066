// confpack.hip -- the confidence maps' download as two bytes per pixel (SURVEY §8 C3 outputs).
//
// build_confidence_map's outputs (estimate_depth_confidences.py:41-79) are valid_count (int32) and
// confidence_map = np.true_divide(consistent_count, valid_count) (float64, 0 where valid_count is 0):
// both are functions of the two per-pixel counts, which are at most the window's neighbour count
// (2 * target_frame_range).  The drop-in driver (mqr/confidence.py) writes every reference frame's maps to
// an npz; downloading the 12 bytes per pixel the maps take was 45 of its 57 ms of compute per 500 frames
// at 640 x 480 (1.84 GB over the link).  Here the maps are computed into HBM by mqr_confidence, reduced on
// the device to (valid, consistent) byte pairs -- each pixel's consistent count recovered from the map and
// checked to give back the map's exact bits -- and only the pairs cross the link; the native npz writer
// (frameio.hip, mqr_write_confidence_npz_counts) expands them back, with the same correctly rounded
// float64 division, while it writes.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <mutex>

#include "mqr_common.hpp"

namespace {

// Pixel i: out = valid | consistent << 8; *bad set when a pixel does not fit (valid outside [0, 255]) or
// its map value is not exactly consistent / valid (never, for maps mqr_confidence made).
__global__ __launch_bounds__(256) void k_pack_counts(const double* __restrict__ conf, const int32_t* __restrict__ valid,
                                                     int64_t n, uint16_t* __restrict__ out, uint32_t* __restrict__ bad) {
    bool fail = false;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int32_t v = valid[i];
        const double c = conf[i];
        const bool in = v >= 0 && v <= 255;
        const int k = in && v > 0 ? (int)rint(c * (double)v) : 0;
        const double back = v > 0 ? (double)k / (double)v : 0.0;
        const bool ok = in && k >= 0 && k <= v && __double_as_longlong(back) == __double_as_longlong(c);
        fail |= !ok;
        out[i] = (uint16_t)((ok ? v : 0) | (ok ? k : 0) << 8);
    }
    if (__ballot(fail) && (threadIdx.x & 63) == 0) atomicOr(bad, 1u);
}

struct PackCtx {
    std::mutex mu;
    hipStream_t s = nullptr;
    void* maps = nullptr;  // [conf f64][valid i32] of the last call
    size_t maps_cap = 0;
    uint16_t* packed = nullptr;
    size_t packed_cap = 0;
    uint32_t* d_bad = nullptr;
    uint32_t* h_bad = nullptr;
};
PackCtx g_pack[64];

int grow(void** p, size_t* cap, size_t want) {
    if (*cap >= want) return 0;
    if (*p) MQR_CHECK_HIP(hipFree(*p));
    *p = nullptr;
    *cap = 0;
    MQR_CHECK_HIP(hipMalloc(p, want));
    *cap = want;
    return 0;
}

}  // namespace

extern "C" {

int mqr_confidence_counts(int device, const float* depths, int depth_loc, int N, int H, int W, const float* K,
                          const float* T_cw, const float* T_cw_inv, const uint8_t* frame_ok, int ref_begin,
                          int ref_end, int frame_range, double depth_max, double error_threshold, uint16_t* counts,
                          int* packed) {
    MQR_REQUIRE(counts && packed, "null argument");
    MQR_REQUIRE(device >= 0 && device < 64, "bad device");
    MQR_REQUIRE(N > 0 && H > 0 && W > 0 && ref_begin >= 0 && ref_begin <= ref_end && ref_end <= N, "bad shape");
    *packed = 0;
    const int64_t n = (int64_t)(ref_end - ref_begin) * H * W;
    if (n == 0) {
        *packed = 1;
        return 0;
    }
    PackCtx& c = g_pack[device];
    std::lock_guard<std::mutex> lock(c.mu);
    MQR_CHECK_HIP(hipSetDevice(device));
    if (!c.s) MQR_CHECK_HIP(hipStreamCreateWithFlags(&c.s, hipStreamNonBlocking));
    if (!c.d_bad) MQR_CHECK_HIP(hipMalloc(&c.d_bad, sizeof(uint32_t)));
    if (!c.h_bad) MQR_CHECK_HIP(hipHostMalloc(&c.h_bad, sizeof(uint32_t), hipHostMallocDefault));
    const size_t bc = (sizeof(double) * n + 255) & ~size_t(255);
    if (grow(&c.maps, &c.maps_cap, bc + sizeof(int32_t) * n) ||
        grow(reinterpret_cast<void**>(&c.packed), &c.packed_cap, sizeof(uint16_t) * n))
        return 1;
    double* dconf = static_cast<double*>(c.maps);
    int32_t* dvalid = reinterpret_cast<int32_t*>(static_cast<char*>(c.maps) + bc);
    // the maps into HBM (mqr_confidence orders itself after the caller's stream and returns complete)
    if (int rc = mqr_confidence(device, depths, depth_loc, N, H, W, K, T_cw, T_cw_inv, frame_ok, ref_begin, ref_end,
                                frame_range, depth_max, error_threshold, dconf, dvalid, MQR_DEVICE))
        return rc;
    MQR_CHECK_HIP(hipMemsetAsync(c.d_bad, 0, sizeof(uint32_t), c.s));
    const unsigned blocks = (unsigned)std::min<int64_t>((n + 255) / 256, 256 * 32);
    hipLaunchKernelGGL(k_pack_counts, dim3(blocks), dim3(256), 0, c.s, dconf, dvalid, n, c.packed, c.d_bad);
    MQR_CHECK_HIP(hipGetLastError());
    MQR_CHECK_HIP(hipMemcpyAsync(c.h_bad, c.d_bad, sizeof(uint32_t), hipMemcpyDeviceToHost, c.s));
    MQR_CHECK_HIP(hipStreamSynchronize(c.s));
    if (*c.h_bad) return 0;  // not representable: *packed stays 0 (the caller then runs mqr_confidence itself)
    if (mqr::copy_to_host(device, counts, c.packed, sizeof(uint16_t) * n, c.s)) return 1;
    MQR_CHECK_HIP(hipStreamSynchronize(c.s));
    *packed = 1;
    return 0;
}

}  // extern "C"

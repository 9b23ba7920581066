// ingest.hip -- device-side depth ingestion: Quest NDC depth buffers ->
// metric depth, the reference's frame-validity verdict and the confidence mask, in one pass.
//
//   DepthDataIO.load_depth_map / is_depth_map_valid   scripts/dataio/depth_data_io.py:33-53, 80-85
//   convert_depth_to_linear / to_linear_depth         scripts/utils/depth_utils.py:21-46
//   confidence masking in load_depth_map              processing/reconstruction/utils/o3d_utils.py:131-142
//
// numpy semantics restated exactly (numpy >= 2, NEP 50 promotion):
//   ndc   = d * 2.0 - 1.0                     float32 (Python-float operands are weak)
//   denom = ndc + y                           float32 if y is a Python float, float64 if y is a
//                                             numpy float64 scalar (DepthDataset.fars/nears)
//   out   = x / denom where denom != 0 else 0 float64 division if x or denom is float64, else
//                                             float32; stored to float32
// The caller says per frame which of near / far were numpy float64 scalars (mqr_decode_depth
// `strong`: bit 0 near, bit 1 far); x and y inherit that from the operands they are computed
// from, except y = -1.0 of the far = inf branch, which stays a Python float.
// Validity: any(d != 0) and any(d != 1) and no NaN and all(d >= 0).
// Mask: depth = 0 where conf < conf_thr, and where valid_count < count_thr.
#include <algorithm>
#include <cmath>
#include <vector>

#include "mqr_common.hpp"

namespace mqr {

struct DecodeFrame {
    double x, y;  // compute_ndc_to_linear_depth_params (float64, as Python computes them)
    int strong;   // bit0: x is a float64 scalar, bit1: y is (denominator in float64)
    int mask;     // apply the confidence mask to this frame
};

// validity flag bits accumulated per frame
constexpr uint32_t kAnyNonZero = 1, kAnyNonOne = 2, kAnyNaN = 4, kAnyNotGE0 = 8;

__global__ __launch_bounds__(256) void k_decode_depth(const float* __restrict__ raw, int64_t HW,
                                                      const DecodeFrame* __restrict__ frames,
                                                      const double* __restrict__ conf,
                                                      const int32_t* __restrict__ vcount, double conf_thr,
                                                      int count_thr, float* __restrict__ out,
                                                      uint32_t* __restrict__ flags) {
    const int f = blockIdx.y;
    const DecodeFrame fr = frames[f];
    const int64_t base = (int64_t)f * HW;
    uint32_t fl = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < HW; i += (int64_t)gridDim.x * blockDim.x) {
        const float d = raw[base + i];
        fl |= (d != 0.0f ? kAnyNonZero : 0u) | (d != 1.0f ? kAnyNonOne : 0u) | (d != d ? kAnyNaN : 0u) |
              (!(d >= 0.0f) ? kAnyNotGE0 : 0u);
        const float ndc = d * 2.0f - 1.0f;
        float z = 0.0f;
        if (fr.strong & 2) {
            const double den = (double)ndc + fr.y;
            if (den != 0.0) z = (float)(fr.x / den);
        } else {
            const float den = ndc + (float)fr.y;
            if (den != 0.0f) z = (fr.strong & 1) ? (float)(fr.x / (double)den) : (float)fr.x / den;
        }
        if (fr.mask) {
            if (conf[base + i] < conf_thr) z = 0.0f;
            if (vcount[base + i] < count_thr) z = 0.0f;
        }
        out[base + i] = z;
    }
    // wave-level OR, then one atomic per wave only for bits the frame's word does not have yet
    // (every wave of a frame would otherwise hit the same address: thousands of serialised atomics)
    for (int o = 32; o > 0; o >>= 1) fl |= (uint32_t)__shfl_xor((int)fl, o, 64);
    if ((threadIdx.x & 63) == 0 && (fl & ~__atomic_load_n(&flags[f], __ATOMIC_RELAXED))) atomicOr(&flags[f], fl);
}

}  // namespace mqr

using namespace mqr;

extern "C" {

int mqr_decode_depth(int device, const float* raw, int raw_loc, int N, int H, int W, const double* nears,
                     const double* fars, const uint8_t* strong, const double* conf, const int32_t* valid_count,
                     const uint8_t* has_mask, int mask_loc, double conf_thr, int count_thr, float* depth_out,
                     int out_loc, uint8_t* frame_ok) {
    MQR_REQUIRE(raw && nears && fars && depth_out && frame_ok, "null argument");
    MQR_REQUIRE(N >= 0 && H > 0 && W > 0, "bad frame shape");
    if (N == 0) return 0;
    const bool any_mask = has_mask && std::any_of(has_mask, has_mask + N, [](uint8_t m) { return m != 0; });
    MQR_REQUIRE(!any_mask || (conf && valid_count), "mask requested without confidence maps");
    MQR_CHECK_HIP(hipSetDevice(device));
    const int64_t HW = (int64_t)H * W, total = HW * N;
    std::vector<DecodeFrame> hf(N);
    for (int f = 0; f < N; ++f) {
        const double nr = nears[f], fa = fars[f];
        DecodeFrame& d = hf[f];
        if (std::isinf(fa) || fa < nr) {  // compute_ndc_to_linear_depth_params, depth_utils.py:21-28
            d.x = -2.0 * nr;
            d.y = -1.0;
            d.strong = strong ? (strong[f] & 1) : 0;  // y = -1.0 is always a Python float
        } else {
            d.x = -2.0 * fa * nr / (fa - nr);
            d.y = -(fa + nr) / (fa - nr);
            d.strong = strong ? ((strong[f] & 3) ? 3 : 0) : 0;
        }
        d.mask = any_mask && has_mask[f];
    }
    hipStream_t s = nullptr;
    MQR_CHECK_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    std::vector<void*> owned;
    auto dev_alloc = [&](size_t bytes) -> void* {
        void* p = nullptr;
        if (hipMalloc(&p, bytes) != hipSuccess) return nullptr;
        owned.push_back(p);
        return p;
    };
    int rc = 0;
    do {
        const float* d_raw = raw;
        if (raw_loc != MQR_DEVICE) {
            float* p = static_cast<float*>(dev_alloc(sizeof(float) * total));
            if (!p || hipMemcpyAsync(p, raw, sizeof(float) * total, hipMemcpyHostToDevice, s) != hipSuccess) {
                set_error("decode: raw upload failed");
                rc = 1;
                break;
            }
            d_raw = p;
        }
        const double* d_conf = conf;
        const int32_t* d_vc = valid_count;
        if (any_mask && mask_loc != MQR_DEVICE) {
            double* pc = static_cast<double*>(dev_alloc(sizeof(double) * total));
            int32_t* pv = static_cast<int32_t*>(dev_alloc(sizeof(int32_t) * total));
            if (!pc || !pv || hipMemcpyAsync(pc, conf, sizeof(double) * total, hipMemcpyHostToDevice, s) ||
                hipMemcpyAsync(pv, valid_count, sizeof(int32_t) * total, hipMemcpyHostToDevice, s)) {
                set_error("decode: confidence upload failed");
                rc = 1;
                break;
            }
            d_conf = pc;
            d_vc = pv;
        }
        float* d_out = out_loc == MQR_DEVICE ? depth_out : static_cast<float*>(dev_alloc(sizeof(float) * total));
        DecodeFrame* d_fr = static_cast<DecodeFrame*>(dev_alloc(sizeof(DecodeFrame) * N));
        uint32_t* d_flags = static_cast<uint32_t*>(dev_alloc(sizeof(uint32_t) * N));
        if (!d_out || !d_fr || !d_flags || hipMemcpyAsync(d_fr, hf.data(), sizeof(DecodeFrame) * N,
                                                          hipMemcpyHostToDevice, s) ||
            hipMemsetAsync(d_flags, 0, sizeof(uint32_t) * N, s)) {
            set_error("decode: device allocation failed");
            rc = 1;
            break;
        }
        const unsigned gx = (unsigned)std::min<int64_t>((HW + 255) / 256, 1024);
        hipLaunchKernelGGL(k_decode_depth, dim3(gx, (unsigned)N), dim3(256), 0, s, d_raw, HW, d_fr, d_conf, d_vc,
                           conf_thr, count_thr, d_out, d_flags);
        if (hipGetLastError() != hipSuccess) {
            set_error("decode: kernel launch failed");
            rc = 1;
            break;
        }
        std::vector<uint32_t> fl(N);
        if (hipMemcpyAsync(fl.data(), d_flags, sizeof(uint32_t) * N, hipMemcpyDeviceToHost, s) ||
            (out_loc != MQR_DEVICE &&
             hipMemcpyAsync(depth_out, d_out, sizeof(float) * total, hipMemcpyDeviceToHost, s)) ||
            hipStreamSynchronize(s)) {
            set_error("decode: copy back failed");
            rc = 1;
            break;
        }
        for (int f = 0; f < N; ++f)
            frame_ok[f] = (fl[f] & kAnyNonZero) && (fl[f] & kAnyNonOne) && !(fl[f] & (kAnyNaN | kAnyNotGE0));
    } while (false);
    (void)hipStreamSynchronize(s);
    for (void* p : owned) (void)hipFree(p);
    (void)hipStreamDestroy(s);
    return rc;
}

}  // extern "C"

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
#include <mutex>
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

// One pixel: NDC decode with the frame's numpy dtype rules, then the confidence mask.
template <bool MASK>
__device__ __forceinline__ float decode_px(float d, const DecodeFrame& fr, double c, int32_t vc, double conf_thr,
                                           int count_thr, uint32_t& fl) {
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
    if (MASK) {
        if (c < conf_thr) z = 0.0f;
        if (vc < count_thr) z = 0.0f;
    }
    return z;
}

// Workgroups stride over 4-pixel groups of one frame (blockIdx.y): 16-byte raw / count / depth
// accesses and two 16-byte confidence loads, so every wave moves whole 1 KiB (raw) or 2 KiB
// (confidence) runs.  VEC = false: scalar tail path for frames whose size is not a multiple of 4.
// BYTES: the mask comes as one byte per pixel (mqr_decode_depth_masked, e.g. from mqr_read_frames_masked)
// instead of the confidence / count maps.
template <bool VEC, bool BYTES = false>
__global__ __launch_bounds__(256) void k_decode_depth(const float* __restrict__ raw, int64_t HW,
                                                      const DecodeFrame* __restrict__ frames,
                                                      const double* __restrict__ conf,
                                                      const int32_t* __restrict__ vcount, double conf_thr,
                                                      int count_thr, float* __restrict__ out,
                                                      uint32_t* __restrict__ flags,
                                                      const uint8_t* __restrict__ mask8 = nullptr) {
    const int f = blockIdx.y;
    const DecodeFrame fr = frames[f];
    const int64_t base = (int64_t)f * HW;
    uint32_t fl = 0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    if (VEC) {
        const int64_t n4 = HW >> 2;
        const float4* r4 = reinterpret_cast<const float4*>(raw + base);
        float4* o4 = reinterpret_cast<float4*>(out + base);
        for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
            const float4 d = r4[i];
            float4 z;
            if (BYTES) {
                const uchar4 m = fr.mask ? reinterpret_cast<const uchar4*>(mask8 + base)[i] : make_uchar4(0, 0, 0, 0);
                // the decode runs for the validity flags even where the mask zeroes the depth
                z.x = decode_px<false>(d.x, fr, 0.0, 0, conf_thr, count_thr, fl);
                z.y = decode_px<false>(d.y, fr, 0.0, 0, conf_thr, count_thr, fl);
                z.z = decode_px<false>(d.z, fr, 0.0, 0, conf_thr, count_thr, fl);
                z.w = decode_px<false>(d.w, fr, 0.0, 0, conf_thr, count_thr, fl);
                if (m.x) z.x = 0.0f;
                if (m.y) z.y = 0.0f;
                if (m.z) z.z = 0.0f;
                if (m.w) z.w = 0.0f;
            } else if (fr.mask) {
                const double2* c2 = reinterpret_cast<const double2*>(conf + base) + 2 * i;
                const double2 ca = c2[0], cb = c2[1];
                const int4 v = reinterpret_cast<const int4*>(vcount + base)[i];
                z.x = decode_px<true>(d.x, fr, ca.x, v.x, conf_thr, count_thr, fl);
                z.y = decode_px<true>(d.y, fr, ca.y, v.y, conf_thr, count_thr, fl);
                z.z = decode_px<true>(d.z, fr, cb.x, v.z, conf_thr, count_thr, fl);
                z.w = decode_px<true>(d.w, fr, cb.y, v.w, conf_thr, count_thr, fl);
            } else {
                z.x = decode_px<false>(d.x, fr, 0.0, 0, conf_thr, count_thr, fl);
                z.y = decode_px<false>(d.y, fr, 0.0, 0, conf_thr, count_thr, fl);
                z.z = decode_px<false>(d.z, fr, 0.0, 0, conf_thr, count_thr, fl);
                z.w = decode_px<false>(d.w, fr, 0.0, 0, conf_thr, count_thr, fl);
            }
            o4[i] = z;
        }
    } else {
        for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < HW; i += stride) {
            const float d = raw[base + i];
            if (BYTES) {
                const float z = decode_px<false>(d, fr, 0.0, 0, conf_thr, count_thr, fl);
                out[base + i] = fr.mask && mask8[base + i] ? 0.0f : z;
            } else {
                out[base + i] = fr.mask ? decode_px<true>(d, fr, conf[base + i], vcount[base + i], conf_thr, count_thr, fl)
                                        : decode_px<false>(d, fr, 0.0, 0, conf_thr, count_thr, fl);
            }
        }
    }
    // workgroup-level OR (wave shuffle, then LDS), then ONE device atomic per workgroup.  A device
    // atomic (or atomic load) per wave on the frame's word serialises at that word's memory
    // channel: with a workgroup per 1024 pixels it capped the whole kernel at ~0.4 TB/s.
    __shared__ uint32_t wg_fl;
    if (threadIdx.x == 0) wg_fl = 0;
    for (int o = 32; o > 0; o >>= 1) fl |= (uint32_t)__shfl_xor((int)fl, o, 64);
    __syncthreads();
    if ((threadIdx.x & 63) == 0 && fl) atomicOr(&wg_fl, fl);
    __syncthreads();
    if (threadIdx.x == 0 && wg_fl) atomicOr(&flags[f], wg_fl);
}

// Per-device decode context, created on first use and kept: a stream, a grow-only scratch buffer
// (staged host inputs / output), the per-frame parameter and flag arrays and their pinned
// mirrors.  Creating a stream and mapping fresh device pages cost milliseconds per call; the
// kernel itself streams 20 B per pixel.  Calls on one device serialise on the context's mutex.
struct DecodeCtx {
    std::mutex mu;
    hipStream_t s = nullptr;
    char* scratch = nullptr;
    size_t scratch_cap = 0;
    DecodeFrame* d_fr = nullptr;
    uint32_t* d_flags = nullptr;
    DecodeFrame* h_fr = nullptr;
    uint32_t* h_flags = nullptr;
    int frame_cap = 0;
};
static DecodeCtx g_decode[64];

static int decode_ctx_reserve(DecodeCtx& c, size_t scratch_bytes, int frames) {
    if (!c.s) MQR_CHECK_HIP(hipStreamCreateWithFlags(&c.s, hipStreamNonBlocking));
    if (scratch_bytes > c.scratch_cap) {
        MQR_CHECK_HIP(hipStreamSynchronize(c.s));
        if (c.scratch) MQR_CHECK_HIP(hipFree(c.scratch));
        c.scratch = nullptr;
        c.scratch_cap = 0;
        MQR_CHECK_HIP(hipMalloc(&c.scratch, scratch_bytes));
        c.scratch_cap = scratch_bytes;
    }
    if (frames > c.frame_cap) {
        MQR_CHECK_HIP(hipStreamSynchronize(c.s));
        const int cap = std::max(frames, 256);
        if (c.d_fr) MQR_CHECK_HIP(hipFree(c.d_fr));
        if (c.d_flags) MQR_CHECK_HIP(hipFree(c.d_flags));
        if (c.h_fr) MQR_CHECK_HIP(hipHostFree(c.h_fr));
        if (c.h_flags) MQR_CHECK_HIP(hipHostFree(c.h_flags));
        c.d_fr = nullptr;
        c.d_flags = nullptr;
        c.h_fr = nullptr;
        c.h_flags = nullptr;
        c.frame_cap = 0;
        MQR_CHECK_HIP(hipMalloc(&c.d_fr, sizeof(DecodeFrame) * cap));
        MQR_CHECK_HIP(hipMalloc(&c.d_flags, sizeof(uint32_t) * cap));
        MQR_CHECK_HIP(hipHostMalloc(&c.h_fr, sizeof(DecodeFrame) * cap, hipHostMallocDefault));
        MQR_CHECK_HIP(hipHostMalloc(&c.h_flags, sizeof(uint32_t) * cap, hipHostMallocDefault));
        c.frame_cap = cap;
    }
    return 0;
}

static size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

}  // namespace mqr

using namespace mqr;

// The decode with the mask as confidence / count maps (mask8 null) or as one byte per pixel (mask8).
static int decode_impl(int device, const float* raw, int raw_loc, int N, int H, int W, const double* nears,
                       const double* fars, const uint8_t* strong, const double* conf, const int32_t* valid_count,
                       const uint8_t* mask8, const uint8_t* has_mask, int mask_loc, double conf_thr, int count_thr,
                       float* depth_out, int out_loc, uint8_t* frame_ok) {
    MQR_REQUIRE(raw && nears && fars && depth_out && frame_ok, "null argument");
    MQR_REQUIRE(N >= 0 && H > 0 && W > 0, "bad frame shape");
    MQR_REQUIRE(device >= 0 && device < 64, "device index out of range");
    if (N == 0) return 0;
    const bool any_mask = has_mask && std::any_of(has_mask, has_mask + N, [](uint8_t m) { return m != 0; });
    MQR_REQUIRE(!any_mask || mask8 || (conf && valid_count), "mask requested without confidence maps");
    MQR_CHECK_HIP(hipSetDevice(device));
    const int64_t HW = (int64_t)H * W, total = HW * N;
    DecodeCtx& c = g_decode[device];
    std::lock_guard<std::mutex> lock(c.mu);
    // scratch layout: [raw f32][conf f64][count i32] or [mask u8] [out f32], only the parts that are staged
    const bool stage_raw = raw_loc != MQR_DEVICE, stage_mask = any_mask && mask_loc != MQR_DEVICE,
               stage_out = out_loc != MQR_DEVICE;
    const size_t b_raw = stage_raw ? align256(sizeof(float) * total) : 0;
    const size_t b_conf = stage_mask && !mask8 ? align256(sizeof(double) * total) : 0;
    const size_t b_vc = stage_mask ? align256((mask8 ? 1 : sizeof(int32_t)) * total) : 0;
    const size_t b_out = stage_out ? align256(sizeof(float) * total) : 0;
    if (decode_ctx_reserve(c, std::max<size_t>(b_raw + b_conf + b_vc + b_out, 256), N)) return 1;
    if ((!stage_raw || (any_mask && !stage_mask) || !stage_out) && order_after_caller(device, c.s)) return 2;
    for (int f = 0; f < N; ++f) {
        const double nr = nears[f], fa = fars[f];
        DecodeFrame& d = c.h_fr[f];
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
    char* sp = c.scratch;
    const float* d_raw = raw;
    if (stage_raw) {
        if (copy_to_device(device, sp, raw, sizeof(float) * total, c.s)) return 1;
        d_raw = reinterpret_cast<const float*>(sp);
        sp += b_raw;
    }
    const double* d_conf = conf;
    const int32_t* d_vc = valid_count;
    const uint8_t* d_m8 = mask8;
    if (stage_mask && mask8) {
        if (copy_to_device(device, sp, mask8, total, c.s)) return 1;
        d_m8 = reinterpret_cast<const uint8_t*>(sp);
        sp += b_vc;
    } else if (stage_mask) {
        if (copy_to_device(device, sp, conf, sizeof(double) * total, c.s)) return 1;
        d_conf = reinterpret_cast<const double*>(sp);
        sp += b_conf;
        if (copy_to_device(device, sp, valid_count, sizeof(int32_t) * total, c.s)) return 1;
        d_vc = reinterpret_cast<const int32_t*>(sp);
        sp += b_vc;
    }
    float* d_out = stage_out ? reinterpret_cast<float*>(sp) : depth_out;
    MQR_CHECK_HIP(hipMemcpyAsync(c.d_fr, c.h_fr, sizeof(DecodeFrame) * N, hipMemcpyHostToDevice, c.s));
    MQR_CHECK_HIP(hipMemsetAsync(c.d_flags, 0, sizeof(uint32_t) * N, c.s));
    auto aligned = [](const void* p, size_t a) { return (reinterpret_cast<uintptr_t>(p) & (a - 1)) == 0; };
    const bool vec = HW % 4 == 0 && aligned(d_raw, 16) && aligned(d_out, 16) &&
                     (!any_mask || (mask8 ? aligned(d_m8, 4) : (aligned(d_conf, 32) && aligned(d_vc, 16))));
    const int64_t work = vec ? HW / 4 : HW;
    // ~4096 workgroups in all (16 per CU), each a long grid-stride run over its frame: enough
    // to fill the chip with few enough workgroups that the per-frame flag atomics stay rare
    const int64_t per_frame = std::max<int64_t>(1, (4096 + N - 1) / N);
    const unsigned gx = (unsigned)std::min<int64_t>((work + 255) / 256, per_frame);
    const dim3 grid(gx, (unsigned)N);
    if (mask8 && vec)
        hipLaunchKernelGGL((k_decode_depth<true, true>), grid, dim3(256), 0, c.s, d_raw, HW, c.d_fr, nullptr, nullptr,
                           conf_thr, count_thr, d_out, c.d_flags, d_m8);
    else if (mask8)
        hipLaunchKernelGGL((k_decode_depth<false, true>), grid, dim3(256), 0, c.s, d_raw, HW, c.d_fr, nullptr, nullptr,
                           conf_thr, count_thr, d_out, c.d_flags, d_m8);
    else if (vec)
        hipLaunchKernelGGL((k_decode_depth<true, false>), grid, dim3(256), 0, c.s, d_raw, HW, c.d_fr, d_conf, d_vc,
                           conf_thr, count_thr, d_out, c.d_flags, nullptr);
    else
        hipLaunchKernelGGL((k_decode_depth<false, false>), grid, dim3(256), 0, c.s, d_raw, HW, c.d_fr, d_conf, d_vc,
                           conf_thr, count_thr, d_out, c.d_flags, nullptr);
    MQR_CHECK_HIP(hipGetLastError());
    MQR_CHECK_HIP(hipMemcpyAsync(c.h_flags, c.d_flags, sizeof(uint32_t) * N, hipMemcpyDeviceToHost, c.s));
    if (stage_out && copy_to_host(device, depth_out, d_out, sizeof(float) * total, c.s)) return 1;
    MQR_CHECK_HIP(hipStreamSynchronize(c.s));
    for (int f = 0; f < N; ++f) {
        const uint32_t fl = c.h_flags[f];
        frame_ok[f] = (fl & kAnyNonZero) && (fl & kAnyNonOne) && !(fl & (kAnyNaN | kAnyNotGE0));
    }
    return 0;
}

extern "C" {

int mqr_decode_depth(int device, const float* raw, int raw_loc, int N, int H, int W, const double* nears,
                     const double* fars, const uint8_t* strong, const double* conf, const int32_t* valid_count,
                     const uint8_t* has_mask, int mask_loc, double conf_thr, int count_thr, float* depth_out,
                     int out_loc, uint8_t* frame_ok) {
    return decode_impl(device, raw, raw_loc, N, H, W, nears, fars, strong, conf, valid_count, nullptr, has_mask,
                       mask_loc, conf_thr, count_thr, depth_out, out_loc, frame_ok);
}

int mqr_decode_depth_masked(int device, const float* raw, int raw_loc, int N, int H, int W, const double* nears,
                            const double* fars, const uint8_t* strong, const uint8_t* mask, const uint8_t* has_mask,
                            int mask_loc, float* depth_out, int out_loc, uint8_t* frame_ok) {
    const bool any_mask = has_mask && N > 0 && std::any_of(has_mask, has_mask + N, [](uint8_t m) { return m != 0; });
    MQR_REQUIRE(!any_mask || mask, "mask requested without a mask array");
    static const uint8_t kNone = 0;  // (a non-null placeholder selecting the byte-mask kernel: never read, no frame masked)
    return decode_impl(device, raw, raw_loc, N, H, W, nears, fars, strong, nullptr, nullptr, any_mask ? mask : &kNone,
                       any_mask ? has_mask : nullptr, mask_loc, 0.0, 0, depth_out, out_loc, frame_ok);
}

}  // extern "C"

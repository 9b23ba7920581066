// confidence.hip -- multi-view depth confidence (reference: scripts/processing/reconstruction/
// confidence_estimation/estimate_depth_confidences.py:15-79 build_confidence_map and
// compute_pixel_error_map.py:4-220).
//
// One thread per reference pixel, the +-r neighbour loop in registers, every frame of the
// sequence resident in HBM (the reference re-reads and re-decodes each frame ~21x from disk).
// Arithmetic is float64 in numpy's order with the two float32 roundings numpy performs
// (interpolated target depth, error), so valid_count / confidence match the reference exactly
// (pinned by tests/golden/confidence_golden.npz).  FP64 VALU + L2-resident gathers: bounded by
// the neighbour-frame gathers, not by HBM streaming.
#include <algorithm>
#include <cmath>
#include <vector>

#include "mqr_common.hpp"

namespace mqr {

struct ConfFrame {
    float K[9];
    float Tcw[16];
    float Tinv[16];
};

// Returns 1 and the float32 error when (ref pixel -> target frame) yields a finite error.
__device__ inline int pixel_error(const float* __restrict__ tgt, int H, int W, const ConfFrame& ft,
                                  const double pw[3], double depth_max, float* err) {
    const float dmf = (float)depth_max;
    double pt[3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
        pt[i] = (double)ft.Tinv[i * 4 + 0] * pw[0] + (double)ft.Tinv[i * 4 + 1] * pw[1] +
                (double)ft.Tinv[i * 4 + 2] * pw[2] + (double)ft.Tinv[i * 4 + 3] * 1.0;
    const double X = pt[0], Y = pt[1], Z = pt[2];
    if (!(Z > 0 && isfinite(Z) && Z <= depth_max && isfinite(X) && isfinite(Y))) return 0;
    const double fx = (double)ft.K[0], fy = (double)ft.K[4], cx = (double)ft.K[2], cy = (double)ft.K[5];
    const double uu = ((X * fx) / Z) + cx;
    const double vv = ((Y * fy) / Z) + cy;
    if (!(isfinite(uu) && isfinite(vv))) return 0;
    const double max_coord = (double)((W > H ? W : H) * 10);
    if (!(uu >= -max_coord && uu < max_coord && vv >= -max_coord && vv < max_coord)) return 0;
    const int u0 = (int)floor(uu), v0 = (int)floor(vv), u1 = u0 + 1, v1 = v0 + 1;
    if (!(u0 >= 0 && u1 < W && v0 >= 0 && v1 < H)) return 0;
    // the two taps of a row in one 8-byte load (4-byte aligned; the L1 path costs per lane, not per byte)
    float2 ab, cd;
    __builtin_memcpy(&ab, tgt + (int64_t)v0 * W + u0, sizeof(float2));
    __builtin_memcpy(&cd, tgt + (int64_t)v1 * W + u0, sizeof(float2));
    const float Ia = ab.x, Ib = ab.y, Ic = cd.x, Id = cd.y;
    if (!(Ib > 0 && Ib <= dmf && Ia > 0 && Ia <= dmf && Ic > 0 && Ic <= dmf && Id > 0 && Id <= dmf)) return 0;
    const double wa = ((double)u1 - uu) * ((double)v1 - vv);
    const double wb = (uu - (double)u0) * ((double)v1 - vv);
    const double wc = ((double)u1 - uu) * (vv - (double)v0);
    const double wd = (uu - (double)u0) * (vv - (double)v0);
    const float zt = (float)(wa * Ia + wb * Ib + wc * Ic + wd * Id);
    if (!(zt > 0 && isfinite(zt))) return 0;
    const double ztd = (double)zt;
    const double xt = ((uu - cx) * ztd) / fx;
    const double yt = ((vv - cy) * ztd) / fy;
    double q[3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
        q[i] = (double)ft.Tcw[i * 4 + 0] * xt + (double)ft.Tcw[i * 4 + 1] * yt + (double)ft.Tcw[i * 4 + 2] * ztd +
               (double)ft.Tcw[i * 4 + 3] * 1.0;
    const double dx = pw[0] - q[0], dy = pw[1] - q[1], dz = pw[2] - q[2];
    *err = (float)sqrt(dx * dx + dy * dy + dz * dz);
    return 1;
}

// depth_to_pointcloud_numpy for one pixel: returns 0 when the ref pixel is not in (0, depth_max].
__device__ inline int ref_point(const ConfFrame& fr, int u, int v, float dref, double depth_max, double pw[3]) {
    if (!(dref > 0 && dref <= (float)depth_max)) return 0;
    const double z = (double)dref;
    const double x = (((double)u - (double)fr.K[2]) * z) / (double)fr.K[0];
    const double y = (((double)v - (double)fr.K[5]) * z) / (double)fr.K[4];
#pragma unroll
    for (int i = 0; i < 3; ++i)
        pw[i] = (double)fr.Tcw[i * 4 + 0] * x + (double)fr.Tcw[i * 4 + 1] * y + (double)fr.Tcw[i * 4 + 2] * z +
                (double)fr.Tcw[i * 4 + 3] * 1.0;
    return 1;
}

__global__ __launch_bounds__(256) void k_confidence(const float* __restrict__ depths, int N, int H, int W,
                                                    const ConfFrame* __restrict__ fr, const uint8_t* __restrict__ ok,
                                                    int ref_begin, int r, double depth_max, float thr,
                                                    double* __restrict__ conf, int32_t* __restrict__ valid) {
    const int64_t HW = (int64_t)H * W;
    const int ref = ref_begin + blockIdx.y;
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= HW) return;
    const int u = (int)(p % W), v = (int)(p / W);
    double pw[3];
    int nv = 0, nc = 0;
    if (ref_point(fr[ref], u, v, depths[(int64_t)ref * HW + p], depth_max, pw)) {
        const int lo = max(0, ref - r), hi = min(N, ref + r + 1);
        for (int t = lo; t < hi; ++t) {
            if (t == ref || !ok[t]) continue;
            float e;
            if (pixel_error(depths + (int64_t)t * HW, H, W, fr[t], pw, depth_max, &e)) {
                ++nv;
                if (e <= thr) ++nc;
            }
        }
    }
    const int64_t o = (int64_t)blockIdx.y * HW + p;
    valid[o] = nv;
    conf[o] = nv == 0 ? 0.0 : (double)nc / (double)nv;
}

__global__ void k_error_map(const float* __restrict__ refd, const float* __restrict__ tgtd, int H, int W,
                            const ConfFrame* __restrict__ fr, double depth_max, float* out) {
    const int64_t HW = (int64_t)H * W;
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= HW) return;
    double pw[3];
    float e = NAN;
    float ev;
    if (ref_point(fr[0], (int)(p % W), (int)(p / W), refd[p], depth_max, pw) &&
        pixel_error(tgtd, H, W, fr[1], pw, depth_max, &ev))
        e = ev;
    out[p] = e;
}

}  // namespace mqr

using namespace mqr;

extern "C" {

int mqr_confidence(int device, const float* depths, int depth_loc, int N, int H, int W, const float* K,
                   const float* T_cw, const float* T_cw_inv, const uint8_t* frame_ok, int ref_begin, int ref_end,
                   int frame_range, double depth_max, double error_threshold, double* conf, int32_t* valid,
                   int out_loc) {
    MQR_REQUIRE(depths && K && T_cw && T_cw_inv && conf && valid, "null argument");
    MQR_REQUIRE(N > 0 && H > 0 && W > 0, "bad shape");
    MQR_REQUIRE(ref_begin >= 0 && ref_end <= N && ref_begin <= ref_end, "bad reference frame range");
    MQR_CHECK_HIP(hipSetDevice(device));
    const int nref = ref_end - ref_begin;
    if (nref == 0) return 0;
    const int64_t HW = (int64_t)H * W;
    hipStream_t s;
    MQR_CHECK_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    std::vector<ConfFrame> fr(N);
    std::vector<uint8_t> okv(N, 1);
    for (int i = 0; i < N; ++i) {
        std::copy(K + 9 * i, K + 9 * i + 9, fr[i].K);
        std::copy(T_cw + 16 * i, T_cw + 16 * i + 16, fr[i].Tcw);
        std::copy(T_cw_inv + 16 * i, T_cw_inv + 16 * i + 16, fr[i].Tinv);
        if (frame_ok) okv[i] = frame_ok[i] ? 1 : 0;
    }
    ConfFrame* dfr = nullptr;
    uint8_t* dok = nullptr;
    float* dd = nullptr;
    double* dconf = conf;
    int32_t* dvalid = valid;
    MQR_CHECK_HIP(hipMalloc(&dfr, sizeof(ConfFrame) * N));
    MQR_CHECK_HIP(hipMalloc(&dok, N));
    MQR_CHECK_HIP(hipMemcpy(dfr, fr.data(), sizeof(ConfFrame) * N, hipMemcpyHostToDevice));
    MQR_CHECK_HIP(hipMemcpy(dok, okv.data(), N, hipMemcpyHostToDevice));
    const float* dsrc = depths;
    if (depth_loc != MQR_DEVICE) {
        MQR_CHECK_HIP(hipMalloc(&dd, sizeof(float) * N * HW));
        MQR_CHECK_HIP(hipMemcpy(dd, depths, sizeof(float) * N * HW, hipMemcpyHostToDevice));
        dsrc = dd;
    }
    if (out_loc != MQR_DEVICE) {
        MQR_CHECK_HIP(hipMalloc(&dconf, sizeof(double) * nref * HW));
        MQR_CHECK_HIP(hipMalloc(&dvalid, sizeof(int32_t) * nref * HW));
    }
    // (float) threshold: numpy compares the float32 error map against a weak Python float.
    hipLaunchKernelGGL(k_confidence, dim3((unsigned)((HW + 255) / 256), nref), dim3(256), 0, s, dsrc, N, H, W, dfr,
                       dok, ref_begin, frame_range, depth_max, (float)error_threshold, dconf, dvalid);
    MQR_CHECK_HIP(hipGetLastError());
    if (out_loc != MQR_DEVICE) {
        MQR_CHECK_HIP(hipMemcpyAsync(conf, dconf, sizeof(double) * nref * HW, hipMemcpyDeviceToHost, s));
        MQR_CHECK_HIP(hipMemcpyAsync(valid, dvalid, sizeof(int32_t) * nref * HW, hipMemcpyDeviceToHost, s));
    }
    MQR_CHECK_HIP(hipStreamSynchronize(s));
    if (out_loc != MQR_DEVICE) {
        (void)hipFree(dconf);
        (void)hipFree(dvalid);
    }
    if (dd) (void)hipFree(dd);
    (void)hipFree(dfr);
    (void)hipFree(dok);
    (void)hipStreamDestroy(s);
    return 0;
}

int mqr_pixel_error_map(int device, const float* ref_depth, const float* tgt_depth, int H, int W, const float* K_ref,
                        const float* K_tgt, const float* T_cw_ref, const float* T_cw_inv_tgt, const float* T_cw_tgt,
                        double depth_max, float* err_out) {
    MQR_REQUIRE(ref_depth && tgt_depth && K_ref && K_tgt && T_cw_ref && T_cw_inv_tgt && T_cw_tgt && err_out,
                "null argument");
    MQR_CHECK_HIP(hipSetDevice(device));
    const int64_t HW = (int64_t)H * W;
    ConfFrame fr[2] = {};
    std::copy(K_ref, K_ref + 9, fr[0].K);
    std::copy(T_cw_ref, T_cw_ref + 16, fr[0].Tcw);
    std::copy(K_tgt, K_tgt + 9, fr[1].K);
    std::copy(T_cw_tgt, T_cw_tgt + 16, fr[1].Tcw);
    std::copy(T_cw_inv_tgt, T_cw_inv_tgt + 16, fr[1].Tinv);
    ConfFrame* dfr = nullptr;
    float *dr = nullptr, *dt = nullptr, *de = nullptr;
    MQR_CHECK_HIP(hipMalloc(&dfr, sizeof(fr)));
    MQR_CHECK_HIP(hipMalloc(&dr, sizeof(float) * HW));
    MQR_CHECK_HIP(hipMalloc(&dt, sizeof(float) * HW));
    MQR_CHECK_HIP(hipMalloc(&de, sizeof(float) * HW));
    MQR_CHECK_HIP(hipMemcpy(dfr, fr, sizeof(fr), hipMemcpyHostToDevice));
    MQR_CHECK_HIP(hipMemcpy(dr, ref_depth, sizeof(float) * HW, hipMemcpyHostToDevice));
    MQR_CHECK_HIP(hipMemcpy(dt, tgt_depth, sizeof(float) * HW, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_error_map, dim3((unsigned)((HW + 255) / 256)), dim3(256), 0, 0, dr, dt, H, W, dfr, depth_max,
                       de);
    MQR_CHECK_HIP(hipGetLastError());
    MQR_CHECK_HIP(hipMemcpy(err_out, de, sizeof(float) * HW, hipMemcpyDeviceToHost));
    (void)hipFree(dfr);
    (void)hipFree(dr);
    (void)hipFree(dt);
    (void)hipFree(de);
    return 0;
}

}  // extern "C"

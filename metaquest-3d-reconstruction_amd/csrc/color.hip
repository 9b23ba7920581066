// color.hip -- per-vertex colour projection from keyframes.
//
// The reference colours its mesh with Open3D's colour-map pipeline: the extracted mesh, the colour
// keyframes and their colour-aligned depth (ray-cast from the mesh, raycast_in_color_view,
// o3d_utils.py:324-341) go to run_rigid_optimizer (optimize_color_pose.py:24-73).  Its colour
// assignment -- the part that is bandwidth work and runs on every iteration -- is the visibility
// test plus per-vertex averaging of upstream ColorMapUtils.cpp (CreateVertexAndImageVisibility,
// SetGeometryColorAverage; recalled, not vendored here -- VERIFY):
//   Vt = T_c [X 1] (float64), u = float(Vt.x fx / Vt.z + cx), v = float(Vt.y fy / Vt.z + cy),
//   d = float(Vt.z); ui = int(round(u)), vi = int(round(v));
//   visible in keyframe c iff d >= 0, (ui, vi) inside the image, depth_c(ui, vi) <= max_depth and
//   |d - depth_c(ui, vi)| < visibility_threshold (float difference, compared in float64);
//   sampled iff also margin <= u < W - margin and margin <= v < H - margin: the colour is the
//   average over the sampled keyframes of (float)image_c(ui, vi) / 255.0f, summed in float64 in
//   keyframe order.
// Not restated: the depth-discontinuity mask and the k-nearest-neighbour fill of vertices no
// keyframe sees (their colour stays 0, count 0), and the pose optimisation itself (OUT of scope).
//
// One thread per vertex, keyframe loop in registers; the keyframe parameters sit in constant-
// cached global memory.  Colour images are RGB uint8 [N][H][W][3], depth float32 [N][H][W].
#include <cmath>
#include <mutex>
#include <vector>

#include "mqr_common.hpp"

namespace mqr {

struct ColorCam {
    double E[12];  // world -> camera, rows 0..2 of T_wc
    double fx, fy, cx, cy;
};

__global__ __launch_bounds__(256) void k_color_vertices(const float* __restrict__ V, int64_t nv,
                                                        const uint8_t* __restrict__ images,
                                                        const float* __restrict__ depths,
                                                        const ColorCam* __restrict__ cams, int N, int H, int W,
                                                        double max_depth, double vis_thr, int margin,
                                                        float* __restrict__ out, int32_t* __restrict__ counts) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nv) return;
    const double X = V[3 * i], Y = V[3 * i + 1], Z = V[3 * i + 2];
    double sr = 0.0, sg = 0.0, sb = 0.0;
    int cnt = 0;
    const int64_t HW = (int64_t)H * W;
    for (int c = 0; c < N; ++c) {
        const ColorCam& cm = cams[c];
        const double vx = cm.E[0] * X + cm.E[1] * Y + cm.E[2] * Z + cm.E[3];
        const double vy = cm.E[4] * X + cm.E[5] * Y + cm.E[6] * Z + cm.E[7];
        const double vz = cm.E[8] * X + cm.E[9] * Y + cm.E[10] * Z + cm.E[11];
        const float u = (float)((vx * cm.fx) / vz + cm.cx);
        const float v = (float)((vy * cm.fy) / vz + cm.cy);
        const float d = (float)vz;
        const int ui = (int)roundf(u), vi = (int)roundf(v);
        if (d < 0.0f || ui < 0 || ui >= W || vi < 0 || vi >= H) continue;
        const int64_t px = (int64_t)c * HW + (int64_t)vi * W + ui;
        const float ds = depths[px];
        if (ds > max_depth) continue;
        if (!((double)fabsf(d - ds) < vis_thr)) continue;
        if (!(u >= margin && u < W - margin && v >= margin && v < H - margin)) continue;
        const uint8_t* p = images + 3 * px;
        // upstream: float r = (float)r_temp / 255.0f, summed into a double vector
        sr += (double)((float)p[0] / 255.0f);
        sg += (double)((float)p[1] / 255.0f);
        sb += (double)((float)p[2] / 255.0f);
        ++cnt;
    }
    out[3 * i] = cnt ? (float)(sr / cnt) : 0.f;
    out[3 * i + 1] = cnt ? (float)(sg / cnt) : 0.f;
    out[3 * i + 2] = cnt ? (float)(sb / cnt) : 0.f;
    if (counts) counts[i] = cnt;
}

}  // namespace mqr

using namespace mqr;

extern "C" {

int mqr_color_vertices(int device, const float* vertices, int64_t nv, int vloc, const uint8_t* images,
                       const float* depths, int img_loc, int N, int H, int W, const double* K, const double* T_wc,
                       double max_depth, double visibility_threshold, int margin, float* colors_out,
                       int32_t* counts_out, int out_loc) {
    MQR_REQUIRE(vertices && images && depths && K && T_wc && colors_out, "null argument");
    MQR_REQUIRE(nv >= 0 && N >= 0 && H > 0 && W > 0, "bad sizes");
    if (nv == 0) return 0;
    MQR_CHECK_HIP(hipSetDevice(device));
    std::vector<ColorCam> cams(N);
    for (int c = 0; c < N; ++c) {
        for (int k = 0; k < 12; ++k) cams[c].E[k] = T_wc[16 * c + k];
        cams[c].fx = K[9 * c + 0];
        cams[c].fy = K[9 * c + 4];
        cams[c].cx = K[9 * c + 2];
        cams[c].cy = K[9 * c + 5];
    }
    hipStream_t s = nullptr;
    MQR_CHECK_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    std::vector<void*> owned;
    int rc = 0;
    auto dev = [&](const void* h, size_t bytes, bool host) -> const void* {
        if (!host) return h;
        void* p = nullptr;
        if (hipMalloc(&p, bytes) != hipSuccess) return nullptr;
        owned.push_back(p);
        if (hipMemcpyAsync(p, h, bytes, hipMemcpyHostToDevice, s) != hipSuccess) return nullptr;
        return p;
    };
    const int64_t HW = (int64_t)H * W;
    const float* dV = static_cast<const float*>(dev(vertices, sizeof(float) * 3 * nv, vloc != MQR_DEVICE));
    const uint8_t* dI = static_cast<const uint8_t*>(dev(images, (size_t)3 * HW * N, img_loc != MQR_DEVICE));
    const float* dD = static_cast<const float*>(dev(depths, sizeof(float) * HW * N, img_loc != MQR_DEVICE));
    const ColorCam* dC = static_cast<const ColorCam*>(dev(cams.data(), sizeof(ColorCam) * std::max(N, 1), true));
    float* dO = colors_out;
    int32_t* dN = counts_out;
    if (out_loc != MQR_DEVICE) {
        void* p = nullptr;
        if (hipMalloc(&p, (sizeof(float) * 3 + sizeof(int32_t)) * nv) == hipSuccess) owned.push_back(p);
        dO = static_cast<float*>(p);
        dN = p ? reinterpret_cast<int32_t*>(static_cast<float*>(p) + 3 * nv) : nullptr;
    }
    if (!dV || !dI || !dD || !dC || !dO) {
        set_error("mqr_color_vertices: device allocation or upload failed");
        rc = 1;
    } else {
        hipLaunchKernelGGL(k_color_vertices, dim3((unsigned)((nv + 255) / 256)), dim3(256), 0, s, dV, nv, dI, dD,
                           dC, N, H, W, max_depth, visibility_threshold, margin, dO, dN);
        if (hipGetLastError() != hipSuccess) {
            set_error("mqr_color_vertices: kernel launch failed");
            rc = 1;
        }
        if (!rc && out_loc != MQR_DEVICE &&
            (hipMemcpyAsync(colors_out, dO, sizeof(float) * 3 * nv, hipMemcpyDeviceToHost, s) != hipSuccess ||
             (counts_out && hipMemcpyAsync(counts_out, dN, sizeof(int32_t) * nv, hipMemcpyDeviceToHost, s) !=
                                hipSuccess))) {
            set_error("mqr_color_vertices: copy back failed");
            rc = 1;
        }
    }
    if (hipStreamSynchronize(s) != hipSuccess && !rc) {
        set_error("mqr_color_vertices: kernel failed");
        rc = 1;
    }
    for (void* p : owned) (void)hipFree(p);
    (void)hipStreamDestroy(s);
    return rc;
}

}  // extern "C"

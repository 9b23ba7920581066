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
// mqr_color_vertices is that visibility-and-average primitive; mqr_color_map (below) is the complete
// assignment -- RGBD depth truncation, depth-discontinuity masks, float64 averages and the
// k-nearest-neighbour fill of vertices no keyframe sees.  The pose optimisation stays OUT of scope.
//
// One thread per vertex, keyframe loop in registers; the keyframe parameters sit in constant-
// cached global memory.  Colour images are RGB uint8 [N][H][W][3], depth float32 [N][H][W].
#include <hipcub/hipcub.hpp>

#include <cmath>
#include <mutex>
#include <memory>
#include <vector>

#include "mqr_common.hpp"
#include "device_block.hpp"

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

// ================================================================== complete colour map (mqr_color_map)
// run_rigid_optimizer's vertex colours with the keyframe poses as given (the pose refinement stays
// OUT of scope; = maximum_iteration 0), upstream ColorMapUtils / Image.cpp as recalled -- VERIFY:
//   RGBD depth d = t_hit / 1.0, d >= depth_trunc (3.0, create_from_color_and_depth's default) -> 0;
//   depth-boundary mask: Sobel dx = (Sobel31 along x, then Sobel32 along y), dy = (Sobel32, Sobel31),
//     every pass a float32 image of double sums of float products over the clamped 3-tap window;
//     sqrt(dx^2 + dy^2) > 0.1 -> 255, dilated over the (2 half + 1)^2 window (half = 3);
//   visibility as k_color_vertices plus mask != 255; float64 averages; vertices no keyframe samples
//   take the float64 mean of their knn (3) nearest sampled vertices' colours (squared-distance ties
//   broken by the lower vertex index).

// horizontal pass of both filters from the truncated depth: hx = Sobel31 along x, hy = Sobel32 along x
__global__ void k_cm_filter_h(const float* __restrict__ t_hit, int64_t total, int H, int W, float depth_trunc,
                              float* __restrict__ hx, float* __restrict__ hy) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    const int x = (int)(i % W);
    const int64_t row = i - x;
    float d[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const int xs = min(max(x + k - 1, 0), W - 1);
        const float v = t_hit[row + xs] / 1.0f;
        d[k] = v >= depth_trunc ? 0.0f : v;
    }
    double a = 0, b = 0;
    a += (double)(d[0] * -1.0f);
    a += (double)(d[1] * 0.0f);
    a += (double)(d[2] * 1.0f);
    b += (double)(d[0] * 1.0f);
    b += (double)(d[1] * 2.0f);
    b += (double)(d[2] * 1.0f);
    hx[i] = (float)a;
    hy[i] = (float)b;
    (void)H;
}

// vertical passes (dx = Sobel32 along y of hx, dy = Sobel31 along y of hy) and the threshold
__global__ void k_cm_filter_v(const float* __restrict__ hx, const float* __restrict__ hy, int64_t total, int H, int W,
                              double disc_thr, uint8_t* __restrict__ m0) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    const int64_t HW = (int64_t)H * W;
    const int64_t f = i / HW;
    const int p = (int)(i - f * HW), y = p / W, x = p % W;
    double a = 0, b = 0;
    const float ka[3] = {1.0f, 2.0f, 1.0f}, kb[3] = {-1.0f, 0.0f, 1.0f};
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const int ys = min(max(y + k - 1, 0), H - 1);
        const int64_t q = f * HW + (int64_t)ys * W + x;
        a += (double)(hx[q] * ka[k]);
        b += (double)(hy[q] * kb[k]);
    }
    const double dx = (double)(float)a, dy = (double)(float)b;
    m0[i] = sqrt(dx * dx + dy * dy) > disc_thr ? 255 : 0;
}

__global__ void k_cm_dilate(const uint8_t* __restrict__ m0, int64_t total, int H, int W, int half,
                            uint8_t* __restrict__ mask) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    const int64_t HW = (int64_t)H * W;
    const int64_t f = i / HW;
    const int p = (int)(i - f * HW), y = p / W, x = p % W;
    uint8_t o = 0;
    for (int yy = max(y - half, 0); yy <= min(y + half, H - 1) && !o; ++yy)
        for (int xx = max(x - half, 0); xx <= min(x + half, W - 1); ++xx)
            if (m0[f * HW + (int64_t)yy * W + xx] == 255) {
                o = 255;
                break;
            }
    mask[i] = o;
}

__global__ __launch_bounds__(256) void k_cm_vertices(const float* __restrict__ V, int64_t nv,
                                                     const uint8_t* __restrict__ images,
                                                     const float* __restrict__ t_hit, const uint8_t* __restrict__ mask,
                                                     const ColorCam* __restrict__ cams, int N, int H, int W,
                                                     double max_depth, double vis_thr, int margin, float depth_trunc,
                                                     double* __restrict__ avg, int32_t* __restrict__ counts) {
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
        const float th = t_hit[px] / 1.0f;
        const float ds = th >= depth_trunc ? 0.0f : th;
        if (ds > max_depth) continue;
        if (mask[px] == 255) continue;
        if (!((double)fabsf(d - ds) < vis_thr)) continue;
        if (!(u >= margin && u < W - margin && v >= margin && v < H - margin)) continue;
        const uint8_t* p = images + 3 * px;
        sr += (double)((float)p[0] / 255.0f);
        sg += (double)((float)p[1] / 255.0f);
        sb += (double)((float)p[2] / 255.0f);
        ++cnt;
    }
    avg[3 * i] = cnt ? sr / cnt : 0.0;
    avg[3 * i + 1] = cnt ? sg / cnt : 0.0;
    avg[3 * i + 2] = cnt ? sb / cnt : 0.0;
    counts[i] = cnt;
}

// ---- knn over the sampled vertices: Morton-sorted buckets of kBucket points under an implicit
// complete binary tree of bucket boxes (heap order, leaves at P + b); exact search in float64.
constexpr int kBucket = 16;
#ifndef MQR_KNN_WAVE
#define MQR_KNN_WAVE 1  // k_cm_knn_fill_wave (1) or the per-lane traversal k_cm_knn_fill (0): A/B builds
#endif

__device__ inline uint32_t ordered_u32(float f) {
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ inline float from_ordered(uint32_t u) {
    return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}

// Bounds of the sampled vertices: grid-stride with a capped grid, wave then workgroup reduction, one
// atomic per bound word and workgroup (256 threads).
__global__ __launch_bounds__(256) void k_cm_bounds(const float* __restrict__ V, const int32_t* __restrict__ ids,
                                                   int64_t n, uint32_t* __restrict__ bb /* min x y z (ordered), max */) {
    __shared__ uint32_t part[4][6];
    uint32_t lo[3] = {~0u, ~0u, ~0u}, hi[3] = {0u, 0u, 0u};
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int32_t v = ids[i];
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            const uint32_t o = ordered_u32(V[3 * (int64_t)v + a]);
            lo[a] = min(lo[a], o);
            hi[a] = max(hi[a], o);
        }
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        uint32_t l = lo[a], h = hi[a];
        for (int o = 32; o >= 1; o >>= 1) {
            l = min(l, (uint32_t)__shfl_xor((int)l, o, 64));
            h = max(h, (uint32_t)__shfl_xor((int)h, o, 64));
        }
        if (lane == 0) {
            part[wave][a] = l;
            part[wave][3 + a] = h;
        }
    }
    __syncthreads();
    if (threadIdx.x < 6) {
        const int c = threadIdx.x;
        uint32_t r = part[0][c];
        for (int w = 1; w < 4; ++w) r = c < 3 ? min(r, part[w][c]) : max(r, part[w][c]);
        if (c < 3) atomicMin(&bb[c], r);
        else atomicMax(&bb[c], r);
    }
}

__device__ inline uint64_t spread21(uint32_t v) {
    uint64_t x = v & 0x1fffff;
    x = (x | x << 32) & 0x1f00000000ffffull;
    x = (x | x << 16) & 0x1f0000ff0000ffull;
    x = (x | x << 8) & 0x100f00f00f00f00full;
    x = (x | x << 4) & 0x10c30c30c30c30c3ull;
    x = (x | x << 2) & 0x1249249249249249ull;
    return x;
}

__global__ void k_cm_morton(const float* __restrict__ V, const int32_t* __restrict__ ids, int64_t n,
                            const uint32_t* __restrict__ bb, uint64_t* __restrict__ keys) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int32_t v = ids[i];
    uint32_t c[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const float lo = from_ordered(bb[a]), hi = from_ordered(bb[3 + a]);
        const float t = hi > lo ? (V[3 * (int64_t)v + a] - lo) / (hi - lo) : 0.f;
        c[a] = (uint32_t)fminf(fmaxf(t * 2097151.0f, 0.f), 2097151.f);
    }
    keys[i] = spread21(c[0]) | spread21(c[1]) << 1 | spread21(c[2]) << 2;
}

// leaf boxes (bucket b = sorted points [kBucket b, kBucket (b + 1)) ); empty leaves get an inverted box.
// Also the points themselves in that order, packed (x, y, z, vertex index bits), for the leaf scans.
__global__ void k_cm_leaf_boxes(const float* __restrict__ V, const int32_t* __restrict__ sorted, int64_t n, int64_t P,
                                float4* __restrict__ lo, float4* __restrict__ hi, float4* __restrict__ pts) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= P) return;
    float l[3] = {INFINITY, INFINITY, INFINITY}, h[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int64_t j = b * kBucket; j < min(n, (b + 1) * kBucket); ++j) {
        const int32_t v = sorted[j];
        const float p[3] = {V[3 * (int64_t)v], V[3 * (int64_t)v + 1], V[3 * (int64_t)v + 2]};
        pts[j] = make_float4(p[0], p[1], p[2], __int_as_float(v));
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            l[a] = fminf(l[a], p[a]);
            h[a] = fmaxf(h[a], p[a]);
        }
    }
    lo[P + b] = make_float4(l[0], l[1], l[2], 0.f);
    hi[P + b] = make_float4(h[0], h[1], h[2], 0.f);
}

__global__ void k_cm_level(int64_t first, int64_t count, float4* __restrict__ lo, float4* __restrict__ hi) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    const int64_t n = first + i, a = 2 * n, b = a + 1;
    lo[n] = make_float4(fminf(lo[a].x, lo[b].x), fminf(lo[a].y, lo[b].y), fminf(lo[a].z, lo[b].z), 0.f);
    hi[n] = make_float4(fmaxf(hi[a].x, hi[b].x), fmaxf(hi[a].y, hi[b].y), fmaxf(hi[a].z, hi[b].z), 0.f);
}

// A lower bound of the squared distance from q to a box, in float32: every operation is correctly rounded
// (relative error <= 2^-24 each, <= 2^-21 for the whole sum of three squares of differences), so shrinking
// by 2^-18 leaves a bound below the exact value; underflow only lowers it.  Pruning on it skips no box the
// exact float64 test would keep, and the visiting order cannot change the result (the list is a total
// order on (d2, index)).
__device__ inline float box_d2_lb(const float q[3], float4 lo, float4 hi) {
    const float l[3] = {lo.x, lo.y, lo.z}, h[3] = {hi.x, hi.y, hi.z};
    float s = 0.f;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const float t = fmaxf(fmaxf(l[a] - q[a], q[a] - h[a]), 0.f);
        s += t * t;
    }
    return s * (1.0f - 0x1p-18f);
}

// The knn (3) nearest sampled vertices of every unseen vertex (exact: float64 squared distances of the
// float32 positions, ties by vertex index, the oracle's k-d tree rule), then the mean of their colours.
// K = knn at compile time: the running best list lives in registers (static indices, an unrolled
// insertion), and the traversal stack in LDS (stack-major: lane t's entry sp at stk[sp * 256 + t],
// conflict-free), sized by the host to the tree's depth + 2 (a nearest-first DFS holds at most one pending
// sibling per level plus the current pair): 20 entries for C5's 2^18 buckets instead of a fixed 32, so
// more workgroups fit a CU's LDS.  Boxes are pruned and ordered in float32 on a proven lower bound
// (box_d2_lb); candidates are compared exactly in float64.  The round-4 form kept a 64 x int64 stack and a
// KMAX = 8 list with dynamic indices in scratch (64 ms for C5's 17.5 M unseen vertices), the first
// round-5 form float64 box tests and a 32-entry stack (44.5 ms, profiles/r05_c5_kernel_stats.csv).
template <int K>
__global__ __launch_bounds__(256) void k_cm_knn_fill(const float* __restrict__ V, const int32_t* __restrict__ qids,
                                                     int64_t nq, const float4* __restrict__ pts, int64_t n,
                                                     int64_t P, const float4* __restrict__ lo,
                                                     const float4* __restrict__ hi, const double* __restrict__ avg,
                                                     float* __restrict__ out) {
    extern __shared__ int32_t stk_lds[];
    int32_t* stk = stk_lds + threadIdx.x;  // entry e of this lane at stk[256 e]
    const int lane = threadIdx.x;
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + lane;
    if (t >= nq) return;
    const int32_t qv = qids[t];
    const float qf[3] = {V[3 * (int64_t)qv], V[3 * (int64_t)qv + 1], V[3 * (int64_t)qv + 2]};
    const double q[3] = {qf[0], qf[1], qf[2]};
    double bd[K];
    int32_t bi[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        bd[k] = __builtin_inf();  // an empty slot sorts after every real candidate
        bi[k] = 0x7fffffff;
    }
    (void)lane;
    int sp = 0;
    stk[256 * sp++] = 1;
    while (sp) {
        const int32_t node = stk[256 * --sp];
        if ((double)box_d2_lb(qf, lo[node], hi[node]) > bd[K - 1]) continue;  // (never while the list has room)
        if (node >= P) {  // bucket
            const int64_t b = node - P;
            for (int64_t j = b * kBucket; j < min(n, (b + 1) * kBucket); ++j) {
                const float4 pt = pts[j];
                // float32 lower bound first (box_d2_lb's argument): most points of a visited bucket cannot
                // enter the list, and those skip the float64 distance
                const float fx = qf[0] - pt.x, fy = qf[1] - pt.y, fz = qf[2] - pt.z;
                if ((double)((fx * fx + fy * fy + fz * fz) * (1.0f - 0x1p-18f)) > bd[K - 1]) continue;
                const int32_t v = __float_as_int(pt.w);
                const double dx = q[0] - (double)pt.x, dy = q[1] - (double)pt.y, dz = q[2] - (double)pt.z;
                const double d2 = dx * dx + dy * dy + dz * dz;
                auto before = [&](int k) { return d2 < bd[k] || (d2 == bd[k] && v < bi[k]); };  // new precedes k
                if (!before(K - 1)) continue;
                // insert at its rank among the K kept, sorted by (d2, index); the last one drops out.  From
                // the end, with static indices: slot k takes slot k - 1's entry if the new one precedes it,
                // else the new entry if it precedes slot k's, else keeps its own
#pragma unroll
                for (int k = K - 1; k >= 0; --k) {
                    if (k > 0 && before(k - 1)) {
                        bd[k] = bd[k - 1];
                        bi[k] = bi[k - 1];
                    } else if (before(k)) {
                        bd[k] = d2;
                        bi[k] = v;
                    }
                }
            }
        } else {  // nearer child popped first
            const int32_t a = 2 * node, c = a + 1;
            const float da = box_d2_lb(qf, lo[a], hi[a]), dc = box_d2_lb(qf, lo[c], hi[c]);
            stk[256 * sp++] = da <= dc ? c : a;
            stk[256 * sp++] = da <= dc ? a : c;
        }
    }
    int nb = 0;
    double c[3] = {0.0, 0.0, 0.0};
#pragma unroll
    for (int k = 0; k < K; ++k)
        if (bd[k] != __builtin_inf()) {
            ++nb;
#pragma unroll
            for (int a = 0; a < 3; ++a) c[a] += avg[3 * (int64_t)bi[k] + a];
        }
    if (nb > 0)
#pragma unroll
        for (int a = 0; a < 3; ++a) c[a] /= (double)nb;
#pragma unroll
    for (int a = 0; a < 3; ++a) out[3 * (int64_t)qv + a] = (float)c[a];
}

// The same search with the traversal shared by a wave (MQR_KNN_WAVE): the wave's 64 queries -- neighbours in
// vertex order, so close in space -- walk one stack of nodes together (node indices wave-uniform, read by
// scalar loads), a node is skipped only when every lane's bound prunes it, and each lane keeps its own
// exact best list.  A lane may so test nodes it would have pruned alone: that only offers it candidates
// its own search would have rejected or met anyway, and the kept list is a total order on (d2, index), so
// the result is the same.  Inactive lanes (past the query count) prune everything.
template <int K>
__global__ __launch_bounds__(256) void k_cm_knn_fill_wave(const float* __restrict__ V, const int32_t* __restrict__ qids,
                                                          int64_t nq, const float4* __restrict__ pts, int64_t n,
                                                          int64_t P, const float4* __restrict__ lo,
                                                          const float4* __restrict__ hi,
                                                          const double* __restrict__ avg, float* __restrict__ out) {
    extern __shared__ int32_t stk_lds[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int32_t* stk = stk_lds + wave * 64;
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool active = t < nq;
    const int32_t qv = active ? qids[t] : 0;
    float qf[3] = {0.f, 0.f, 0.f};
    if (active) {
        qf[0] = V[3 * (int64_t)qv];
        qf[1] = V[3 * (int64_t)qv + 1];
        qf[2] = V[3 * (int64_t)qv + 2];
    }
    const double q[3] = {qf[0], qf[1], qf[2]};
    double bd[K];
    int32_t bi[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        bd[k] = active ? __builtin_inf() : -1.0;  // an inactive lane prunes every node
        bi[k] = 0x7fffffff;
    }
    if (__ballot(active) == 0) return;  // (wave-uniform)
    int sp = 0;
    if (lane == 0) stk[0] = 1;
    sp = 1;
    while (sp) {
        __builtin_amdgcn_wave_barrier();
        const int32_t node = __builtin_amdgcn_readfirstlane(stk[--sp]);
        const float4 nlo = lo[node], nhi = hi[node];
        if (!__ballot((double)box_d2_lb(qf, nlo, nhi) <= bd[K - 1])) continue;
        if (node >= P) {  // bucket
            const int64_t b = node - P;
            const int64_t e = min(n, (b + 1) * kBucket);
            for (int64_t j = b * kBucket; j < e; ++j) {
                const float4 pt = pts[j];
                const float fx = qf[0] - pt.x, fy = qf[1] - pt.y, fz = qf[2] - pt.z;
                if ((double)((fx * fx + fy * fy + fz * fz) * (1.0f - 0x1p-18f)) > bd[K - 1]) continue;
                const int32_t v = __float_as_int(pt.w);
                const double dx = q[0] - (double)pt.x, dy = q[1] - (double)pt.y, dz = q[2] - (double)pt.z;
                const double d2 = dx * dx + dy * dy + dz * dz;
                auto before = [&](int k) { return d2 < bd[k] || (d2 == bd[k] && v < bi[k]); };
                if (!before(K - 1)) continue;
#pragma unroll
                for (int k = K - 1; k >= 0; --k) {
                    if (k > 0 && before(k - 1)) {
                        bd[k] = bd[k - 1];
                        bi[k] = bi[k - 1];
                    } else if (before(k)) {
                        bd[k] = d2;
                        bi[k] = v;
                    }
                }
            }
        } else {  // both children, the one nearer for most lanes popped first
            const int32_t a = 2 * node, c = a + 1;
            const float da = box_d2_lb(qf, lo[a], hi[a]), dc = box_d2_lb(qf, lo[c], hi[c]);
            const uint64_t m = __ballot(active && da <= dc), act = __ballot(active);
            const bool a_first = 2 * __popcll(m) >= __popcll(act);
            __builtin_amdgcn_wave_barrier();
            if (lane == 0) {
                stk[sp] = a_first ? c : a;
                stk[sp + 1] = a_first ? a : c;
            }
            sp += 2;
        }
    }
    if (!active) return;
    int nb = 0;
    double cc[3] = {0.0, 0.0, 0.0};
#pragma unroll
    for (int k = 0; k < K; ++k)
        if (bd[k] != __builtin_inf()) {
            ++nb;
#pragma unroll
            for (int a = 0; a < 3; ++a) cc[a] += avg[3 * (int64_t)bi[k] + a];
        }
    if (nb > 0)
#pragma unroll
        for (int a = 0; a < 3; ++a) cc[a] /= (double)nb;
#pragma unroll
    for (int a = 0; a < 3; ++a) out[3 * (int64_t)qv + a] = (float)cc[a];
}

__global__ void k_cm_out_seen(const double* __restrict__ avg, const int32_t* __restrict__ counts, int64_t nv,
                              float* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nv || counts[i] == 0) return;
#pragma unroll
    for (int a = 0; a < 3; ++a) out[3 * i + a] = (float)avg[3 * i + a];
}

__global__ void k_cm_flags(const int32_t* __restrict__ counts, int64_t nv, uint8_t* __restrict__ seen,
                           uint8_t* __restrict__ unseen) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nv) return;
    seen[i] = counts[i] > 0;
    unseen[i] = counts[i] == 0;
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
    if ((vloc == MQR_DEVICE || img_loc == MQR_DEVICE || out_loc == MQR_DEVICE) && order_after_caller(device, s)) {
        (void)hipStreamDestroy(s);
        return 2;
    }
    int rc = 0;
    const int64_t HW = (int64_t)H * W;
    const bool hv = vloc != MQR_DEVICE, hi = img_loc != MQR_DEVICE, ho = out_loc != MQR_DEVICE;
    // device staging from the device-block cache (device_block.hpp), returned after the final synchronisation
    CachedBlock blk(device, (hv ? 12 * (size_t)nv : 0) + (hi ? 7 * (size_t)HW * N : 0) +
                                sizeof(ColorCam) * std::max(N, 1) + (ho ? 16 * (size_t)nv : 0) + 6 * 256);
    auto dev = [&](const void* h, size_t bytes, bool host) -> const void* {
        if (!host) return h;
        void* p = blk.take(bytes);
        if (!p || copy_to_device(device, p, h, bytes, s)) return nullptr;
        return p;
    };
    const float* dV = static_cast<const float*>(dev(vertices, sizeof(float) * 3 * nv, vloc != MQR_DEVICE));
    const uint8_t* dI = static_cast<const uint8_t*>(dev(images, (size_t)3 * HW * N, img_loc != MQR_DEVICE));
    const float* dD = static_cast<const float*>(dev(depths, sizeof(float) * HW * N, img_loc != MQR_DEVICE));
    const ColorCam* dC = static_cast<const ColorCam*>(dev(cams.data(), sizeof(ColorCam) * std::max(N, 1), true));
    float* dO = colors_out;
    int32_t* dN = counts_out;
    if (out_loc != MQR_DEVICE) {
        void* p = blk.take((sizeof(float) * 3 + sizeof(int32_t)) * nv);
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
            (copy_to_host(device, colors_out, dO, sizeof(float) * 3 * nv, s) ||
             (counts_out && copy_to_host(device, counts_out, dN, sizeof(int32_t) * nv, s)))) {
            set_error("mqr_color_vertices: copy back failed");
            rc = 1;
        }
    }
    if (hipStreamSynchronize(s) != hipSuccess && !rc) {
        set_error("mqr_color_vertices: kernel failed");
        rc = 1;
    }
    (void)hipStreamDestroy(s);
    return rc;
}

int mqr_color_map(int device, const float* vertices, int64_t nv, int vloc, const uint8_t* images, const float* t_hit,
                  int img_loc, int N, int H, int W, const double* K, const double* T_wc, double max_depth,
                  double visibility_threshold, int margin, double disc_threshold, int half_dilation, double depth_trunc,
                  int knn, float* colors_out, int32_t* counts_out, int out_loc) {
    MQR_REQUIRE(vertices && images && t_hit && K && T_wc && colors_out, "null argument");
    MQR_REQUIRE(nv >= 0 && N >= 0 && H > 0 && W > 0 && knn >= 0 && knn <= 8 && half_dilation >= 0, "bad sizes");
    MQR_REQUIRE(nv < (int64_t{1} << 31), "mqr_color_map: vertex ids are int32");
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
    if ((vloc == MQR_DEVICE || img_loc == MQR_DEVICE || out_loc == MQR_DEVICE) && order_after_caller(device, s)) {
        (void)hipStreamDestroy(s);
        return 2;
    }
    // device staging from the device-block cache (device_block.hpp): the visibility pass's arrays in one
    // block, the knn pass's (sized once the seen vertices are counted) in a second; both returned after
    // the final synchronisation
    const int64_t HW0 = (int64_t)H * W, NHW0 = HW0 * N;
    size_t tb_sel = 0;
    {
        hipcub::CountingInputIterator<int32_t> it0(0);
        if (hipcub::DeviceSelect::Flagged(nullptr, tb_sel, it0, (const uint8_t*)nullptr, (int32_t*)nullptr,
                                          (int64_t*)nullptr, (int)nv, s) != hipSuccess) {
            (void)hipStreamDestroy(s);
            set_error("mqr_color_map: select sizing failed");
            return 1;
        }
    }
    const bool hv = vloc != MQR_DEVICE, hi = img_loc != MQR_DEVICE;
    CachedBlock blk(device, (hv ? 12 * (size_t)nv : 0) + (hi ? 7 * (size_t)NHW0 : 0) + sizeof(ColorCam) * std::max(N, 1) +
                                10 * (size_t)NHW0 + (24 + 4 + 12 + 1 + 1 + 8) * (size_t)nv + 16 + tb_sel + 16 * 256);
    std::unique_ptr<CachedBlock> blk_knn;
    CachedBlock* cur = &blk;
    auto alloc = [&](size_t bytes) -> void* { return cur->take(std::max<size_t>(bytes, 16)); };
    auto dev = [&](const void* h, size_t bytes, bool host) -> const void* {
        if (!host) return h;
        void* p = alloc(bytes);
        if (!p || copy_to_device(device, p, h, bytes, s)) return nullptr;
        return p;
    };
    int rc = 0;
    auto fail = [&](const char* msg) {
        set_error(msg);
        rc = 1;
    };
    const int64_t HW = (int64_t)H * W, NHW = HW * N;
    const float* dV = static_cast<const float*>(dev(vertices, sizeof(float) * 3 * nv, vloc != MQR_DEVICE));
    const uint8_t* dI = static_cast<const uint8_t*>(dev(images, (size_t)3 * NHW, img_loc != MQR_DEVICE));
    const float* dT = static_cast<const float*>(dev(t_hit, sizeof(float) * NHW, img_loc != MQR_DEVICE));
    const ColorCam* dC = static_cast<const ColorCam*>(dev(cams.data(), sizeof(ColorCam) * std::max(N, 1), true));
    float* hx = static_cast<float*>(alloc(sizeof(float) * NHW));
    float* hy = static_cast<float*>(alloc(sizeof(float) * NHW));
    uint8_t* m0 = static_cast<uint8_t*>(alloc(NHW));
    uint8_t* mask = static_cast<uint8_t*>(alloc(NHW));
    double* avg = static_cast<double*>(alloc(sizeof(double) * 3 * nv));
    int32_t* cnt = static_cast<int32_t*>(alloc(sizeof(int32_t) * nv));
    float* dO = out_loc == MQR_DEVICE ? colors_out : static_cast<float*>(alloc(sizeof(float) * 3 * nv));
    uint8_t* fseen = static_cast<uint8_t*>(alloc(nv));
    uint8_t* funseen = static_cast<uint8_t*>(alloc(nv));
    int32_t* ids = static_cast<int32_t*>(alloc(sizeof(int32_t) * 2 * nv));  // seen, then unseen
    int64_t* nsel = static_cast<int64_t*>(alloc(2 * sizeof(int64_t)));
    if (!dV || !dI || !dT || !dC || !hx || !hy || !m0 || !mask || !avg || !cnt || !dO || !fseen || !funseen || !ids ||
        !nsel) {
        fail("mqr_color_map: device allocation or upload failed");
    }
    int64_t nseen = 0, nunseen = 0;
    if (!rc) {
        const unsigned gi = (unsigned)((NHW + 255) / 256), gv = (unsigned)((nv + 255) / 256);
        if (NHW > 0) {
            hipLaunchKernelGGL(k_cm_filter_h, dim3(gi), dim3(256), 0, s, dT, NHW, H, W, (float)depth_trunc, hx, hy);
            hipLaunchKernelGGL(k_cm_filter_v, dim3(gi), dim3(256), 0, s, hx, hy, NHW, H, W, disc_threshold, m0);
            hipLaunchKernelGGL(k_cm_dilate, dim3(gi), dim3(256), 0, s, m0, NHW, H, W, half_dilation, mask);
        }
        hipLaunchKernelGGL(k_cm_vertices, dim3(gv), dim3(256), 0, s, dV, nv, dI, dT, mask, dC, N, H, W, max_depth,
                           visibility_threshold, margin, (float)depth_trunc, avg, cnt);
        hipLaunchKernelGGL(k_cm_flags, dim3(gv), dim3(256), 0, s, cnt, nv, fseen, funseen);
        size_t tb = tb_sel;
        hipcub::CountingInputIterator<int32_t> it(0);
        void* tmp = rc ? nullptr : alloc(tb);
        if (!rc && (!tmp || hipcub::DeviceSelect::Flagged(tmp, tb, it, fseen, ids, nsel, (int)nv, s) != hipSuccess ||
                    hipcub::DeviceSelect::Flagged(tmp, tb, it, funseen, ids + nv, nsel + 1, (int)nv, s) != hipSuccess))
            fail("mqr_color_map: select failed");
        int64_t h[2] = {0, 0};
        if (!rc && (hipMemcpyAsync(h, nsel, sizeof h, hipMemcpyDeviceToHost, s) != hipSuccess ||
                    hipStreamSynchronize(s) != hipSuccess))
            fail("mqr_color_map: visibility pass failed");
        nseen = h[0];
        nunseen = h[1];
        if (!rc && hipMemsetAsync(dO, 0, sizeof(float) * 3 * nv, s) != hipSuccess) fail("mqr_color_map: memset failed");
        if (!rc && nseen > 0)
            hipLaunchKernelGGL(k_cm_out_seen, dim3(gv), dim3(256), 0, s, avg, cnt, nv, dO);
        if (!rc && knn > 0 && nseen > 0 && nunseen > 0) {
            const int64_t nb = (nseen + kBucket - 1) / kBucket;
            int64_t P = 1;
            while (P < nb) P <<= 1;
            size_t tbs = 0;
            if (hipcub::DeviceRadixSort::SortPairs(nullptr, tbs, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                                   (const int32_t*)nullptr, (int32_t*)nullptr, (int)nseen, 0, 63, s) !=
                hipSuccess)
                fail("mqr_color_map: knn allocation failed");
            blk_knn.reset(new CachedBlock(device, 24 + 16 * (size_t)nseen + 4 * (size_t)nseen + 64 * (size_t)P +
                                                      16 * (size_t)nseen + tbs + 8 * 256));
            cur = blk_knn.get();
            uint32_t* bb = static_cast<uint32_t*>(alloc(6 * sizeof(uint32_t)));
            uint64_t* keys = static_cast<uint64_t*>(alloc(sizeof(uint64_t) * 2 * nseen));
            int32_t* sorted = static_cast<int32_t*>(alloc(sizeof(int32_t) * nseen));
            float4* blo = static_cast<float4*>(alloc(sizeof(float4) * 2 * P));
            float4* bhi = static_cast<float4*>(alloc(sizeof(float4) * 2 * P));
            float4* pts = static_cast<float4*>(alloc(sizeof(float4) * nseen));
            if (!rc && (!bb || !keys || !sorted || !blo || !bhi || !pts)) fail("mqr_color_map: knn allocation failed");
            void* tmps = rc ? nullptr : alloc(tbs);
            if (!rc && !tmps) fail("mqr_color_map: knn allocation failed");
            if (!rc) {
                const uint32_t init[6] = {~0u, ~0u, ~0u, 0u, 0u, 0u};
                const unsigned gs = (unsigned)((nseen + 255) / 256);
                if (hipMemcpyAsync(bb, init, sizeof init, hipMemcpyHostToDevice, s) != hipSuccess) fail("mqr_color_map: copy");
                hipLaunchKernelGGL(k_cm_bounds, dim3(std::min(gs, 4096u)), dim3(256), 0, s, dV, ids, nseen, bb);
                hipLaunchKernelGGL(k_cm_morton, dim3(gs), dim3(256), 0, s, dV, ids, nseen, bb, keys);
                if (hipcub::DeviceRadixSort::SortPairs(tmps, tbs, keys, keys + nseen, ids, sorted, (int)nseen, 0, 63, s) !=
                    hipSuccess)
                    fail("mqr_color_map: sort failed");
                hipLaunchKernelGGL(k_cm_leaf_boxes, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, s, dV, sorted, nseen,
                                   P, blo, bhi, pts);
                for (int64_t first = P / 2; first >= 1; first /= 2)
                    hipLaunchKernelGGL(k_cm_level, dim3((unsigned)((first + 255) / 256)), dim3(256), 0, s, first, first,
                                       blo, bhi);
                const dim3 gq((unsigned)((nunseen + 255) / 256));
                int depth = 0;  // levels below the root of the P-leaf tree
                while ((int64_t{1} << depth) < P) ++depth;
                const bool wave = MQR_KNN_WAVE && depth + 2 <= 64;  // (the wave stack holds 64 entries)
                const size_t lds = wave ? sizeof(int32_t) * 4 * 64 : sizeof(int32_t) * 256 * (size_t)(depth + 2);
                auto fill = [&](auto kern) {
                    hipLaunchKernelGGL(kern, gq, dim3(256), lds, s, dV, ids + nv, nunseen, pts, nseen, P, blo, bhi,
                                       avg, dO);
                };
                switch (knn) {  // knn in [1, 8] (checked on entry)
                    case 1: wave ? fill(k_cm_knn_fill_wave<1>) : fill(k_cm_knn_fill<1>); break;
                    case 2: wave ? fill(k_cm_knn_fill_wave<2>) : fill(k_cm_knn_fill<2>); break;
                    case 3: wave ? fill(k_cm_knn_fill_wave<3>) : fill(k_cm_knn_fill<3>); break;
                    case 4: wave ? fill(k_cm_knn_fill_wave<4>) : fill(k_cm_knn_fill<4>); break;
                    case 5: wave ? fill(k_cm_knn_fill_wave<5>) : fill(k_cm_knn_fill<5>); break;
                    case 6: wave ? fill(k_cm_knn_fill_wave<6>) : fill(k_cm_knn_fill<6>); break;
                    case 7: wave ? fill(k_cm_knn_fill_wave<7>) : fill(k_cm_knn_fill<7>); break;
                    default: wave ? fill(k_cm_knn_fill_wave<8>) : fill(k_cm_knn_fill<8>); break;
                }
            }
        }
        if (!rc && hipGetLastError() != hipSuccess) fail("mqr_color_map: kernel launch failed");
        if (!rc && out_loc != MQR_DEVICE &&
            (copy_to_host(device, colors_out, dO, sizeof(float) * 3 * nv, s) ||
             (counts_out && copy_to_host(device, counts_out, cnt, sizeof(int32_t) * nv, s))))
            fail("mqr_color_map: copy back failed");
        if (!rc && out_loc == MQR_DEVICE && counts_out &&
            hipMemcpyAsync(counts_out, cnt, sizeof(int32_t) * nv, hipMemcpyDeviceToDevice, s) != hipSuccess)
            fail("mqr_color_map: copy failed");
    }
    if (hipStreamSynchronize(s) != hipSuccess && !rc) fail("mqr_color_map: kernel failed");
    (void)hipStreamDestroy(s);
    return rc;
}

}  // extern "C"

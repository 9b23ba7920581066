// confidence.hip -- multi-view depth confidence (reference: scripts/processing/reconstruction/
// confidence_estimation/estimate_depth_confidences.py:15-79 build_confidence_map and
// compute_pixel_error_map.py:4-220).
//
// One thread per reference pixel, the +-r neighbour loop in registers, every frame of the
// sequence resident in HBM (the reference re-reads and re-decodes each frame ~21x from disk).
// Arithmetic is float64 in numpy's order with the two float32 roundings numpy performs
// (interpolated target depth, error), so valid_count / confidence match the reference exactly
// (pinned by tests/golden/confidence_golden.npz).  The kernel is FP64-VALU bound; the per-(pixel,
// neighbour) instruction count is cut without changing a result bit: frame parameters widened
// once on the host, the float32 error's threshold test as one float64 compare of the squared
// distance, the quotients by Z sharing one refined reciprocal and those by fx / fy using a
// host-rounded reciprocal (Markstein correction), all checked against IEEE division
// (mqr_check_div64, tests/test_gpu_numerics.py).
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <type_traits>
#include <vector>

#include "mqr_common.hpp"

namespace mqr {

// Per-frame parameters, widened to double on the host (numpy promotes the float32 K / T entries to
// float64 in every product; widening is exact, so doing it once per frame changes no bit), plus the
// correctly rounded reciprocals of fx and fy for the quotient below.
struct ConfFrame {
    double fx, fy, cx, cy;
    double rfx, rfy;  // RN(1 / fx), RN(1 / fy)
    double Tcw[12];   // camera -> world, rows 0..2
    double Tinv[12];  // world -> camera (float32 np.linalg.inv of Tcw, widened)
    // consistency band terms (pixel_decide): c1 = dR (1 + eR), c0 = dT (1 + eR) + eR (sd + 1) + 1e-9
    // from dR = ||R_inv - R^-1||_F, dT = |t_inv - t*| (Tinv against the exact inverse of Tcw) and
    // eR = ||R^T R - I||_F of Tcw's rotation; +inf when they are not finite
    double c1, c0;
    // float32 prefilter (pixel_decide32): the float32 Tinv and K entries as given, and per coordinate
    // of Tinv pw the bound of the float32 evaluation's error, E = ea[c] m + eb[c] with m = max |pw|
    // (ea = 8u sum |R row|, eb = 8u |t|, rounded up; u = 2^-24)
    float Tf[12];
    float fxf, fyf, cxf, cyf;
    float cxu, cyu;  // 2u |cx| (1 + 4u), 2u |cy| (1 + 4u): decide32_stage1_bf's bound of 2u |uu|, 2u |vv|
    float ea[3], eb[3];
    float eam, ebm;  // max(ea), max(eb): decide32_stage1_bf's one bound for all three coordinates
    float eam8, ebm8;  // 8 eam, max(8 ebm, 1e-6): its depth test Z >= max(8 E, 1e-6) in one fma (implied)
    int ok;  // frame_ok (a neighbour that is not ok is skipped, as the reference skips failed loads)
    // as a reference frame (host, per call): the largest c1 / c0 of its ok neighbours in the +-r window,
    // and (windows of <= 64 frames) the window's neighbour mask -- bit i: frame max(0, ref - r) + i is
    // ok and not the reference -- so the kernel walks its neighbours with a scalar bit scan
    double wc1, wc0;
    uint64_t wmask;
};

// ---- correctly rounded float64 quotients without the v_div_scale / v_div_fixup wrapper ----------
// (i) a / d with d's reciprocal refined once and shared by several numerators: the compiler's own
// division sequence (v_rcp_f64, two Newton steps, quotient, one residual correction) minus
// v_div_scale / v_div_fmas scaling and v_div_fixup, which leave operands and result unchanged while
// |a|, |d| and the quotient stay within [2^-500, 2^500] (callers check; zero numerators are exact).
struct Rcp64 {
    double d, r;
};
__device__ __forceinline__ Rcp64 rcp64_refine(double d) {
    const double r0 = __builtin_amdgcn_rcp(d);
    const double e0 = __builtin_fma(-d, r0, 1.0);
    const double r1 = __builtin_fma(r0, e0, r0);
    const double e1 = __builtin_fma(-d, r1, 1.0);
    return {d, __builtin_fma(r1, e1, r1)};
}
__device__ __forceinline__ double div64_core(double a, const Rcp64& rd) {
    const double q = a * rd.r;
    const double rem = __builtin_fma(-rd.d, q, a);
    return __builtin_fma(rem, rd.r, q);
}
__device__ __forceinline__ bool div64_safe(double x) {
    const double m = fabs(x);
    return m == 0.0 || (m >= 0x1p-500 && m <= 0x1p500);
}
// (ii) a / b with y = RN(1 / b) computed on the host: q = RN(a y) is within one ulp of a / b, and
// RN(q + (a - b q) y) is then RN(a / b) (Markstein's theorem; radix 2, round to nearest).
__device__ __forceinline__ double div64_by_rn_rcp(double a, double b, double y) {
    const double q = a * y;
    const double rem = __builtin_fma(-b, q, a);
    return __builtin_fma(rem, y, q);
}

// One (ref pixel, target frame) evaluation of compute_pixel_error_map.py:120-220 in numpy's float64
// order with its two float32 roundings.  Returns 1 when the pixel gets a finite-input error; `d2`
// = the squared distance whose sqrt, rounded to float32, is the reference's error.
__device__ inline int pixel_error_d2(const float* __restrict__ tgt, int H, int W, const ConfFrame& ft,
                                     const double pw[3], double depth_max, double* d2) {
    const float dmf = (float)depth_max;
    double pt[3];
#pragma unroll
    for (int i = 0; i < 3; ++i)  // (... + T3 * 1.0): the product with 1.0 is exact
        pt[i] = ft.Tinv[i * 4 + 0] * pw[0] + ft.Tinv[i * 4 + 1] * pw[1] + ft.Tinv[i * 4 + 2] * pw[2] + ft.Tinv[i * 4 + 3];
    const double X = pt[0], Y = pt[1], Z = pt[2];
    if (!(Z > 0 && isfinite(Z) && Z <= depth_max && isfinite(X) && isfinite(Y))) return 0;
    const double ax = X * ft.fx, ay = Y * ft.fy;
    double qx, qy;
    if (div64_safe(Z) && div64_safe(ax) && div64_safe(ay) && fabs(ax) <= 0x1p400 * Z && fabs(ay) <= 0x1p400 * Z) {
        const Rcp64 rz = rcp64_refine(Z);  // shared by both quotients
        qx = div64_core(ax, rz);
        qy = div64_core(ay, rz);
    } else {
        qx = ax / Z;
        qy = ay / Z;
    }
    const double uu = qx + ft.cx;
    const double vv = qy + ft.cy;
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
    const double xt = div64_by_rn_rcp((uu - ft.cx) * ztd, ft.fx, ft.rfx);
    const double yt = div64_by_rn_rcp((vv - ft.cy) * ztd, ft.fy, ft.rfy);
    double q[3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
        q[i] = ft.Tcw[i * 4 + 0] * xt + ft.Tcw[i * 4 + 1] * yt + ft.Tcw[i * 4 + 2] * ztd + ft.Tcw[i * 4 + 3];
    const double dx = pw[0] - q[0], dy = pw[1] - q[1], dz = pw[2] - q[2];
    *d2 = dx * dx + dy * dy + dz * dz;
    return 1;
}

// The reference's consistency test err <= threshold (err = |pw - q| as float32, q the target pixel
// back-projected at its interpolated depth zt and mapped to the world by Tcw) decided without the
// back-projection whenever the answer is clear, exactly as the full computation decides it:
//   q - pw = Tcw p' - pw with p' = (xt, yt, zt) the back-projection, which lies on the ray through
//   pt = Tinv pw at depth zt up to rounding (xt = X zt / Z (1 + 5u) + ulp(uu) zt / fx), so with
//   R = Tcw's rotation and Tinv = Tcw^-1 + E:
//     |pw - q| = |Z - zt| |pt| / Z (1 +- eR) +- (dR |pw| + dT) (1 + eR) +- tiny
//   where dR = ||R_inv - R^-1||_F, dT = |t_inv - t*| and eR = ||R^T R - I||_F are the frame's
//   (host-computed) defects of the float32 matrices.  With the band B = c1 |pw| + c0 around
//   sd = sqrt(d2_max) (c1 = dR (1 + eR), c0 = dT (1 + eR) + eR (sd + 1) + 1e-9, maxima over the
//   reference frame's neighbours, k_confidence) the pair is consistent when
//   |Z - zt|^2 |pt|^2 <= lo2 Z^2 (lo2 = (sd - B)^2 (1 - 1e-12)) and inconsistent when > hi2 Z^2
//   (hi2 = (sd + B)^2 (1 + 1e-12)); the margins cover the fp64 roundings.  Only pairs inside the band
//   take the full float64 back-projection (pixel_error_d2's tail).  A NaN / infinite band (a frame
//   whose defects are not finite) fails both compares and sends every pair to the exact tail.
// The validity tests are pixel_error_d2's, restated without changing a decision:
//   * Z <= zmax (= min(depth_max, DBL_MAX)) also rejects Z = inf;
//   * X, Y are not tested: a non-finite X or Y gives a non-finite uu / vv, which fails the range test;
//   * the range test 0 <= uu < W - 1, 0 <= vv < H - 1 is exactly floor(uu) >= 0, floor(uu) + 1 < W
//     (and for v), and implies the |coord| < 10 max(W, H) and finiteness tests (NaN fails it);
//   * (double)u1 = floor(uu) + 1 exactly.
// Returns 0 = no finite error (not counted), 1 = consistent, 2 = inconsistent, | kTail when decided by
// the float64 back-projection.
constexpr int kTail = 4;
__device__ inline int pixel_decide(const float* __restrict__ tgt, int W, double wm1, double hm1, const ConfFrame& ft,
                                   const double pw[3], double zmax, float dmf, double lo2, double hi2,
                                   double d2_max) {
    if (!ft.ok) return 0;  // a neighbour that is not ok is skipped (frame_ok)
    // (loading every frame parameter in one batch before the first branch measured 3 % slower: the
    // scalar reads hit the scalar cache, and 98 SGPRs cost occupancy)
    const double* Ti = ft.Tinv;
    const double Z = Ti[8] * pw[0] + Ti[9] * pw[1] + Ti[10] * pw[2] + Ti[11];
    if (!(Z > 0 && Z <= zmax)) return 0;
    const double X = Ti[0] * pw[0] + Ti[1] * pw[1] + Ti[2] * pw[2] + Ti[3];
    const double Y = Ti[4] * pw[0] + Ti[5] * pw[1] + Ti[6] * pw[2] + Ti[7];
    const double ax = X * ft.fx, ay = Y * ft.fy;
    const double aax = fabs(ax), aay = fabs(ay), zb = 0x1p400 * Z;
    // div64_safe(Z) && div64_safe(ax) && div64_safe(ay) && |ax|, |ay| <= 2^400 Z, without short-circuit
    const bool fast = (Z >= 0x1p-500) & (Z <= 0x1p500) & ((aax >= 0x1p-500) | (ax == 0.0)) &
                      ((aay >= 0x1p-500) | (ay == 0.0)) & (aax <= zb) & (aay <= zb);
    double qx, qy;
    if (__builtin_expect(fast, 1)) {
        const Rcp64 rz = rcp64_refine(Z);
        qx = div64_core(ax, rz);
        qy = div64_core(ay, rz);
    } else {
        qx = ax / Z;
        qy = ay / Z;
    }
    const double uu = qx + ft.cx;
    const double vv = qy + ft.cy;
    if (!((uu >= 0.0) & (uu < wm1) & (vv >= 0.0) & (vv < hm1))) return 0;
    const double fu0 = floor(uu), fv0 = floor(vv);
    const int u0 = (int)fu0, v0 = (int)fv0;
    // both rows' taps read before any test on them (short-circuit tests between the two reads made
    // the compiler issue the second read after the first had returned)
    float2 ab, cd;
    const float* row0 = tgt + (int64_t)v0 * W + u0;
    __builtin_memcpy(&ab, row0, sizeof(float2));
    __builtin_memcpy(&cd, row0 + W, sizeof(float2));
    const float Ia = ab.x, Ib = ab.y, Ic = cd.x, Id = cd.y;
    const bool taps = (Ib > 0) & (Ib <= dmf) & (Ia > 0) & (Ia <= dmf) & (Ic > 0) & (Ic <= dmf) & (Id > 0) & (Id <= dmf);
    if (!taps) return 0;
    const double du1 = fu0 + 1.0, dv1 = fv0 + 1.0;
    // the filter, on a float32 interpolation zf of the target depth: every weight and product is
    // positive, so zf is within 7 * 2^-24 relative of the reference's sum and zt (its float32
    // rounding) within 2^-24: |zf - zt| <= 2^-21 zt <= 2^-21 depth_max, covered by the band's
    // 2^-18 depth_max * ray-length term (fill_frame).  The reference's tests zt > 0 and finite hold
    // for positive finite taps (weights >= 0 summing to 1), so they cannot reject a pair here.
    const float gu = (float)(du1 - uu), gv = (float)(dv1 - vv), fu = (float)(uu - fu0), fv = (float)(vv - fv0);
    const float zf = __builtin_fmaf(fu * fv, Id, __builtin_fmaf(gu * fv, Ic, __builtin_fmaf(fu * gv, Ib, (gu * gv) * Ia)));
    const double dz = Z - (double)zf, Z2 = Z * Z;
    const double lhs = dz * dz * (X * X + Y * Y + Z2);
    if (lhs <= lo2 * Z2) return 1;
    if (lhs > hi2 * Z2) return 2;
    // inside the band: the reference's own interpolation and float64 back-projection (kTail marks the
    // decisions taken here, for mqr_confidence_stats)
    const double wa = (du1 - uu) * (dv1 - vv);
    const double wb = (uu - fu0) * (dv1 - vv);
    const double wc = (du1 - uu) * (vv - fv0);
    const double wd = (uu - fu0) * (vv - fv0);
    const float zt = (float)(wa * Ia + wb * Ib + wc * Ic + wd * Id);
    if (!(zt > 0 && isfinite(zt))) return kTail;
    const double ztd = (double)zt;
    const double xt = div64_by_rn_rcp((uu - ft.cx) * ztd, ft.fx, ft.rfx);
    const double yt = div64_by_rn_rcp((vv - ft.cy) * ztd, ft.fy, ft.rfy);
    double q[3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
        q[i] = ft.Tcw[i * 4 + 0] * xt + ft.Tcw[i * 4 + 1] * yt + ft.Tcw[i * 4 + 2] * ztd + ft.Tcw[i * 4 + 3];
    const double ex = pw[0] - q[0], ey = pw[1] - q[1], ez = pw[2] - q[2];
    const double d2 = ex * ex + ey * ey + ez * ez;
    // a NaN error is not valid (valid_count += ~isnan(error_map), estimate_depth_confidences.py:66)
    if (d2 != d2) return kTail;
    return kTail | (d2 <= d2_max ? 1 : 2);
}

// The same decision as pixel_decide from a float32 forward projection with rigorous error bounds:
// returns 0 / 1 / 2 where every quantity it rests on is certain, -1 where it is not (the caller then
// runs pixel_decide's float64 path from scratch).  With X, Y, Z the float32 Tinv pw (error <= E_c =
// 8u (sum |R row| max|pw| + |t|): three FMAs with one rounding each, pw rounded to float32 once):
//   * Z <= 0 or Z > zmax certain -> 0; Z's bracket straddling either bound -> -1;
//   * uu = fx X / Z + cx (v_rcp_f32 within 1 ulp, two products, one sum) is within
//     E_u = |fx| / Z (E_X + (|X| + E_X) E_Z / (Z - E_Z)) (1 + 8u) + 5u |qx| + 2u |uu| of the reference's
//     float64 uu (whose own rounding, ~2^-50 relative, the 8u factors cover); likewise vv;
//   * uu certainly < 0 or >= W - 1 (or vv) -> 0; floor(uu), floor(vv) certain when uu, vv lie at
//     least E_u, E_v away from an integer, else -1 -- then the taps, the range test and the tap test are
//     the reference's exactly;
//   * the band filter of pixel_decide on float32 values: zf from float32 weights moves by at most
//     E_u (|Ib - Ia| + |Id - Ic|) + E_v (|Ic - Ia| + |Id - Ib|) against the weights of the exact uu, vv
//     (the band's zterm already covers the float32 interpolation itself); with E_dz = E_Z + that + u zf
//     and E_P the bound of X^2 + Y^2 + Z^2, the pair is consistent when (|dz| + E_dz)^2 (P + E_P) <=
//     lo2 (Z - E_Z)^2 and inconsistent when (|dz| - E_dz)^2 (P - E_P) > hi2 (Z + E_Z)^2, each side
//     given 8u of rounding slack; otherwise -1.
// Every test is written so that a NaN operand fails it (-> -1, the float64 path decides).
// float32 neighbours of a double: the largest float <= x / the smallest float >= x (NaN stays NaN,
// values past FLT_MAX go to FLT_MAX / +inf)
__device__ __forceinline__ float float_step(float f, bool up) {  // adjacent float toward +-inf (f finite)
    if (f == 0.0f) return up ? 0x1p-149f : -0x1p-149f;
    const uint32_t b = __float_as_uint(f);
    return __uint_as_float((f > 0.0f) == up ? b + 1 : b - 1);
}
__device__ __forceinline__ float round_down_f(double x) {
    const float f = (float)x;
    return (double)f > x ? float_step(f, false) : f;
}
__device__ __forceinline__ float round_up_f(double x) {
    const float f = (float)x;
    return (double)f < x ? float_step(f, true) : f;
}
struct Pix32 {
    float p[3], m;     // pw as float32, max |pw| (rounded up)
    float lo2, hi2;    // the band bounds, rounded down / up
    float zlo, zhi;    // zmax rounded down / up
    float lo2s, hi2s;  // lo2 (1 - 16u) / (1 + 16u) rounded down, hi2 (1 + 16u) / (1 - 16u) rounded up
                       // (decide32_stage2_bf: the slack for its products' roundings folded in)
};
// Stage 1 of pixel_decide32 for one (pixel, neighbour) pair: the float32 projection, its error
// bounds and the range / floor certainty tests, and -- for a pair that gets that far -- the two tap
// rows' loads, issued here so that they are in flight while the next neighbour's stage 1 runs
// (k_confidence pipelines the neighbour loop: the kernel is bound by these loads' latency, not by
// its VALU work).  st: 0 decided (no finite error), 1 taps pending, -1 undecided (float64 path).
struct Stage32 {
    int st;
    bool go, und;  // (BF: st == 1 / st == -1 as lane masks -- stage 2's decision stays in boolean form)
    float Z, EZ, P, EP, uu, vv, Eu, Ev;  // (floor(uu), floor(vv) are recomputed in stage 2: registers)
    float2 ab, cd;
};
template <bool DIAG = false>  // DIAG (timing only, wrong results): no tap loads
__device__ __forceinline__ Stage32 decide32_stage1(const float* __restrict__ tgt, int W, int H, float wm1, float hm1,
                                                   const ConfFrame& ft, const Pix32& px) {
    constexpr float u = 0x1p-24f;
    Stage32 r;
    r.st = 0;
    const float* T = ft.Tf;
    const float X = __builtin_fmaf(T[0], px.p[0], __builtin_fmaf(T[1], px.p[1], __builtin_fmaf(T[2], px.p[2], T[3])));
    const float Y = __builtin_fmaf(T[4], px.p[0], __builtin_fmaf(T[5], px.p[1], __builtin_fmaf(T[6], px.p[2], T[7])));
    const float Z = __builtin_fmaf(T[8], px.p[0], __builtin_fmaf(T[9], px.p[1], __builtin_fmaf(T[10], px.p[2], T[11])));
    const float EX = __builtin_fmaf(ft.ea[0], px.m, ft.eb[0]);
    const float EY = __builtin_fmaf(ft.ea[1], px.m, ft.eb[1]);
    const float EZ = __builtin_fmaf(ft.ea[2], px.m, ft.eb[2]);
    // (comparisons of computed sums are made strict where rounding could otherwise flip them:
    // RN(x) > c implies x > c and RN(x) < c implies x < c for a representable c)
    const float zl = Z - EZ, zh = Z + EZ;
    r.Z = Z;
    r.EZ = EZ;
    if (Z <= -EZ) return r;     // Z <= 0 certain
    if (zl > px.zhi) return r;  // Z > zmax certain
    r.st = -1;
    if (!(zl > 0.0f && zh < px.zlo && EZ <= 0.125f * Z && Z >= 1e-6f)) return r;
    const float inv = __builtin_amdgcn_rcpf(Z);
    const float qx = (X * ft.fxf) * inv, qy = (Y * ft.fyf) * inv;
    const float uu = qx + ft.cxf, vv = qy + ft.cyf;
    const float irl = inv * (1.0f + 2.0f * EZ * inv);  // >= 1 / (Z - E_Z) for E_Z <= Z / 8
    const float ezr = EZ * irl;
    const float Eu = __builtin_fabsf(ft.fxf) * inv * (EX + (__builtin_fabsf(X) + EX) * ezr) * (1.0f + 16.0f * u) +
                     5.0f * u * __builtin_fabsf(qx) + 2.0f * u * __builtin_fabsf(uu);
    const float Ev = __builtin_fabsf(ft.fyf) * inv * (EY + (__builtin_fabsf(Y) + EY) * ezr) * (1.0f + 16.0f * u) +
                     5.0f * u * __builtin_fabsf(qy) + 2.0f * u * __builtin_fabsf(vv);
    if ((uu + Eu < 0.0f) | (uu - Eu > wm1) | (vv + Ev < 0.0f) | (vv - Ev > hm1)) {  // out of range certain
        r.st = 0;
        return r;
    }
    const float fu0 = __builtin_floorf(uu), fv0 = __builtin_floorf(vv);
    const float ru = uu - fu0, rv = vv - fv0;  // exact (|uu|, |vv| < 2^23 here)
    if (!((ru >= Eu) & (ru + Eu < 1.0f) & (rv >= Ev) & (rv + Ev < 1.0f) & (uu < 0x1p22f) & (vv < 0x1p22f))) return r;
    const int u0 = (int)fu0, v0 = (int)fv0;
    if (!((u0 >= 0) & (u0 + 1 < W) & (v0 >= 0) & (v0 + 1 < H))) {
        r.st = 0;
        return r;
    }
    r.st = 1;
    r.P = __builtin_fmaf(X, X, __builtin_fmaf(Y, Y, Z * Z));
    r.EP = 2.0f * (__builtin_fabsf(X) * EX + __builtin_fabsf(Y) * EY + Z * EZ) + (EX * EX + EY * EY + EZ * EZ) +
           8.0f * u * r.P;
    r.uu = uu;
    r.vv = vv;
    r.Eu = Eu;
    r.Ev = Ev;
    if (DIAG) {
        r.ab = make_float2(1.0f + r.uu * 1e-30f, 1.0f);
        r.cd = make_float2(1.0f, 1.0f + r.vv * 1e-30f);
        return r;
    }
    const float* row0 = tgt + (int64_t)v0 * W + u0;  // the two taps of a row in one 8-byte load
    __builtin_memcpy(&r.ab, row0, sizeof(float2));
    __builtin_memcpy(&r.cd, row0 + W, sizeof(float2));
    return r;
}

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
// decide32_stage1 without branches (BF): every lane evaluates the whole chain and the decision is
// selected at the end; the two tap rows are read by buffer loads whose offset is past the frame's
// end (reads 0, which fails the tap test) for lanes that do not reach them.  The same decisions as
// decide32_stage1 (NaN operands still fail every test they meet); the frame's byte count 4HW + 4W
// must fit 31 bits (host).
__device__ __forceinline__ Stage32 decide32_stage1_bf(__amdgpu_buffer_rsrc_t rs, uint32_t W4, uint32_t past_end,
                                                      int W, int H, const ConfFrame& ft, const Pix32& px) {
    constexpr float u = 0x1p-24f;
    Stage32 r;
    const float* T = ft.Tf;
    const float X = __builtin_fmaf(T[0], px.p[0], __builtin_fmaf(T[1], px.p[1], __builtin_fmaf(T[2], px.p[2], T[3])));
    const float Y = __builtin_fmaf(T[4], px.p[0], __builtin_fmaf(T[5], px.p[1], __builtin_fmaf(T[6], px.p[2], T[7])));
    const float Z = __builtin_fmaf(T[8], px.p[0], __builtin_fmaf(T[9], px.p[1], __builtin_fmaf(T[10], px.p[2], T[11])));
    // one bound E >= E_X, E_Y, E_Z (the frame's largest row terms)
    const float EZ = __builtin_fmaf(ft.eam, px.m, ft.ebm);
    r.Z = Z;
    r.EZ = EZ;
    // Z <= 0 or Z > zmax certain -> 0; Z in (0, zmax] certain with E_Z <= Z / 8 and Z >= 1e-6 (then
    // Z - E_Z >= 7 Z / 8 > 0) -> go on; else -1.  (fmaxf drops a NaN E_Z, whose Z + E_Z then fails.)
    const bool none_z = (Z <= -EZ) | (Z - EZ > px.zhi);
    const bool ok_z = (Z >= __builtin_fmaf(ft.eam8, px.m, ft.ebm8)) & (Z + EZ < px.zlo);  // Z >= max(8 E, 1e-6)
    const float inv = __builtin_amdgcn_rcpf(Z);
    const float qx = (X * ft.fxf) * inv, qy = (Y * ft.fyf) * inv;
    const float uu = qx + ft.cxf, vv = qy + ft.cyf;
    // |uu - uu*| <= (|fx| E_X + |fx X / Z| E_Z) / (Z - E_Z) + 5u |qx| + 2u |uu|  (decide32_stage1), with
    // qx = fx X / Z in float within 3u and 2u |uu| <= 2u |qx| + 2u |cx| (1 + 4u): every term positive, the
    // bound's own roundings inside its 1 + 16u factor (folded into irl)
    // E / (Z - E) <= x (1 + 2x) for x = E / Z <= 1/8, evaluated as e1 (1 + 2 e1) with e1 = E inv (three
    // roundings: rcp, product, fma), E carrying the 1 + 16u slack (host): with E_X = E_Y = E_Z = E,
    // (|fx| E + |qx| E) / (Z - E) (1 + 16u) <= (|fx| + |qx|) ei
    const float e1 = EZ * inv;
    const float ei = __builtin_fmaf(e1 + e1, e1, e1);
    const float aqx = __builtin_fabsf(qx), aqy = __builtin_fabsf(qy);
    const float Eu = __builtin_fmaf(__builtin_fabsf(ft.fxf) + aqx, ei, __builtin_fmaf(7.5f * u, aqx, ft.cxu));
    const float Ev = __builtin_fmaf(__builtin_fabsf(ft.fyf) + aqy, ei, __builtin_fmaf(7.5f * u, aqy, ft.cyu));
    const float fu0 = __builtin_floorf(uu), fv0 = __builtin_floorf(vv);
    const float ru = uu - fu0, rv = vv - fv0;  // exact for every float
    // floor certain: uu, vv at least E away from an integer (implies |uu|, |vv| < 2^23, where ru > 0 is
    // possible, so the int conversions below cannot saturate; NaN fails it)
    const bool sure = (ru >= Eu) & (ru + Eu < 1.0f) & (rv >= Ev) & (rv + Ev < 1.0f);
    const int u0 = (int)fu0, v0 = (int)fv0;
    const bool in_img = ((uint32_t)u0 < (uint32_t)(W - 1)) & ((uint32_t)v0 < (uint32_t)(H - 1));
    // none_z -> 0; else !ok_z or the floors uncertain -> -1 (near the image border too: rare); else
    // out of the image -> 0; else taps
    const bool go = ok_z & sure & in_img;
    r.go = go;
    r.und = !(go | none_z | (ok_z & sure));
    // P = X^2 + Y^2 + Z^2 and, in EP, a RELATIVE bound rho of its error (stage 2 uses P (1 +- rho)):
    // |P* - P| <= 2 E (|X| + |Y| + Z) + 3 E^2 <= 2 sqrt(3) E sqrt(P) + 3 E^2 and sqrt(P) >= Z, so
    // rho = 2 sqrt(3) (E / Z) + 3 (E / Z)^2 + 8u (P's own roundings), E / Z <= ei; 3.5 and 3.01 cover the
    // roundings of rho itself
    r.P = __builtin_fmaf(X, X, __builtin_fmaf(Y, Y, Z * Z));
    r.EP = __builtin_fmaf(ei, __builtin_fmaf(3.01f, ei, 3.5f), 8.0f * u);
    r.uu = ru;  // (the fractions: stage 2 interpolates with them)
    r.vv = rv;
    r.Eu = Eu;
    r.Ev = Ev;
    const uint32_t off = go ? __umul24((uint32_t)v0, W4) + ((uint32_t)u0 << 2) : past_end;
    const u32x2 a = __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0, 0);
    const u32x2 c = __builtin_amdgcn_raw_buffer_load_b64(rs, off, W4, 0);  // (the next row: scalar offset)
    r.ab = make_float2(__uint_as_float(a.x), __uint_as_float(a.y));
    r.cd = make_float2(__uint_as_float(c.x), __uint_as_float(c.y));
    return r;
}

// Stage 2: the tap test and the band filter on the float32 values (see the comment above); returns
// 0 / 1 / 2, or -1 when the float64 path must decide.
// dmb: the bits of depth_max as float32 when it is > 0, else 0.  A tap passes the reference's
// 0 < I <= depth_max exactly when bits(I) - 1 < dmb as unsigned integers: positive floats (and +inf)
// order like their bits, +-0, negatives and NaNs fall outside -- four subtractions, two maxima and one
// compare for the eight float compares.
__device__ __forceinline__ int decide32_stage2(const Stage32& r, const Pix32& px, uint32_t dmb) {
    constexpr float u = 0x1p-24f;
    if (r.st <= 0) return r.st;
    const float Ia = r.ab.x, Ib = r.ab.y, Ic = r.cd.x, Id = r.cd.y;
    const uint32_t tmax = max(max(__float_as_uint(Ia) - 1u, __float_as_uint(Ib) - 1u),
                              max(__float_as_uint(Ic) - 1u, __float_as_uint(Id) - 1u));
    if (!(tmax < dmb)) return 0;
    const float fu0 = __builtin_floorf(r.uu), fv0 = __builtin_floorf(r.vv);
    const float fu = r.uu - fu0, fv = r.vv - fv0;
    const float gu = (fu0 + 1.0f) - r.uu, gv = (fv0 + 1.0f) - r.vv;
    const float zf = __builtin_fmaf(fu * fv, Id, __builtin_fmaf(gu * fv, Ic, __builtin_fmaf(fu * gv, Ib, (gu * gv) * Ia)));
    const float Edz = r.EZ + r.Eu * (__builtin_fabsf(Ib - Ia) + __builtin_fabsf(Id - Ic)) +
                      r.Ev * (__builtin_fabsf(Ic - Ia) + __builtin_fabsf(Id - Ib)) + 8.0f * u * zf;
    const float dz = __builtin_fabsf(r.Z - zf);
    const float zl = r.Z - r.EZ, zh = r.Z + r.EZ;  // (the same roundings as in stage 1)
    const float a1 = dz + Edz;
    if (a1 * a1 * (r.P + r.EP) * (1.0f + 16.0f * u) <= px.lo2 * (zl * zl) * (1.0f - 16.0f * u)) return 1;
    const float a0 = dz - Edz;
    if ((a0 > 0.0f) & (a0 * a0 * (r.P - r.EP) * (1.0f - 16.0f * u) > px.hi2 * (zh * zh) * (1.0f + 16.0f * u)))
        return 2;
    return -1;
}

// decide32_stage2 without branches (BF): every lane consumes its taps (an early return left tap loads
// in flight past the loop's back edge, and the compiler waited for them where their registers were
// reused) -- the same decisions, as lane masks: valid (decision > 0), consistent (== 1), deferred (< 0)
// (the caller counts them with carry-in adds instead of selecting and re-testing an integer code)
struct Dec32 {
    bool valid, cons, dfr;
};
__device__ __forceinline__ Dec32 decide32_stage2_bf(const Stage32& r, const Pix32& px, uint32_t dmb) {
    constexpr float u = 0x1p-24f;
    const float Ia = r.ab.x, Ib = r.ab.y, Ic = r.cd.x, Id = r.cd.y;
    // the tap test: every tap in (0, depth_max] -- positive floats order like their bits, +0 is the
    // smallest pattern, negatives and NaNs lie above every positive finite pattern
    const uint32_t bA = __float_as_uint(Ia), bB = __float_as_uint(Ib), bC = __float_as_uint(Ic), bD = __float_as_uint(Id);
    const uint32_t tmax = max(max(bA, bB), max(bC, bD)), tmin = min(min(bA, bB), min(bC, bD));
    const bool taps = (tmin != 0u) & (tmax <= dmb);  // (dmb = 0: tmax <= 0 forces tmin = 0)
    // zf by three lerps on the fractions (r.uu, r.vv): within 4u max(I) <= 2^-22 depth_max of the exact
    // interpolation at the float32 uu, vv -- inside the band's 2^-18 depth_max ray-length term, like the
    // reference's own float32 rounding of zt; the weights' dependence on uu, vv is at most the taps'
    // range per unit, so E_dz = E_Z + 2 (E_u + E_v) (max - min) + 8u zf
    const float fu = r.uu, fv = r.vv;
    // (along v first: the row pairs (Ia, Ib), (Ic, Id) as loaded are the packed operands -- no
    // register shuffle of the taps, whose copies at the loop's back edge waited for the loads)
    const float za = __builtin_fmaf(fv, Ic - Ia, Ia), zb = __builtin_fmaf(fv, Id - Ib, Ib);
    const float zf = __builtin_fmaf(fu, zb - za, za);
    const float span = __uint_as_float(tmax) - __uint_as_float(tmin);
    const float eu2 = r.Eu + r.Ev;
    const float Edz = __builtin_fmaf(eu2 + eu2, span, __builtin_fmaf(8.0f * u, zf, r.EZ));
    const float dz = __builtin_fabsf(r.Z - zf);
    const float zl = r.Z - r.EZ, zh = r.Z + r.EZ;
    const float a1 = dz + Edz, a0 = dz - Edz;
    const float Phi = __builtin_fmaf(r.P, r.EP, r.P), Plo = __builtin_fmaf(-r.P, r.EP, r.P);  // (EP: relative)
    const bool in_band_lo = (a1 * a1) * Phi <= px.lo2s * (zl * zl);
    const bool out_band_hi = (a0 > 0.0f) & ((a0 * a0) * Plo > px.hi2s * (zh * zh));
    const bool gt = r.go & taps;
    Dec32 d;
    d.valid = gt & (in_band_lo | out_band_hi);
    d.cons = gt & in_band_lo;
    d.dfr = r.und | (gt & !(in_band_lo | out_band_hi));
    return d;
}

// depth_to_pointcloud_numpy for one pixel: returns 0 when the ref pixel is not in (0, depth_max].
__device__ inline int ref_point(const ConfFrame& fr, int u, int v, float dref, double depth_max, double pw[3]) {
    if (!(dref > 0 && dref <= (float)depth_max)) return 0;
    const double z = (double)dref;
    const double x = div64_by_rn_rcp(((double)u - fr.cx) * z, fr.fx, fr.rfx);
    const double y = div64_by_rn_rcp(((double)v - fr.cy) * z, fr.fy, fr.rfy);
#pragma unroll
    for (int i = 0; i < 3; ++i)
        pw[i] = fr.Tcw[i * 4 + 0] * x + fr.Tcw[i * 4 + 1] * y + fr.Tcw[i * 4 + 2] * z + fr.Tcw[i * 4 + 3];
    return 1;
}

// d2_max: the largest double d2 with (float)sqrt(d2) <= threshold (host, exact); the reference's
// `err <= threshold` on the float32 error map is d2 <= d2_max (sqrt and both roundings monotone).
// STATS: count the pairs per deciding stage into st[4] (pairs, float32 prefilter, float64 filter,
// float64 back-projection) -- mqr_confidence_stats.
// NARROW: a window of at most 32 frames (r <= 15): 32-bit deferral masks.
// W8: held to 8 waves per SIMD (the production instances: BF, !WIDE, !STATS) -- 61 instead of 68
// VGPRs, nothing spilled: 6.84 vs 6.89 ms, 8 alternating processes each,
// profiles/r04_ab_confidence_variants.json (the other instances would spill).  With SLP vectorisation,
// 30 fewer VALU per two pairs but 76 VGPRs / 6 waves, it ran 7.4-7.8 ms: the loop's load latency, not
// only its issue, counts.
template <bool STATS, bool WIDE, bool DIAG = false, bool BF = false, bool NARROW = false, bool W8 = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(W8 ? 8 : 1, 8))) void k_confidence(const float* __restrict__ depths, int N, int H, int W,
                                                    const ConfFrame* __restrict__ fr, int ref_begin, int r,
                                                    double depth_max, double d2_max, double sd,
                                                    double* __restrict__ conf, int32_t* __restrict__ valid,
                                                    unsigned long long* __restrict__ st) {
    const int64_t HW = (int64_t)H * W;
    // (grouping the grid as G reference frames per pixel tile, for L2 reuse of the neighbours' taps,
    // measured no faster for G = 4 ... 64)
    const int rloc = blockIdx.y;
    const int ref = ref_begin + rloc;
#ifndef MQR_CONF_XCD
#define MQR_CONF_XCD 1
#endif
    // XCD bands: workgroups go to the 8 XCDs round-robin, so tile bx of a row of tiles divisible by 8 is
    // remapped for XCD x to work on the x-th eighth of the image -- its neighbour taps then come from
    // one band of each neighbour frame (~25 MB of window / 8), which the XCD's own 4 MB L2 can hold,
    // instead of from the whole frames: 6.48-6.51 vs 7.01-7.10 ms, 6 alternating processes each,
    // identical maps (profiles/r04_ab_confidence_variants.json r04r; MQR_CONF_XCD=0: the plain order)
    unsigned bx = blockIdx.x;
    if (MQR_CONF_XCD && (gridDim.x & 7u) == 0) bx = (bx & 7u) * (gridDim.x >> 3) + (bx >> 3);
    const int64_t p0 = (int64_t)bx * blockDim.x + threadIdx.x;
    if (!STATS && p0 >= HW) return;  // (STATS: the wave reductions below need every lane)
    const int64_t p = p0 < HW ? p0 : HW - 1;
    const int u = (int)(p % W), v = (int)(p / W);
    double pw[3];
    int nv = 0, nc = 0;
    uint32_t n_pairs = 0, n_f32 = 0, n_tail = 0;
    if (p0 < HW && ref_point(fr[ref], u, v, depths[(int64_t)ref * HW + p], depth_max, pw)) {
        const int lo = max(0, ref - r), hi = min(N, ref + r + 1);
        // the consistency band (pixel_decide): the neighbours' largest defect terms, then per pixel
        const double c1 = fr[ref].wc1, c0 = fr[ref].wc0;
        const double pw_norm = sqrt(pw[0] * pw[0] + pw[1] * pw[1] + pw[2] * pw[2]) * (1.0 + 1e-12);
        const double B = c1 * pw_norm + c0;
        const double blo = sd - B, bhi = sd + B;
        const double lo2 = blo > 0 ? blo * blo * (1.0 - 1e-12) : -1.0;
        const double hi2 = bhi * bhi * (1.0 + 1e-12);
        const double zmax = fmin(depth_max, 0x1.fffffffffffffp1023);
        const float dmf = (float)depth_max;
        const uint32_t dmb = dmf > 0.0f ? __float_as_uint(dmf) : 0u;
        const double wm1 = (double)(W - 1), hm1 = (double)(H - 1);
        Pix32 px;
        float mx = 0.0f;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            px.p[i] = (float)pw[i];
            mx = fmaxf(mx, __builtin_fabsf(px.p[i]));
        }
        px.m = mx * (1.0f + 0x1p-22f);
        px.lo2 = lo2 >= 1e-12 ? round_down_f(lo2) : -1.0f;  // (no float32 underflow in the products)
        px.hi2 = round_up_f(hi2);
        px.zlo = round_down_f(zmax);
        px.zhi = round_up_f(zmax);
        px.lo2s = lo2 >= 1e-12 ? round_down_f(lo2 * ((1.0 - 0x1p-20) / (1.0 + 0x1p-20)) * (1.0 - 0x1p-40)) : -1.0f;
        px.hi2s = round_up_f(hi2 * ((1.0 + 0x1p-20) / (1.0 - 0x1p-20)) * (1.0 + 0x1p-40));
        const float wm1f = (float)(W - 1), hm1f = (float)(H - 1);
        // the neighbour loop, pipelined: stage 1 of the next neighbour (its projection, tests and tap
        // loads) runs before stage 2 of the current one, so one pair's tap loads are in flight while
        // the other's are computed; pairs the float32 path cannot decide are collected in `defer`
        // (bit t - lo) and decided by the float64 path after the loop (outside the hot loop's registers)
        // (WIDE: windows of more than 64 frames (r > 31), in chunks of 64 neighbours -- one defer bit each)
        // (one chunk without WIDE: no outer loop, whose back edge made the compiler assume tap loads in
        // flight at the top of the neighbour loop and wait for them)
        auto run_chunk = [&](const int clo, const int chi) {
            auto next_t = [&](int t) {
                for (++t; t < chi; ++t)
                    if (t != ref && fr[t].ok) break;  // the reference frame and frames not ok are skipped
                return t;
            };
            using dmask_t = std::conditional_t<NARROW, uint32_t, uint64_t>;
            dmask_t defer = 0;
            int t = next_t(clo - 1);
            const uint32_t fbytes = 4u * (uint32_t)HW, W4 = 4u * (uint32_t)W;
            auto stage1 = [&](int tt) {
                if constexpr (BF)
                    return decide32_stage1_bf(__builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(depths + (int64_t)tt * HW),
                                                                                (short)0, (int)fbytes, 0x00020000),
                                              W4, fbytes, W, H, fr[tt], px);
                else
                    return decide32_stage1<DIAG>(depths + (int64_t)tt * HW, W, H, wm1f, hm1f, fr[tt], px);
            };
            auto account = [&](const Stage32& st, int tt) {
                bool valid, cons, dfr;
                if constexpr (BF) {
                    const Dec32 d = decide32_stage2_bf(st, px, dmb);
                    valid = d.valid;
                    cons = d.cons;
                    dfr = d.dfr;
                } else {
                    const int dcs = decide32_stage2(st, px, dmb);
                    valid = dcs > 0;
                    cons = dcs == 1;
                    dfr = dcs < 0;
                }
                if (STATS) {
                    ++n_pairs;
                    n_f32 += !dfr;
                }
#if MQR_CONF_BALLOT_DEFER  // (A/B library: the update behind a wave-uniform ballot)
                if (__ballot(dfr))
#endif
                    defer |= (dmask_t)(dfr ? 1u : 0u) << (tt - clo);
                nv += valid;
                nc += cons;
            };
            // unrolled by two with the stages' roles alternating, and stage 1 issued unconditionally (past
            // the last neighbour it re-runs the current one, result unused): a `cur = nxt` copy of the tap
            // registers, or loads issued on only one path, made the compiler wait at the end of every
            // iteration for the loads it had just issued
            if constexpr (!WIDE) {  // the neighbours from the window mask (scalar bit scan)
                uint64_t m = fr[ref].wmask;
                auto pop = [&]() {
                    const int tt = clo + __builtin_ctzll(m);
                    m &= m - 1;
                    return tt;
                };
                if (m) {
                    int ta = pop();
                    Stage32 a = stage1(ta), b;
#pragma clang loop unroll(disable)
                    // (sched_barrier: the scheduler otherwise hoisted the previous pair's stage 2 above the
                    // next pair's loads and waited for its taps at the top of each half)
                    while (true) {
                        const bool more = m != 0;
                        const int tb = more ? pop() : ta;
                        b = stage1(tb);
                        __builtin_amdgcn_sched_barrier(0);
                        account(a, ta);
                        if (!more) break;
                        const bool more2 = m != 0;
                        ta = more2 ? pop() : tb;
                        a = stage1(ta);
                        __builtin_amdgcn_sched_barrier(0);
                        account(b, tb);
                        if (!more2) break;
                    }
                }
            } else if (t < chi) {
                Stage32 a = stage1(t), b;
#pragma clang loop unroll(disable)
                while (true) {
                    const int t2 = next_t(t);
                    b = stage1(t2 < chi ? t2 : t);
                    account(a, t);
                    if (t2 >= chi) break;
                    t = next_t(t2);
                    a = stage1(t < chi ? t : t2);
                    account(b, t2);
                    if (t >= chi) break;
                }
            }
            while (defer) {
                const int td = clo + (NARROW ? __builtin_ctz((uint32_t)defer) : __builtin_ctzll((uint64_t)defer));
                defer &= defer - 1;
                int dcs = pixel_decide(depths + (int64_t)td * HW, W, wm1, hm1, fr[td], pw, zmax, dmf, lo2, hi2, d2_max);
                if (STATS) n_tail += dcs >> 2;
                dcs &= 3;
                nv += dcs != 0;
                nc += dcs == 1;
            }
        };
        if constexpr (WIDE) {
#pragma clang loop unroll(disable)
            for (int clo = lo; clo < hi; clo += 64) run_chunk(clo, min(hi, clo + 64));
        } else {
            run_chunk(lo, hi);
        }
    }
    if (STATS) {
        const uint32_t t[3] = {n_pairs, n_f32, n_tail};
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            uint32_t v = t[i];
            for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
            if ((threadIdx.x & 63) == 0 && v) atomicAdd(&st[i == 0 ? 0 : i == 1 ? 1 : 3], (unsigned long long)v);
        }
    }
    if (p0 >= HW) return;
    const int64_t o = (int64_t)rloc * HW + p;
    valid[o] = nv;
    conf[o] = nv == 0 ? 0.0 : (double)nc / (double)nv;
}

__global__ void k_error_map(const float* __restrict__ refd, const float* __restrict__ tgtd, int H, int W,
                            const ConfFrame* __restrict__ fr, double depth_max, float* out) {
    const int64_t HW = (int64_t)H * W;
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= HW) return;
    double pw[3], d2;
    float e = NAN;
    if (ref_point(fr[0], (int)(p % W), (int)(p / W), refd[p], depth_max, pw) &&
        pixel_error_d2(tgtd, H, W, fr[1], pw, depth_max, &d2))
        e = (float)sqrt(d2);
    out[p] = e;
}

// Self-test of the two quotient paths against IEEE division: mode 0 = div64_core (shared refined
// reciprocal), 1 = div64_by_rn_rcp with y = RN(1/b) computed here by IEEE division.  Pairs from a
// counter-based hash: a uniform in [-a_max, a_max] and b in [b_lo, b_hi] (log-uniform), plus the
// bit-neighbourhood of exact halfway-prone values.  Counts mismatches.
__global__ void k_check_div64(int mode, uint64_t seed, uint64_t count, double a_max, double b_lo, double b_hi,
                              unsigned long long* mismatches, double* first_bad) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    uint64_t h1 = mix64(seed ^ (2 * i + 1)), h2 = mix64(seed + 0x9e3779b97f4a7c15ull * (i + 7));
    const double ua = (double)(h1 >> 11) * 0x1p-53, ub = (double)(h2 >> 11) * 0x1p-53;
    double a = (2.0 * ua - 1.0) * a_max;
    if (h1 & 1) a = __longlong_as_double(__double_as_longlong(a) ^ (h2 & 0xff));  // low-bit perturbation
    const double b = exp2(log2(b_lo) + ub * (log2(b_hi) - log2(b_lo)));
    const double want = a / b;
    double got;
    if (mode == 0) got = div64_core(a, rcp64_refine(b));
    else got = div64_by_rn_rcp(a, b, 1.0 / b);
    if (__double_as_longlong(got) != __double_as_longlong(want)) {
        atomicAdd(mismatches, 1ull);
        first_bad[0] = a;
        first_bad[1] = b;
    }
}

}  // namespace mqr

using namespace mqr;

namespace {
void fill_frame(const float* K, const float* Tcw, const float* Tinv, double sd, int H, int W, float dmf, ConfFrame& f) {
    f.fx = (double)K[0];
    f.fy = (double)K[4];
    f.cx = (double)K[2];
    f.cy = (double)K[5];
    f.ok = 1;
    f.rfx = 1.0 / f.fx;  // correctly rounded (IEEE host division)
    f.rfy = 1.0 / f.fy;
    for (int k = 0; k < 12; ++k) {
        f.Tcw[k] = (double)Tcw[k];
        f.Tinv[k] = Tinv ? (double)Tinv[k] : 0.0;
    }
    // consistency filter terms (pixel_decide): defects of the float32 matrices, in double, with slack
    const double* T = f.Tcw;
    const double a = T[0], b = T[1], c = T[2], d = T[4], e = T[5], g = T[6], h = T[8], i = T[9], j = T[10];
    const double det = a * (e * j - g * i) - b * (d * j - g * h) + c * (d * i - e * h);
    double inv[9] = {(e * j - g * i) / det, (c * i - b * j) / det, (b * g - c * e) / det,
                     (g * h - d * j) / det, (a * j - c * h) / det, (c * d - a * g) / det,
                     (d * i - e * h) / det, (b * h - a * i) / det, (a * e - b * d) / det};
    double dR = 0.0, dT = 0.0, eR = 0.0;
    for (int r = 0; r < 3; ++r) {
        const double ts = -(inv[3 * r] * T[3] + inv[3 * r + 1] * T[7] + inv[3 * r + 2] * T[11]);
        dT += (f.Tinv[4 * r + 3] - ts) * (f.Tinv[4 * r + 3] - ts);
        for (int k = 0; k < 3; ++k) {
            dR += (f.Tinv[4 * r + k] - inv[3 * r + k]) * (f.Tinv[4 * r + k] - inv[3 * r + k]);
            double rtr = 0.0;  // (R^T R)_{rk}
            for (int m = 0; m < 3; ++m) rtr += T[4 * m + r] * T[4 * m + k];
            eR += (rtr - (r == k)) * (rtr - (r == k));
        }
    }
    const bool finite = std::isfinite(det) && det != 0.0 && std::isfinite(dR) && std::isfinite(dT) && std::isfinite(eR);
    dR = std::sqrt(dR) * 1.01 + 1e-12;
    dT = std::sqrt(dT) * 1.01 + 1e-12;
    eR = std::sqrt(eR) * 1.01 + 1e-12;
    // |Z - zf| vs |Z - zt| (pixel_decide's float32 interpolation): 2^-18 depth_max times the longest
    // ray |pt| / Z = sqrt(1 + ((u - cx) / fx)^2 + ((v - cy) / fy)^2) over the image (a corner)
    const double ax = std::max(std::fabs(-f.cx), std::fabs((W - 1) - f.cx)) / std::fabs(f.fx);
    const double ay = std::max(std::fabs(-f.cy), std::fabs((H - 1) - f.cy)) / std::fabs(f.fy);
    const double zterm = 0x1p-18 * (double)dmf * std::sqrt(1.0 + ax * ax + ay * ay) * 1.01;
    // sd NaN (no consistent error possible): the band is irrelevant, every pair takes the exact tail
    const double c1 = dR * (1.0 + eR), c0 = (dT + zterm) * (1.0 + eR) + eR * (sd + 1.0) + 1e-9;
    f.c1 = finite && std::isfinite(c1) ? c1 : INFINITY;
    f.c0 = finite && std::isfinite(c0) ? c0 : INFINITY;
    // float32 prefilter (pixel_decide32): the given float32 entries, and the error bound terms rounded
    // up (8u = 2^-21; a non-finite entry makes them inf / NaN, which sends every pair to float64)
    f.fxf = K[0];
    f.fyf = K[4];
    f.cxf = K[2];
    f.cxu = (float)(std::fabs((double)K[2]) * 0x1p-23 * (1.0 + 0x1p-22));
    f.cyu = (float)(std::fabs((double)K[5]) * 0x1p-23 * (1.0 + 0x1p-22));
    f.cyf = K[5];
    for (int k = 0; k < 12; ++k) f.Tf[k] = Tinv ? Tinv[k] : 0.0f;
    for (int r = 0; r < 3; ++r) {
        const double a = ((double)std::fabs(f.Tf[4 * r]) + std::fabs(f.Tf[4 * r + 1]) + std::fabs(f.Tf[4 * r + 2])) *
                         0x1p-21 * (1.0 + 0x1p-20);
        const double b = (double)std::fabs(f.Tf[4 * r + 3]) * 0x1p-21 * (1.0 + 0x1p-20) + 0x1p-126;
        f.ea[r] = std::nextafter((float)a, INFINITY);
        f.eb[r] = std::nextafter((float)b, INFINITY);
    }
    // (fmax: a NaN entry is dropped, but then Tf holds a NaN and every pair fails); times 1 + 16u rounded
    // up: the slack decide32_stage1_bf's E_u / E_v need for their own roundings, carried by E itself
    // (a larger E is a valid bound wherever E is used)
    f.eam = std::nextafter((float)(std::fmax(std::fmax(f.ea[0], f.ea[1]), f.ea[2]) * (1.0 + 0x1p-20)), INFINITY);
    f.ebm = std::nextafter((float)(std::fmax(std::fmax(f.eb[0], f.eb[1]), f.eb[2]) * (1.0 + 0x1p-20)), INFINITY);
    // RN(8 eam m + 8 ebm) = 8 RN(eam m + ebm) = 8 E (powers of two scale exactly), and with the 1e-6 floor
    // in the addend RN(8 eam m + max(8 ebm, 1e-6)) >= max(8 E, 1e-6): the one-fma test implies the two
    f.eam8 = 8.0f * f.eam;
    f.ebm8 = std::fmax(8.0f * f.ebm, 1e-6f);
}

// Largest double d2 >= 0 with (float)sqrt(d2) <= thr (binary search over the ordered bit patterns
// of non-negative doubles; the host's sqrt and float conversion are IEEE, like the device's).
double d2_threshold(float thr) {
    auto ok = [&](uint64_t bits) {
        double d;
        std::memcpy(&d, &bits, sizeof d);
        return (float)std::sqrt(d) <= thr;
    };
    if (!ok(0)) return -1.0;  // thr < 0 (or NaN): nothing is consistent
    uint64_t lo = 0, hi = 0x7ff0000000000000ull;  // ok(lo); +inf
    if (ok(hi)) return INFINITY;
    while (hi - lo > 1) {
        const uint64_t mid = lo + (hi - lo) / 2;
        if (ok(mid)) lo = mid;
        else hi = mid;
    }
    double d;
    std::memcpy(&d, &lo, sizeof d);
    return d;
}
constexpr int kConfDevices = 64;
struct ConfCache {
    std::mutex mu;
    hipStream_t s = nullptr;
    ConfFrame* dfr = nullptr;  // device frame parameters, grow-only
    ConfFrame* hfr = nullptr;  // pinned staging
    int cap = 0;
    bool stats = false;                 // mqr_confidence_stats: count pairs per deciding stage
    bool diag = false;                  // mqr_confidence_stats enable = 2: no tap loads (timing only)
    bool branchy = false;               // enable = 4: the branchy float32 stages (A/B; 3 = the default)
    unsigned long long* dst = nullptr;  // device counters [4]
    int64_t last[4] = {0, 0, 0, 0};     // pairs, float32 prefilter, float64 filter, float64 back-projection
    // grow-only device staging of host-array calls (uploaded depths; conf + valid before their download):
    // a hipMalloc / hipFree pair of ~240 MB per 64-frame call cost more than the kernel
    void* d_in = nullptr;
    size_t d_in_cap = 0;
    void* d_out = nullptr;
    size_t d_out_cap = 0;
};

int grow(void** p, size_t* cap, size_t want) {
    if (*cap >= want) return 0;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    if (hipMalloc(p, want) != hipSuccess) {
        (void)hipGetLastError();
        return 1;
    }
    *cap = want;
    return 0;
}
ConfCache g_conf_cache[kConfDevices];
}  // namespace

#ifndef MQR_SRC_TAG
#define MQR_SRC_TAG "untagged"
#endif
namespace mqr {
const char* confidence_src_tag() { return MQR_SRC_TAG; }
}  // namespace mqr

extern "C" {

int mqr_confidence(int device, const float* depths, int depth_loc, int N, int H, int W, const float* K,
                   const float* T_cw, const float* T_cw_inv, const uint8_t* frame_ok, int ref_begin, int ref_end,
                   int frame_range, double depth_max, double error_threshold, double* conf, int32_t* valid,
                   int out_loc) {
    MQR_REQUIRE(depths && K && T_cw && T_cw_inv && conf && valid, "null argument");
    MQR_REQUIRE(N > 0 && H > 0 && W > 0, "bad shape");
    MQR_REQUIRE(ref_begin >= 0 && ref_end <= N && ref_begin <= ref_end, "bad reference frame range");
    MQR_REQUIRE(device >= 0 && device < kConfDevices, "bad device");
    MQR_CHECK_HIP(hipSetDevice(device));
    const int nref = ref_end - ref_begin;
    if (nref == 0) return 0;
    const int64_t HW = (int64_t)H * W;
    // (float) threshold: numpy compares the float32 error map against a weak Python float.
    const double d2max = d2_threshold((float)error_threshold);
    const double sd = d2max >= 0 ? std::sqrt(d2max) : NAN;
    // per-device stream and frame-parameter buffers, kept between calls: a stream create / destroy and
    // a hipMalloc / hipFree pair per call (hipFree synchronises the device) cost ~0.5 ms of a 13 ms call
    ConfCache& cc = g_conf_cache[device];
    std::lock_guard<std::mutex> lock(cc.mu);
    if (!cc.s) MQR_CHECK_HIP(hipStreamCreateWithFlags(&cc.s, hipStreamNonBlocking));
    if (cc.cap < N) {
        if (cc.dfr) (void)hipFree(cc.dfr);
        if (cc.hfr) (void)hipHostFree(cc.hfr);
        cc.dfr = nullptr;
        cc.hfr = nullptr;
        cc.cap = 0;
        MQR_CHECK_HIP(hipMalloc(&cc.dfr, sizeof(ConfFrame) * N));
        MQR_CHECK_HIP(hipHostMalloc(&cc.hfr, sizeof(ConfFrame) * N, hipHostMallocDefault));
        cc.cap = N;
    }
    hipStream_t s = cc.s;
    ConfFrame* fr = cc.hfr;
    MQR_CHECK_HIP(hipStreamSynchronize(s));  // the previous call's upload has finished with hfr
    if ((depth_loc == MQR_DEVICE || out_loc == MQR_DEVICE) && order_after_caller(device, s)) return 2;
    for (int i = 0; i < N; ++i) {
        fill_frame(K + 9 * i, T_cw + 16 * i, T_cw_inv + 16 * i, sd, H, W, (float)depth_max, fr[i]);
        fr[i].ok = frame_ok ? (frame_ok[i] ? 1 : 0) : 1;
    }
    for (int i = ref_begin; i < ref_end; ++i) {  // the reference frames' window terms
        const int lo = std::max(0, i - frame_range), hi = std::min(N, i + frame_range + 1);
        double c1 = 0.0, c0 = 0.0;
        uint64_t m = 0;
        for (int t = lo; t < hi; ++t)
            if (t != i && fr[t].ok) {
                c1 = std::fmax(c1, fr[t].c1);
                c0 = std::fmax(c0, fr[t].c0);
                if (t - lo < 64) m |= 1ull << (t - lo);
            }
        fr[i].wc1 = c1;
        fr[i].wc0 = c0;
        fr[i].wmask = m;
    }
    ConfFrame* dfr = cc.dfr;
    float* dd = nullptr;
    double* dconf = conf;
    int32_t* dvalid = valid;
    MQR_CHECK_HIP(hipMemcpyAsync(dfr, fr, sizeof(ConfFrame) * N, hipMemcpyHostToDevice, s));
    const float* dsrc = depths;
    if (depth_loc != MQR_DEVICE) {
        MQR_REQUIRE(grow(&cc.d_in, &cc.d_in_cap, sizeof(float) * N * HW) == 0, "mqr_confidence: device allocation failed");
        dd = static_cast<float*>(cc.d_in);
        if (copy_to_device(device, dd, depths, sizeof(float) * N * HW, s)) return 1;
        dsrc = dd;
    }
    if (out_loc != MQR_DEVICE) {
        const size_t bc = (sizeof(double) * nref * HW + 255) & ~(size_t)255;
        MQR_REQUIRE(grow(&cc.d_out, &cc.d_out_cap, bc + sizeof(int32_t) * nref * HW) == 0,
                    "mqr_confidence: device allocation failed");
        dconf = static_cast<double*>(cc.d_out);
        dvalid = reinterpret_cast<int32_t*>(static_cast<char*>(cc.d_out) + bc);
    }
    const dim3 grid((unsigned)((HW + 255) / 256), nref);
    const bool wide = frame_range > 31;    // a window of more than 64 frames: chunked defer masks
    const bool narrow = frame_range <= 15;  // at most 32 frames: 32-bit defer masks
    // the branch-free float32 stages (default) address the frames with 32-bit byte offsets; the branchy
    // ones (mode 4, the first round-4 form) remain for frames past that and for A/Bs
    const bool bf = !cc.branchy && 4 * (HW + W) < (int64_t{1} << 31);
    auto launch = [&](auto kern, unsigned long long* st) {
        hipLaunchKernelGGL(kern, grid, dim3(256), 0, s, dsrc, N, H, W, dfr, ref_begin, frame_range, depth_max, d2max,
                           sd, dconf, dvalid, st);
    };
    if (cc.stats) {
        if (!cc.dst) MQR_CHECK_HIP(hipMalloc(&cc.dst, 4 * sizeof(unsigned long long)));
        MQR_CHECK_HIP(hipMemsetAsync(cc.dst, 0, 4 * sizeof(unsigned long long), s));
        if (bf)
            wide ? launch(k_confidence<true, true, false, true>, cc.dst)
                 : narrow ? launch(k_confidence<true, false, false, true, true>, cc.dst)
                          : launch(k_confidence<true, false, false, true>, cc.dst);
        else
            wide ? launch(k_confidence<true, true>, cc.dst) : launch(k_confidence<true, false>, cc.dst);
    } else if (cc.diag) {  // timing diagnostics only (wrong results): no tap loads
        launch(k_confidence<false, false, true>, nullptr);
    } else if (bf) {
        wide ? launch(k_confidence<false, true, false, true>, nullptr)
             : narrow ? launch(k_confidence<false, false, false, true, true, true>, nullptr)
                      : launch(k_confidence<false, false, false, true, false, true>, nullptr);
    } else {
        wide ? launch(k_confidence<false, true>, nullptr) : launch(k_confidence<false, false>, nullptr);
    }
    MQR_CHECK_HIP(hipGetLastError());
    if (cc.stats) {
        unsigned long long h[4];
        MQR_CHECK_HIP(hipMemcpyAsync(h, cc.dst, sizeof(h), hipMemcpyDeviceToHost, s));
        MQR_CHECK_HIP(hipStreamSynchronize(s));
        cc.last[0] = (int64_t)h[0];
        cc.last[1] = (int64_t)h[1];
        cc.last[3] = (int64_t)h[3];
        cc.last[2] = cc.last[0] - cc.last[1] - cc.last[3];
    }
    int rc = 0;
    if (out_loc != MQR_DEVICE)
        rc = copy_to_host(device, conf, dconf, sizeof(double) * nref * HW, s) ||
             copy_to_host(device, valid, dvalid, sizeof(int32_t) * nref * HW, s);
    if (!rc) MQR_CHECK_HIP(hipStreamSynchronize(s));
    return rc;
}

int mqr_confidence_stats(int device, int enable, int64_t* last4) {
    MQR_REQUIRE(device >= 0 && device < kConfDevices, "bad device");
    ConfCache& cc = g_conf_cache[device];
    std::lock_guard<std::mutex> lock(cc.mu);
    if (enable >= 0) {
        cc.stats = enable == 1;
        cc.diag = enable == 2;
        cc.branchy = enable == 4;
    }
    if (last4)
        for (int i = 0; i < 4; ++i) last4[i] = cc.last[i];
    return 0;
}

int mqr_check_div64(int device, int mode, uint64_t seed, uint64_t count, double a_max, double b_lo, double b_hi,
                    uint64_t* mismatches, double* first_bad) {
    MQR_REQUIRE(mismatches && first_bad && (mode == 0 || mode == 1) && b_lo > 0 && b_hi >= b_lo, "bad arguments");
    MQR_CHECK_HIP(hipSetDevice(device));
    unsigned long long* dm = nullptr;
    double* db = nullptr;
    MQR_CHECK_HIP(hipMalloc(&dm, sizeof(unsigned long long)));
    MQR_CHECK_HIP(hipMalloc(&db, 2 * sizeof(double)));
    MQR_CHECK_HIP(hipMemset(dm, 0, sizeof(unsigned long long)));
    MQR_CHECK_HIP(hipMemset(db, 0, 2 * sizeof(double)));
    const uint64_t chunk = 1ull << 28;
    for (uint64_t off = 0; off < count; off += chunk) {
        const uint64_t c = std::min<uint64_t>(chunk, count - off);
        hipLaunchKernelGGL(k_check_div64, dim3((unsigned)((c + 255) / 256)), dim3(256), 0, 0, mode, seed + off, c, a_max,
                           b_lo, b_hi, dm, db);
        MQR_CHECK_HIP(hipGetLastError());
    }
    unsigned long long m = 0;
    MQR_CHECK_HIP(hipMemcpy(&m, dm, sizeof m, hipMemcpyDeviceToHost));
    MQR_CHECK_HIP(hipMemcpy(first_bad, db, 2 * sizeof(double), hipMemcpyDeviceToHost));
    (void)hipFree(dm);
    (void)hipFree(db);
    *mismatches = m;
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
    fill_frame(K_ref, T_cw_ref, nullptr, NAN, H, W, 0.f, fr[0]);
    fill_frame(K_tgt, T_cw_tgt, T_cw_inv_tgt, NAN, H, W, 0.f, fr[1]);
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

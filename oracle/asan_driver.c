/* asan_driver.c -- runs every entry point of the CPU oracle (mqr_oracle.c) once on a procedural
 * scene, for the AddressSanitizer / UndefinedBehaviorSanitizer build (sanitizers on
 * the CPU restatement).  TEST INFRASTRUCTURE ONLY.  `make -C oracle asan` builds and runs it; a
 * memory error or undefined behaviour aborts with a non-zero exit.
 *
 * Scene: a sphere of radius 0.5 m at the origin seen from 8 cameras on a 1.5 m ring (the C1
 * geometry) at 80 x 60, 2 cm voxels (pool growth from capacity 4), R = 16 and 8;
 * touch + integrate per frame, export / import, point and mesh extraction, confidence and
 * pixel-error maps, ray casting of the extracted mesh. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct orc_vbg orc_vbg;
orc_vbg* orc_vbg_create(float voxel_size, int R, int64_t capacity);
void orc_vbg_destroy(orc_vbg* v);
int64_t orc_vbg_size(const orc_vbg* v);
void orc_set_threads(int n);
int orc_touch(const float* depth, int H, int W, const double* K, const double* T, float voxel_size, int R,
              float depth_scale, float depth_max, float trunc_mult, int32_t* keys_out, int64_t* n_out);
int orc_integrate(orc_vbg* v, const int32_t* keys, int64_t n, const float* depth, int H, int W, const double* K,
                  const double* T, float depth_scale, float depth_max, float trunc_mult);
int orc_export(const orc_vbg* v, int32_t* keys, float* tsdf, float* weight);
int orc_import(orc_vbg* v, const int32_t* keys, const float* tsdf, const float* weight, int64_t n);
int64_t orc_extract_points(const orc_vbg* v, float thr, float** pos_out, float** nrm_out);
int64_t orc_extract_mesh(const orc_vbg* v, float thr, float** vtx_out, float** nrm_out, int32_t** tri_out,
                         int64_t* ntri_out);
void orc_free(void* p);
int orc_pixel_error_map(const float* ref_depth, const float* tgt_depth, int H, int W, const float* Kr,
                        const float* Kt, const float* Tr, const float* Tt_inv, const float* Tt, double depth_max,
                        float* err_out);
int orc_confidence(const float* depths, const uint8_t* frame_valid, const float* K, const float* Tcw,
                   const float* Tcw_inv, int N, int H, int W, int ref, int r, double depth_max, double err_thr,
                   double* conf, int32_t* valid);
int orc_raycast(const float* V, int64_t nv, const int32_t* T, int64_t nt, const float* rays, int64_t nrays,
                float* t_hit, int32_t* prim);

enum { N = 8, H = 60, W = 80 };

/* camera -> world rotation (columns right, down, forward) and eye of camera i on the ring */
static void pose(int i, double Rcw[9], double eye[3]) {
    const double a = 2.0 * 3.14159265358979323846 * i / N;
    eye[0] = 1.5 * cos(a), eye[1] = 0.2, eye[2] = 1.5 * sin(a);
    double f[3] = {-eye[0], -eye[1], -eye[2]}, up[3] = {0, 1, 0}, r[3], d[3];
    double nf = sqrt(f[0] * f[0] + f[1] * f[1] + f[2] * f[2]);
    for (int k = 0; k < 3; ++k) f[k] /= nf;
    r[0] = f[1] * up[2] - f[2] * up[1], r[1] = f[2] * up[0] - f[0] * up[2], r[2] = f[0] * up[1] - f[1] * up[0];
    double nr = sqrt(r[0] * r[0] + r[1] * r[1] + r[2] * r[2]);
    for (int k = 0; k < 3; ++k) r[k] /= nr;
    d[0] = f[1] * r[2] - f[2] * r[1], d[1] = f[2] * r[0] - f[0] * r[2], d[2] = f[0] * r[1] - f[1] * r[0];
    for (int k = 0; k < 3; ++k) Rcw[3 * k] = r[k], Rcw[3 * k + 1] = d[k], Rcw[3 * k + 2] = f[k];
}

int main(void) {
    orc_set_threads(2);
    static float depth[N][H * W];
    double K[9] = {65.0, 0, 39.5, 0, 65.0, 29.5, 0, 0, 1}, T[N][16];
    float K32[N][9], Tcw32[N][16], Tinv32[N][16];
    for (int i = 0; i < N; ++i) {
        double R_[9], e[3];
        pose(i, R_, e);
        /* world -> camera: [R^T | -R^T e] */
        memset(T[i], 0, sizeof(T[i]));
        for (int a = 0; a < 3; ++a) {
            for (int b = 0; b < 3; ++b) T[i][4 * a + b] = R_[3 * b + a];
            T[i][4 * a + 3] = -(R_[a] * e[0] + R_[3 + a] * e[1] + R_[6 + a] * e[2]);
        }
        T[i][15] = 1.0;
        for (int k = 0; k < 9; ++k) K32[i][k] = (float)K[k];
        for (int k = 0; k < 16; ++k) Tinv32[i][k] = (float)T[i][k];
        memset(Tcw32[i], 0, sizeof(Tcw32[i]));
        for (int a = 0; a < 3; ++a) {
            for (int b = 0; b < 3; ++b) Tcw32[i][4 * a + b] = (float)R_[3 * a + b];
            Tcw32[i][4 * a + 3] = (float)e[a];
        }
        Tcw32[i][15] = 1.0f;
        for (int v = 0; v < H; ++v)
            for (int u = 0; u < W; ++u) {  /* ray-sphere hit depth along the camera z axis */
                double dc[3] = {(u - K[2]) / K[0], (v - K[5]) / K[4], 1.0}, dw[3];
                for (int a = 0; a < 3; ++a) dw[a] = R_[3 * a] * dc[0] + R_[3 * a + 1] * dc[1] + R_[3 * a + 2] * dc[2];
                double A = dw[0] * dw[0] + dw[1] * dw[1] + dw[2] * dw[2];
                double B = 2 * (dw[0] * e[0] + dw[1] * e[1] + dw[2] * e[2]);
                double C = e[0] * e[0] + e[1] * e[1] + e[2] * e[2] - 0.25;
                double disc = B * B - 4 * A * C;
                depth[i][v * W + u] = disc >= 0 ? (float)((-B - sqrt(disc)) / (2 * A)) : 0.0f;
            }
    }
    int32_t* keys = malloc(sizeof(int32_t) * 3 * 4 * (H / 4) * (W / 4));
    for (int R = 16; R >= 8; R /= 2) {
        orc_vbg* v = orc_vbg_create(0.02f, R, 4);
        for (int i = 0; i < N; ++i) {
            int64_t n = 0;
            if (orc_touch(depth[i], H, W, K, T[i], 0.02f, R, 1.0f, 3.0f, 4.0f, keys, &n)) return 1;
            if (orc_integrate(v, keys, n, depth[i], H, W, K, T[i], 1.0f, 3.0f, 4.0f)) return 1;
        }
        const int64_t nb = orc_vbg_size(v), R3 = (int64_t)R * R * R;
        int32_t* bk = malloc(sizeof(int32_t) * 3 * nb);
        float* ts = malloc(sizeof(float) * nb * R3);
        float* wt = malloc(sizeof(float) * nb * R3);
        orc_export(v, bk, ts, wt);
        orc_vbg* v2 = orc_vbg_create(0.02f, R, 1);
        if (orc_import(v2, bk, ts, wt, nb)) return 1;
        float *pp, *pn, *mv, *mn;
        int32_t* mt;
        int64_t nt = 0;
        const int64_t np = orc_extract_points(v2, 1.5f, &pp, &pn);
        const int64_t nv = orc_extract_mesh(v2, 1.5f, &mv, &mn, &mt, &nt);
        printf("R=%d blocks=%lld points=%lld vertices=%lld triangles=%lld\n", R, (long long)nb, (long long)np,
               (long long)nv, (long long)nt);
        if (R == 16 && nt > 0) {  /* cast the camera-0 rays at the extracted mesh */
            float* rays = malloc(sizeof(float) * 6 * H * W);
            float* th = malloc(sizeof(float) * H * W);
            int32_t* pr = malloc(sizeof(int32_t) * H * W);
            for (int p = 0; p < H * W; ++p) {
                const float dc[3] = {(float)(((p % W) - K[2]) / K[0]), (float)(((p / W) - K[5]) / K[4]), 1.0f};
                for (int a = 0; a < 3; ++a) {
                    rays[6 * p + a] = Tcw32[0][4 * a + 3];
                    rays[6 * p + 3 + a] = Tcw32[0][4 * a] * dc[0] + Tcw32[0][4 * a + 1] * dc[1] + Tcw32[0][4 * a + 2] * dc[2];
                }
            }
            orc_raycast(mv, nv, mt, nt, rays, H * W, th, pr);
            free(rays), free(th), free(pr);
        }
        orc_free(pp), orc_free(pn), orc_free(mv), orc_free(mn), orc_free(mt);
        free(bk), free(ts), free(wt);
        orc_vbg_destroy(v2);
        orc_vbg_destroy(v);
    }
    free(keys);
    static double conf[H * W];
    static int32_t valid[H * W];
    static float err[H * W];
    uint8_t ok[N] = {1, 1, 0, 1, 1, 1, 1, 1};
    for (int ref = 0; ref < N; ref += 3)
        orc_confidence(&depth[0][0], ok, &K32[0][0], &Tcw32[0][0], &Tinv32[0][0], N, H, W, ref, 2, 3.0, 0.05, conf,
                       valid);
    orc_pixel_error_map(depth[0], depth[1], H, W, K32[0], K32[1], Tcw32[0], Tinv32[1], Tcw32[1], 3.0, err);
    int64_t nval = 0;
    for (int p = 0; p < H * W; ++p) nval += valid[p];
    printf("confidence: %lld valid neighbour samples at the last reference frame\nasan driver ok\n", (long long)nval);
    return 0;
}

// What does the first large device -> host copy of a process pay for?  (tools/d2h_probe.py: the first
// 48 MB mqr_memcpy took 46.6 ms, the second 1.6 ms.)  After the context exists (hipMalloc + one kernel),
// times each set-up step the first round-5 d2h_parallel performed on its first call: stream creation, pinned staging
// allocation (8 x 8 MB, or one 64 MB block), event creation, and the first D2H copy on each new stream.
// One JSON line.   hipcc --offload-arch=gfx950 -O2 -o tools/_ab/d2h_setup_probe tools/d2h_setup_probe.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

static double ms_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

__global__ void k_nop(int* p) {
    if (p && threadIdx.x == 1024) p[0] = 0;
}

int main() {
    using clk = std::chrono::steady_clock;
    CK(hipSetDevice(0));
    char* d;
    CK(hipMalloc(&d, size_t(64) << 20));
    k_nop<<<1, 64>>>(nullptr);
    CK(hipDeviceSynchronize());
    auto t = clk::now();
    hipStream_t s[4];
    for (auto& x : s) CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
    double streams = ms_since(t);
    t = clk::now();
    void* b8[8];
    for (auto& x : b8) CK(hipHostMalloc(&x, size_t(8) << 20, hipHostMallocDefault));
    double pin8 = ms_since(t);
    t = clk::now();
    void* b64;
    CK(hipHostMalloc(&b64, size_t(64) << 20, hipHostMallocDefault));
    double pin64 = ms_since(t);
    t = clk::now();
    void* b64nc;
    CK(hipHostMalloc(&b64nc, size_t(64) << 20, hipHostMallocNonCoherent));
    double pin64nc = ms_since(t);
    t = clk::now();
    hipEvent_t ev[8];
    for (auto& x : ev) CK(hipEventCreateWithFlags(&x, hipEventDisableTiming));
    double events = ms_since(t);
    double first_copy[4], second_copy[4];
    for (int i = 0; i < 4; ++i) {
        t = clk::now();
        CK(hipMemcpyAsync(b8[2 * i], d, size_t(8) << 20, hipMemcpyDeviceToHost, s[i]));
        CK(hipStreamSynchronize(s[i]));
        first_copy[i] = ms_since(t);
        t = clk::now();
        CK(hipMemcpyAsync(b8[2 * i + 1], d, size_t(8) << 20, hipMemcpyDeviceToHost, s[i]));
        CK(hipStreamSynchronize(s[i]));
        second_copy[i] = ms_since(t);
    }
    t = clk::now();
    CK(hipMemcpy(b64, d, size_t(64) << 20, hipMemcpyDeviceToHost));
    double copy64 = ms_since(t);
    t = clk::now();
    CK(hipMemcpy(b64nc, d, size_t(64) << 20, hipMemcpyDeviceToHost));
    double copy64nc = ms_since(t);
    printf("{\"streams_x4_ms\": %.3f, \"hostmalloc_8x8mb_ms\": %.3f, \"hostmalloc_64mb_ms\": %.3f, "
           "\"hostmalloc_64mb_noncoherent_ms\": %.3f, \"events_x8_ms\": %.3f, "
           "\"first_8mb_copy_per_new_stream_ms\": [%.3f, %.3f, %.3f, %.3f], "
           "\"second_8mb_copy_ms\": [%.3f, %.3f, %.3f, %.3f], \"copy_64mb_ms\": %.3f, \"copy_64mb_noncoherent_ms\": %.3f}\n",
           streams, pin8, pin64, pin64nc, events, first_copy[0], first_copy[1], first_copy[2], first_copy[3],
           second_copy[0], second_copy[1], second_copy[2], second_copy[3], copy64, copy64nc);
    return 0;
}

// Device -> pageable-host copy designs for the C5 mesh (~1 GB): which one makes a fresh host array
// hold the device bytes fastest?  Standalone (no libmqr), one JSON line per design:
//   pinned      hipMemcpy into hipHostMalloc memory (the DMA ceiling)
//   staged:T    round 5's mqr d2h_parallel shape: T threads, 2 x 8 MB pinned chunks each
//   touch:P+staged:T   P threads first-touch the destination (one byte per 4 KiB), then staged:T
//   register:P  P threads first-touch, hipHostRegister, one hipMemcpy straight into it, unregister
//   kernel_pinned       a copy kernel storing into hipHostMalloc memory (instead of the SDMA engine)
//   kernel_register:P   P threads first-touch, hipHostRegister (mapped), the copy kernel stores straight
//                       into the destination, unregister
// The destination is a fresh 2 MiB-aligned MADV_HUGEPAGE mapping each time (what numpy's allocator
// hands out for large arrays on this host: THP "madvise").
//   hipcc --offload-arch=gfx950 -O2 -o tools/_ab/d2h_modes tools/d2h_modes.hip -lpthread
#include <hip/hip_runtime.h>
#include <sys/mman.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

// grid-stride 16-byte copy; the stores go to host memory over the fabric (vector stores)
__global__ __launch_bounds__(256) void k_copy16(uint4* __restrict__ dst, const uint4* __restrict__ src, size_t n16) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) dst[i] = src[i];
}

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct Fresh {
    char* base = nullptr;
    char* p = nullptr;
    size_t n = 0, map = 0;
    explicit Fresh(size_t bytes) : n(bytes), map(bytes + (2u << 20)) {
        base = (char*)mmap(nullptr, map, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        if (base == MAP_FAILED) { perror("mmap"); exit(1); }
        p = (char*)(((uintptr_t)base + (2u << 20) - 1) & ~(uintptr_t)((2u << 20) - 1));
        madvise(p, n, MADV_HUGEPAGE);
    }
    ~Fresh() { munmap(base, map); }
};

static void par_touch(char* p, size_t n, int P) {
    std::vector<std::thread> th;
    size_t per = ((n / P) + 4095) & ~size_t(4095);
    for (int i = 0; i < P; ++i)
        th.emplace_back([=] {
            size_t lo = (size_t)i * per, hi = std::min(n, lo + per);
            for (size_t o = lo; o < hi; o += 4096) p[o] = 0;
        });
    for (auto& t : th) t.join();
}

struct Stage {
    hipStream_t s;
    void* buf[2];
    hipEvent_t ev[2];
};

static void staged(int dev, char* dst, const char* src, size_t bytes, int T, size_t chunk, std::vector<Stage>& st) {
    size_t nchunks = (bytes + chunk - 1) / chunk;
    auto work = [&](int t) {
        CK(hipSetDevice(dev));
        Stage& S = st[t];
        auto len = [&](size_t k) { return std::min(chunk, bytes - k * chunk); };
        auto issue = [&](size_t k, int b) {
            CK(hipMemcpyAsync(S.buf[b], src + k * chunk, len(k), hipMemcpyDeviceToHost, S.s));
            CK(hipEventRecord(S.ev[b], S.s));
        };
        int b = 0;
        if ((size_t)t < nchunks) issue(t, 0);
        for (size_t k = t; k < nchunks; k += T) {
            if (k + T < nchunks) issue(k + T, b ^ 1);
            CK(hipEventSynchronize(S.ev[b]));
            memcpy(dst + k * chunk, S.buf[b], len(k));
            b ^= 1;
        }
        CK(hipStreamSynchronize(S.s));
    };
    std::vector<std::thread> th;
    for (int t = 1; t < T; ++t) th.emplace_back(work, t);
    work(0);
    for (auto& x : th) x.join();
}

int main(int argc, char** argv) {
    const size_t bytes = argc > 1 ? strtoull(argv[1], nullptr, 10) : (size_t(1) << 30);
    const int dev = 0;
    CK(hipSetDevice(dev));
    char* d;
    CK(hipMalloc(&d, bytes));
    CK(hipMemset(d, 0x5a, bytes));
    CK(hipDeviceSynchronize());
    auto gbs = [&](double s) { return bytes / s / 1e9; };
    auto check = [&](const char* h) {
        for (size_t o = 0; o < bytes; o += 1 << 20)
            if ((unsigned char)h[o] != 0x5a) return false;
        return (unsigned char)h[bytes - 1] == 0x5a;
    };
    std::vector<Stage> st(16);
    for (auto& S : st) {
        CK(hipStreamCreateWithFlags(&S.s, hipStreamNonBlocking));
        for (int b = 0; b < 2; ++b) {
            CK(hipHostMalloc(&S.buf[b], size_t(32) << 20, hipHostMallocDefault));
            CK(hipEventCreateWithFlags(&S.ev[b], hipEventDisableTiming));
        }
    }
    {
        char* pin;
        CK(hipHostMalloc((void**)&pin, bytes, hipHostMallocDefault));
        double best = 1e9;
        for (int r = 0; r < 3; ++r) {
            double t0 = now();
            CK(hipMemcpy(pin, d, bytes, hipMemcpyDeviceToHost));
            best = std::min(best, now() - t0);
        }
        printf("{\"design\": \"pinned\", \"gbs\": %.2f, \"ms\": %.2f, \"ok\": %s}\n", gbs(best), 1e3 * best,
               check(pin) ? "true" : "false");
        CK(hipHostFree(pin));
    }
    for (int grid : {256, 1024, 4096}) {
        char* pin;
        CK(hipHostMalloc((void**)&pin, bytes, hipHostMallocDefault));
        char* dp;
        CK(hipHostGetDevicePointer((void**)&dp, pin, 0));
        double best = 1e9;
        for (int r = 0; r < 3; ++r) {
            double t0 = now();
            k_copy16<<<grid, 256>>>((uint4*)dp, (const uint4*)d, bytes / 16);
            CK(hipDeviceSynchronize());
            best = std::min(best, now() - t0);
        }
        printf("{\"design\": \"kernel_pinned\", \"grid\": %d, \"gbs\": %.2f, \"ms\": %.2f, \"ok\": %s}\n", grid,
               gbs(best), 1e3 * best, check(pin) ? "true" : "false");
        fflush(stdout);
        CK(hipHostFree(pin));
    }
    for (int grid : {1024, 4096}) {
        Fresh f(bytes);
        double t0 = now();
        par_touch(f.p, bytes, 16);
        double t1 = now();
        CK(hipHostRegister(f.p, bytes, hipHostRegisterMapped));
        char* dp;
        CK(hipHostGetDevicePointer((void**)&dp, f.p, 0));
        double t2 = now();
        k_copy16<<<grid, 256>>>((uint4*)dp, (const uint4*)d, bytes / 16);
        CK(hipDeviceSynchronize());
        double t3 = now();
        CK(hipHostUnregister(f.p));
        double t4 = now();
        printf("{\"design\": \"kernel_register\", \"grid\": %d, \"touch_threads\": 16, \"gbs\": %.2f, \"ms\": %.2f, "
               "\"touch_ms\": %.2f, \"register_ms\": %.2f, \"copy_ms\": %.2f, \"unregister_ms\": %.2f, \"ok\": %s}\n",
               grid, gbs(t4 - t0), 1e3 * (t4 - t0), 1e3 * (t1 - t0), 1e3 * (t2 - t1), 1e3 * (t3 - t2), 1e3 * (t4 - t3),
               check(f.p) ? "true" : "false");
        fflush(stdout);
    }
    const int Ts[] = {1, 2, 4, 8};
    const size_t chunks[] = {size_t(8) << 20, size_t(32) << 20};
    for (size_t chunk : chunks)
        for (int T : Ts)
            for (int P : {0, 16}) {
                Fresh f(bytes);
                double t0 = now();
                if (P) par_touch(f.p, bytes, P);
                double t1 = now();
                staged(dev, f.p, d, bytes, T, chunk, st);
                double t2 = now();
                printf("{\"design\": \"%sstaged\", \"threads\": %d, \"chunk_mb\": %zu, \"touch_threads\": %d, "
                       "\"gbs\": %.2f, \"ms\": %.2f, \"touch_ms\": %.2f, \"ok\": %s}\n",
                       P ? "touch+" : "", T, chunk >> 20, P, gbs(t2 - t0), 1e3 * (t2 - t0), 1e3 * (t1 - t0),
                       check(f.p) ? "true" : "false");
                fflush(stdout);
            }
    for (int P : {1, 8, 16}) {
        Fresh f(bytes);
        double t0 = now();
        par_touch(f.p, bytes, P);
        double t1 = now();
        hipError_t e = hipHostRegister(f.p, bytes, hipHostRegisterDefault);
        double t2 = now();
        if (e != hipSuccess) {
            printf("{\"design\": \"register\", \"touch_threads\": %d, \"error\": \"%s\"}\n", P, hipGetErrorString(e));
            (void)hipGetLastError();
            continue;
        }
        CK(hipMemcpy(f.p, d, bytes, hipMemcpyDeviceToHost));
        double t3 = now();
        CK(hipHostUnregister(f.p));
        double t4 = now();
        printf("{\"design\": \"register\", \"touch_threads\": %d, \"gbs\": %.2f, \"ms\": %.2f, \"touch_ms\": %.2f, "
               "\"register_ms\": %.2f, \"copy_ms\": %.2f, \"unregister_ms\": %.2f, \"ok\": %s}\n",
               P, gbs(t4 - t0), 1e3 * (t4 - t0), 1e3 * (t1 - t0), 1e3 * (t2 - t1), 1e3 * (t3 - t2),
               1e3 * (t4 - t3), check(f.p) ? "true" : "false");
        fflush(stdout);
    }
    return 0;
}

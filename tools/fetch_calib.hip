// fetch_calib -- known-byte read kernels for calibrating the L2 -> fabric read counters on gfx950.
//
// FETCH_SIZE (rocprofv3) = 128 TCC_BUBBLE + 64 (TCC_EA0_RDREQ - TCC_BUBBLE - TCC_EA0_RDREQ_32B) +
// 32 TCC_EA0_RDREQ_32B bytes (counter_defs.yaml).  It reads exactly half of a wide streaming read on
// gfx950 (MI355X_MICROARCH.md, HBM), and the integrate kernel's depth reads are 4-byte gathers, whose
// request widths nobody has measured.  Each kernel here reads a region that no earlier kernel left
// in L2 or the Infinity Cache (a 512 MiB streaming pass over an unrelated region runs before each),
// with a known number of distinct lines:
//   stream      16 B per lane, coalesced:           every byte of 512 MiB
//   gather_line one 4-byte word per 128-B line:      4 Mi lines, random order
//   gather_half one 4-byte word per 64-B half line:  8 Mi halves (both halves of every line), random
//   gather_32   one 4-byte word per 32-B sector:     16 Mi sectors (all four of every line), random
//   gather_row  64 lanes gather 4-byte words spread over one 2.5 KiB image row (integrate-like):
//               every line of 512 MiB read, each line by ~8 lanes of one wave
// Output: one JSON line per kernel (name, distinct lines, bytes if lines were fetched whole, ms).
// tools/pmc_calib.sh collects the counters over this program and the integrate workload.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                              \
        }                                                                              \
    } while (0)

constexpr uint64_t kRegion = 512ull << 20;  // bytes per region
constexpr int kRegions = 6;                 // flush, stream, line, half, sector, row

__global__ __launch_bounds__(256) void k_cal_stream(const float4* __restrict__ p, uint64_t n, float* __restrict__ out) {
    float acc = 0.f;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        const float4 v = p[i];
        acc += v.x + v.y + v.z + v.w;
    }
    if (acc == 1.2345f) out[blockIdx.x] = acc;  // never true for zeroed data: keeps the loads live
}

// One 4-byte word at unit index perm(i) * stride_words, perm(i) = (i * kOdd) mod units (units a power
// of two: a permutation), for i in [0, units).
__global__ __launch_bounds__(256) void k_cal_gather(const float* __restrict__ p, uint64_t units, int stride_words,
                                                    float* __restrict__ out) {
    constexpr uint64_t kOdd = 0x9E3779B1ull;
    float acc = 0.f;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < units; i += (uint64_t)gridDim.x * 256) {
        const uint64_t u = (i * kOdd) & (units - 1);
        acc += p[u * (uint64_t)stride_words];
    }
    if (acc == 1.2345f) out[blockIdx.x] = acc;
}

// Integrate-like: wave w takes image row r = perm(w) of a 640-float-wide "frame" array and its 64
// lanes read columns 10 * lane (a 2.5 KiB row, every 128-B line hit by 3-4 lanes); 8 passes per row
// offset the columns so that every word of the row is read once.
__global__ __launch_bounds__(256) void k_cal_row(const float* __restrict__ p, uint64_t rows, float* __restrict__ out) {
    constexpr uint64_t kOdd = 0x9E3779B1ull;
    constexpr int kW = 640;
    const int lane = threadIdx.x & 63;
    float acc = 0.f;
    for (uint64_t w = blockIdx.x * 4ull + (threadIdx.x >> 6); w < rows; w += (uint64_t)gridDim.x * 4) {
        const uint64_t r = (w * kOdd) % rows;
        const float* row = p + r * kW;
#pragma unroll
        for (int k = 0; k < 10; ++k) acc += row[10 * lane + k];
    }
    if (acc == 1.2345f) out[blockIdx.x] = acc;
}

int main() {
    float* buf = nullptr;
    float* sink = nullptr;
    CK(hipMalloc(&buf, kRegion * kRegions));
    CK(hipMalloc(&sink, 1 << 20));
    CK(hipMemset(buf, 0, kRegion * kRegions));
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto region = [&](int r) { return reinterpret_cast<char*>(buf) + (uint64_t)r * kRegion; };
    auto flush = [&]() {
        hipLaunchKernelGGL(k_cal_stream, dim3(8192), dim3(256), 0, 0, reinterpret_cast<const float4*>(region(0)),
                           kRegion / 16, sink);
        CK(hipGetLastError());
    };
    auto timed = [&](const char* name, uint64_t lines, auto launch) {
        flush();
        CK(hipEventRecord(e0, 0));
        launch();
        CK(hipGetLastError());
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        std::printf("{\"kernel\": \"%s\", \"distinct_lines\": %llu, \"line_bytes\": %llu, \"ms\": %.4f}\n", name,
                    (unsigned long long)lines, (unsigned long long)(lines * 128), ms);
    };
    for (int rep = 0; rep < 2; ++rep) {  // rep 0 warms the code objects; both are recorded
        timed("stream", kRegion / 128, [&] {
            hipLaunchKernelGGL(k_cal_stream, dim3(8192), dim3(256), 0, 0,
                               reinterpret_cast<const float4*>(region(1)), kRegion / 16, sink);
        });
        timed("gather_line", kRegion / 128, [&] {
            hipLaunchKernelGGL(k_cal_gather, dim3(8192), dim3(256), 0, 0, reinterpret_cast<const float*>(region(2)),
                               kRegion / 128, 32, sink);
        });
        timed("gather_half", kRegion / 128, [&] {
            hipLaunchKernelGGL(k_cal_gather, dim3(8192), dim3(256), 0, 0, reinterpret_cast<const float*>(region(3)),
                               kRegion / 64, 16, sink);
        });
        timed("gather_32", kRegion / 128, [&] {
            hipLaunchKernelGGL(k_cal_gather, dim3(8192), dim3(256), 0, 0, reinterpret_cast<const float*>(region(4)),
                               kRegion / 32, 8, sink);
        });
        const uint64_t rows = kRegion / (640 * 4);
        timed("gather_row", rows * 640 * 4 / 128, [&] {
            hipLaunchKernelGGL(k_cal_row, dim3(4096), dim3(256), 0, 0, reinterpret_cast<const float*>(region(5)), rows,
                               sink);
        });
    }
    CK(hipFree(buf));
    CK(hipFree(sink));
    return 0;
}

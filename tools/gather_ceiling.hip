// gather_ceiling -- throughput of 4-byte depth gathers on MI355X, per lane pattern (diagnostic tool;
// no part of the library).  Every thread issues ITERS x 8 raw-buffer dword loads from a 640 x 480
// float frame (1.2 MB: L2-resident, like the integrate kernel's depth frames) and sums them; the
// launch has 8 waves per SIMD on every CU.  Patterns (lane l of a wave, load k):
//   same         all lanes one pixel
//   coalesced    64 consecutive pixels
//   brick        the integrate kernel's brick map: lane (x, y, z) = (l % 8, l / 8 % 2, l / 16) ->
//                pixel (c + 1.3 x + 0.4 z, r + 1.3 y + 0.3 z) -- ~6 distinct 128-byte lines per load
//   brick_even   brick, odd lanes masked off (exec): does the cost follow lanes or instructions?
//   brick_x4     brick lanes, 16-byte loads (each lane reads its pixel's aligned 16-byte window)
//   brick_x2     brick lanes, 8-byte loads (each lane reads its pixel's aligned 8-byte window)
//   brick_x4_lds brick lanes, 16-byte windows by LDS-DMA (global_load_lds_dwordx4: lane i's window
//                lands at the wave's LDS base + 16 i), then each lane reads its dword from LDS
//   window       random pixels of a 64 x 16 window
//   frame        random pixels of the whole frame
// The window origin moves every iteration, so L1 reuse stays what the integrate kernel sees.
// Prints one JSON line per pattern: ns per gather instruction per CU (the launch time divided by
// the gather instructions one CU issued) and lanes per ns per CU.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));           \
            exit(1);                                                                            \
        }                                                                                       \
    } while (0)

constexpr int W = 640, H = 480, ITERS = 256, NT = 512;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}

template <int P>
__global__ __launch_bounds__(NT) void k_gather(const float* __restrict__ frame, float* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[P == 8 ? NT / 64 * 8 * 256 : 1];  // 8 KB per wave
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(frame), (short)0, W * H * 4, 0x00020000);
    const int l = threadIdx.x & 63;
    const uint32_t wave = (blockIdx.x * NT + threadIdx.x) >> 6;
    int dx[8], dy[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int x = l & 7, y = (l >> 3) & 1, z = l >> 4;
        switch (P) {
            case 0: dx[k] = 0; dy[k] = 2 * k; break;
            case 1: dx[k] = l; dy[k] = 2 * k; break;
            case 2: case 3: case 4: case 7: case 8:
                dx[k] = (13 * x + 4 * z) / 10 + 3 * (k & 3);
                dy[k] = (13 * y + 3 * z) / 10 + 11 * (k >> 2);
                break;
            case 5: {
                const uint32_t h = hash32(wave * 577 + l * 8 + k);
                dx[k] = h & 63;
                dy[k] = (h >> 6) & 15;
                break;
            }
            default: {
                const uint32_t h = hash32(wave * 577 + l * 8 + k);
                dx[k] = h % 560;
                dy[k] = (h >> 12) % 400;
            }
        }
    }
    float acc = 0.f;
    if (P == 3 && (l & 1)) return;
    for (int it = 0; it < ITERS; ++it) {
        const uint32_t h = hash32(wave * 131 + it);
        const int c = P == 6 ? (int)(h % 80) : (int)(h % (W - 80)), r = P == 6 ? (int)((h >> 10) % 80) : (int)((h >> 10) % (H - 48));
        float v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t off = 4u * (uint32_t)((r + dy[k]) * W + c + dx[k]);
            if (P == 4) {
                const u32x4 q = __builtin_amdgcn_raw_buffer_load_b128(rs, off & ~15u, 0, 0);
                v[k] = __uint_as_float(q.x) + __uint_as_float(q.w);
            } else if (P == 7) {
                const uint2 q = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(rs, off & ~7u, 0, 0));
                v[k] = __uint_as_float((off & 4u) ? q.y : q.x);
            } else if (P == 8) {
                uint32_t* base = lds + (threadIdx.x >> 6) * 8 * 256 + k * 256;  // wave-uniform
                __builtin_amdgcn_global_load_lds(reinterpret_cast<const char*>(frame) + (off & ~15u), base, 16, 0, 0);
                v[k] = 0.f;
            } else {
                v[k] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0));
            }
        }
        if (P == 8) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const uint32_t off = 4u * (uint32_t)((r + dy[k]) * W + c + dx[k]);
                v[k] = __uint_as_float(lds[(threadIdx.x >> 6) * 8 * 256 + k * 256 + l * 4 + ((off >> 2) & 3u)]);
            }
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) acc += v[k];
    }
    out[blockIdx.x * NT + threadIdx.x] = acc;
}

template <int P>
static void run(const char* name, const float* d_frame, float* d_out, int grid, int cus) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(k_gather<P>, dim3(grid), dim3(NT), 0, 0, d_frame, d_out);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    std::vector<float> ms;
    for (int r = 0; r < 7; ++r) {
        CK(hipEventRecord(a, 0));
        hipLaunchKernelGGL(k_gather<P>, dim3(grid), dim3(NT), 0, 0, d_frame, d_out);
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float t;
        CK(hipEventElapsedTime(&t, a, b));
        ms.push_back(t);
    }
    std::sort(ms.begin(), ms.end());
    const double t = ms[ms.size() / 2];
    const double waves = (double)grid * NT / 64;
    const double instr_per_cu = waves * ITERS * 8 / cus;
    const double lanes = (P == 3 ? 32.0 : 64.0);
    printf("{\"pattern\": \"%s\", \"ms\": %.4f, \"ns_per_gather_instr_per_cu\": %.3f, \"lanes_per_ns_per_cu\": %.3f, "
           "\"bytes_per_lane\": %d}\n",
           name, t, t * 1e6 / instr_per_cu, instr_per_cu * lanes / (t * 1e6), (P == 4 || P == 8) ? 16 : P == 7 ? 8 : 4);
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
}

int main() {
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    std::vector<float> h(W * H);
    for (int i = 0; i < W * H; ++i) h[i] = 1.0f + (float)(i % 97) * 0.01f;
    float *d_frame, *d_out;
    CK(hipMalloc(&d_frame, sizeof(float) * W * H));
    const int grid = cus * 8;  // 8 waves / SIMD x 4 SIMDs = 32 waves = 4 workgroups of 512 per CU, x2 for tails
    CK(hipMalloc(&d_out, sizeof(float) * (size_t)grid * NT));
    CK(hipMemcpy(d_frame, h.data(), sizeof(float) * W * H, hipMemcpyHostToDevice));
    run<0>("same", d_frame, d_out, grid, cus);
    run<1>("coalesced", d_frame, d_out, grid, cus);
    run<2>("brick", d_frame, d_out, grid, cus);
    run<3>("brick_even", d_frame, d_out, grid, cus);
    run<4>("brick_x4", d_frame, d_out, grid, cus);
    run<7>("brick_x2", d_frame, d_out, grid, cus);
    run<8>("brick_x4_lds", d_frame, d_out, grid, cus);
    run<5>("window", d_frame, d_out, grid, cus);
    run<6>("frame", d_frame, d_out, grid, cus);
    CK(hipFree(d_frame));
    CK(hipFree(d_out));
    return 0;
}

// Sustained i8 MFMA rate and shader clock by operand pattern on gfx950 (is the exact search kernel power-bound,
// and what makes an MFMA cheaper?). One wave per SIMD on every CU runs back-to-back MFMAs for ~0.4 s, cycling
// through 4 operand sets per lane (random per lane, seeded); wave 0 of each block stamps s_memtime /
// s_memrealtime around its loop, so the in-kernel clock is cycles / (realtime ticks / 100 MHz).
// Patterns (A operand; B always random bytes):
//   0 random bytes, 1 top byte zero (A >> 8), 2 two zero bytes (A >> 16), 3 one small byte (A >> 24 of a 30-bit
//   digit word), 4 all zero, 5 sparse v_smfmac_i32_32x32x64_i8 (random compressed A, random B, 16x the B bytes),
//   6 dense v_mfma_i32_16x16x64_i8 on random operands (4 accumulators of 4 registers; ns per 16x16x64 instruction
//   = half the MACs of a 32x32x32 one)
// build: hipcc --offload-arch=gfx950 -O3 -o build/mb_power tools/mb_power.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef int i32x16 __attribute__((ext_vector_type(16)));

__device__ unsigned hash(unsigned x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}

template <int PAT>
__global__ __launch_bounds__(256, 1) void k_pow(int iters, unsigned seed, long long* stamps, int* out) {
    i32x4 a[4];
    i32x8 b[4];
    for (int s = 0; s < 4; ++s)
        for (int k = 0; k < 8; ++k) {
            unsigned r = hash(seed ^ (threadIdx.x * 977u + blockIdx.x * 131071u + s * 7919u + k * 104729u));
            unsigned w = hash(r + 12345u);
            if (k < 4) {
                unsigned v = r;
                if (PAT == 1) v = r >> 8;
                if (PAT == 2) v = r >> 16;
                if (PAT == 3) v = (r >> 24) & 0x7f;
                if (PAT == 4) v = 0;
                a[s][k] = (int)v;
            }
            b[s][k] = (int)w;
        }
    i32x16 c[4] = {};
    long long t0 = 0, r0 = 0;
    if (threadIdx.x == 0) {
        t0 = __builtin_amdgcn_s_memtime();
        r0 = __builtin_amdgcn_s_memrealtime();
    }
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            if (PAT == 5)
                asm volatile("v_smfmac_i32_32x32x64_i8 %0, %1, %2, %3" : "+v"(c[s]) : "v"(a[s]), "v"(b[s]), "v"(0x44444444));
            else if (PAT == 6)
                asm volatile("v_mfma_i32_16x16x64_i8 %0, %1, %2, %0"
                             : "+v"(*reinterpret_cast<i32x4*>(&c[s]))
                             : "v"(a[s]), "v"(i32x4{b[s][0], b[s][1], b[s][2], b[s][3]}));
            else
                asm volatile("v_mfma_i32_32x32x32_i8 %0, %1, %2, %0" : "+v"(c[s]) : "v"(a[s]), "v"(i32x4{b[s][0], b[s][1], b[s][2], b[s][3]}));
        }
    }
    asm volatile("s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7");
    if (threadIdx.x == 0) {
        const long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        stamps[2 * blockIdx.x] = t1 - t0;
        stamps[2 * blockIdx.x + 1] = r1 - r0;
    }
    int r = 0;
    for (int s = 0; s < 4; ++s)
        for (int k = 0; k < 16; ++k) r += c[s][k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <int PAT>
static void run(const char* name, int iters, long long* st, int* out) {
    hipLaunchKernelGGL(k_pow<PAT>, dim3(256), dim3(256), 0, 0, iters / 4, 1u, st, out);  // warm up
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_pow<PAT>, dim3(256), dim3(256), 0, 0, iters, 7u, st, out);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    std::vector<long long> h(512);
    hipMemcpy(h.data(), st, 512 * sizeof(long long), hipMemcpyDeviceToHost);
    std::vector<double> clk;
    for (int i = 0; i < 256; ++i) clk.push_back((double)h[2 * i] / ((double)h[2 * i + 1] / 100e6) / 1e9);
    std::sort(clk.begin(), clk.end());
    const double nm = (double)iters * 4;  // MFMAs per wave (= per SIMD)
    printf("%-34s %8.2f ms  %6.2f ns/MFMA  %5.1f cyc/MFMA  clock %.3f GHz (p10 %.3f p90 %.3f)\n", name, ms,
           ms * 1e6 / nm, ms * 1e-3 * clk[128] * 1e9 / nm, clk[128], clk[25], clk[230]);
}

int main() {
    long long* st;
    int* out;
    hipMalloc(&st, 512 * sizeof(long long));
    hipMalloc(&out, 256 * 256 * sizeof(int));
    const int iters = 7000000;  // 2.8e7 MFMAs per SIMD: ~0.4 s at 13-16 ns per MFMA
    for (int rep = 0; rep < 2; ++rep) {
        run<0>("dense, random A", iters, st, out);
        run<1>("dense, A top byte zero", iters, st, out);
        run<2>("dense, A two bytes zero", iters, st, out);
        run<3>("dense, A one small byte", iters, st, out);
        run<4>("dense, A zero", iters, st, out);
        run<5>("sparse smfmac K=64, random", iters, st, out);
        run<6>("dense 16x16x64, random", iters, st, out);
    }
    return 0;
}

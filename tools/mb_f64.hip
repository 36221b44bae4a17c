// Microbenchmark + layout probe for the NUFFT spreading kernel design (gfx950):
//  1. v_mfma_f64_16x16x4_f64 operand/result lane maps with exact small integers;
//  2. back-to-back f64 MFMA rate (one wave per SIMD, 4 independent accumulators);
//  3. fp64 FMA VALU rate;
//  4. f64 MFMA interleaved with V fp64 FMAs per MFMA (does the VALU hide under the matrix pipe?).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/bin/mb_f64 tools/mb_f64.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef double f64x4 __attribute__((ext_vector_type(4)));

__global__ void k_layout(double* out) {
    const int l = threadIdx.x;
    // A[i][k] = i + 100 k at lane (i = l & 15, k = l >> 4) if the documented map holds; B[k][j] = 1 if k == 1 else 0
    const double a = (double)((l & 15) + 100 * (l >> 4));
    const double b = ((l >> 4) == 1) ? (double)(1 + (l & 15)) : 0.0;
    f64x4 c = {0, 0, 0, 0};
    c = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
    for (int r = 0; r < 4; ++r) out[l * 4 + r] = c[r];
}

template <int MODE, int V>
__global__ __launch_bounds__(256) void k_rate(double* out, int iters) {
    const int t = threadIdx.x;
    f64x4 a0 = {0, 0, 0, 0}, a1 = a0, a2 = a0, a3 = a0;
    double A = t * 1e-3 + 0.5, B = t * 2e-3 - 0.25;
    double d[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) d[j] = t * 1e-3 + j;
    for (int it = 0; it < iters; ++it) {
        if (MODE & 1) {
            a0 = __builtin_amdgcn_mfma_f64_16x16x4f64(A, B, a0, 0, 0, 0);
            if (MODE & 2) {
#pragma unroll
                for (int j = 0; j < V; ++j) d[j & 15] = __builtin_fma(d[j & 15], 0.999, 1e-4);
            }
            a1 = __builtin_amdgcn_mfma_f64_16x16x4f64(B, A, a1, 0, 0, 0);
            if (MODE & 2) {
#pragma unroll
                for (int j = 0; j < V; ++j) d[(j + 5) & 15] = __builtin_fma(d[(j + 5) & 15], 0.999, 1e-4);
            }
            a2 = __builtin_amdgcn_mfma_f64_16x16x4f64(A, A, a2, 0, 0, 0);
            if (MODE & 2) {
#pragma unroll
                for (int j = 0; j < V; ++j) d[(j + 9) & 15] = __builtin_fma(d[(j + 9) & 15], 0.999, 1e-4);
            }
            a3 = __builtin_amdgcn_mfma_f64_16x16x4f64(B, B, a3, 0, 0, 0);
            if (MODE & 2) {
#pragma unroll
                for (int j = 0; j < V; ++j) d[(j + 13) & 15] = __builtin_fma(d[(j + 13) & 15], 0.999, 1e-4);
            }
        } else if (MODE & 2) {
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int j = 0; j < V; ++j) d[(j + 4 * r) & 15] = __builtin_fma(d[(j + 4 * r) & 15], 0.999, 1e-4);
        }
    }
    double s = 0;
    for (int j = 0; j < 16; ++j) s += d[j];
    for (int j = 0; j < 4; ++j) s += a0[j] + a1[j] + a2[j] + a3[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int MODE, int V>
static double run(double* out, int blocks, int iters) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    k_rate<MODE, V><<<blocks, 256>>>(out, iters);
    hipEventRecord(e0);
    k_rate<MODE, V><<<blocks, 256>>>(out, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    return ms;
}

int main() {
    double* d = nullptr;
    hipMalloc(&d, 1 << 24);
    k_layout<<<1, 64>>>(d);
    std::vector<double> h(256);
    hipMemcpy(h.data(), d, 256 * sizeof(double), hipMemcpyDeviceToHost);
    // D[i][j] = sum_k A[i][k] B[k][j] = A[i][1] * (1 + j) = (i + 100) (1 + j) under the documented A/B maps.
    int bad = 0;
    for (int l = 0; l < 64; ++l)
        for (int r = 0; r < 4; ++r) {
            const int col = l & 15, row = (l >> 4) + 4 * r;
            const double want = (double)(row + 100) * (double)(1 + col);
            if (h[l * 4 + r] != want) {
                if (bad < 8) printf("layout mismatch lane %d reg %d: got %g want %g\n", l, r, h[l * 4 + r], want);
                ++bad;
            }
        }
    printf("layout: %s (%d mismatches)\n", bad ? "MISMATCH" : "documented map holds", bad);
    int ncu = 256;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    const int blocks = ncu;  // one 256-thread block per CU = one wave per SIMD
    const int iters = 20000;
    const double simds = 4.0 * ncu;
    {
        const double ms = run<1, 0>(d, blocks, iters);
        const double n = 4.0 * iters;  // MFMAs per wave
        printf("f64 MFMA back-to-back: %.3f ms, %.2f ns per MFMA per SIMD, %.1f TFLOP/s\n", ms, ms * 1e6 / n,
               n * simds * 2048.0 / (ms * 1e-3) / 1e12);
    }
    {
        const double ms = run<2, 16>(d, blocks, iters);
        const double n = 4.0 * 16 * iters;  // fp64 FMA instructions per wave
        printf("fp64 VALU FMA: %.3f ms, %.2f ns per instruction per SIMD, %.1f TFLOP/s\n", ms, ms * 1e6 / n,
               n * simds * 64 * 2.0 / (ms * 1e-3) / 1e12);
    }
#define MIX(VV)                                                                                                  \
    {                                                                                                            \
        const double ms = run<3, VV>(d, blocks, iters);                                                          \
        const double n = 4.0 * iters;                                                                            \
        printf("f64 MFMA + %2d fp64 FMA per MFMA: %.2f ns per MFMA per SIMD (MFMA %.1f TF + VALU %.1f TF)\n", VV, \
               ms * 1e6 / n, n * simds * 2048.0 / (ms * 1e-3) / 1e12,                                            \
               n * VV * simds * 64 * 2.0 / (ms * 1e-3) / 1e12);                                                   \
    }
    MIX(2) MIX(4) MIX(6) MIX(8) MIX(12) MIX(16)
    // two waves per SIMD: 512-thread blocks
    hipFree(d);
    return 0;
}

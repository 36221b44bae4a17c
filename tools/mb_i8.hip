// Microbenchmark + layout probe for the exact-integer search kernel design (gfx950):
//  1. v_mfma_i32_32x32x32_i8 operand/result lane maps with exact integers;
//  2. issue cost of fp64 FMA, fp32 FMA and 32-bit integer VALU, one and two waves per SIMD;
//  3. i8 MFMA back-to-back, and i8 MFMA interleaved with fp64 VALU.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ int8_t av(int lane, int j) { return (int8_t)(((lane * 7 + j * 13) % 23) - 11); }
__device__ __forceinline__ int8_t bv(int lane, int j) { return (int8_t)(((lane * 5 + j * 3 + 1) % 19) - 9); }

__global__ void k_layout(int* out) {
    const int l = threadIdx.x;
    int8_t a[16], b[16];
    for (int j = 0; j < 16; ++j) { a[j] = av(l, j); b[j] = bv(l, j); }
    i32x4 A, B;
    __builtin_memcpy(&A, a, 16);
    __builtin_memcpy(&B, b, 16);
    i32x16 c = {};
    c = __builtin_amdgcn_mfma_i32_32x32x32_i8(A, B, c, 0, 0, 0);
    for (int r = 0; r < 16; ++r) out[l * 16 + r] = c[r];
}

template <int MODE, int V>
__global__ __launch_bounds__(256) void k_rate(double* out, int iters) {
    i32x16 a0 = {}, a1 = {}, a2 = {}, a3 = {};
    const int t = threadIdx.x;
    i32x4 A = {t, t * 3, t ^ 5, t + 7}, B = {t * 11, t + 1, t ^ 9, t * 2};
    double d[16];
    float f[16];
    unsigned u[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) { d[j] = t * 1e-3 + j; f[j] = t * 1e-3f + j; u[j] = t * 31u + j; }
    for (int it = 0; it < iters; ++it) {
        if (MODE & 1) {
            a0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(A, B, a0, 0, 0, 0);
            a1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(B, A, a1, 0, 0, 0);
            a2 = __builtin_amdgcn_mfma_i32_32x32x32_i8(A, A, a2, 0, 0, 0);
            a3 = __builtin_amdgcn_mfma_i32_32x32x32_i8(B, B, a3, 0, 0, 0);
        }
        if (MODE & 2) {  // fp64 FMA
#pragma unroll
            for (int r = 0; r < V / 16; ++r)
#pragma unroll
                for (int j = 0; j < 16; ++j) d[j] = __builtin_fma(d[j], 0.999, 1e-4);
        }
        if (MODE & 4) {  // fp32 FMA
#pragma unroll
            for (int r = 0; r < V / 16; ++r)
#pragma unroll
                for (int j = 0; j < 16; ++j) f[j] = __builtin_fmaf(f[j], 0.999f, 1e-4f);
        }
        if (MODE & 8) {  // integer add / xor (VALU)
#pragma unroll
            for (int r = 0; r < V / 16; ++r)
#pragma unroll
                for (int j = 0; j < 16; ++j) u[j] = (u[j] + 0x00808080u) ^ (0x00808080u + r);
        }
        if (MODE & 16) {  // fp64 mul
#pragma unroll
            for (int r = 0; r < V / 16; ++r)
#pragma unroll
                for (int j = 0; j < 16; ++j) d[j] = d[j] * 0.999;
        }
    }
    double s = 0;
    for (int j = 0; j < 16; ++j) s += a0[j] + a1[j] + a2[j] + a3[j] + d[j] + f[j] + u[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int MODE, int V>
double run(double* out, int blocks, int iters) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    k_rate<MODE, V><<<blocks, 256>>>(out, 10);
    hipEventRecord(e0);
    k_rate<MODE, V><<<blocks, 256>>>(out, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    return ms;
}

int main() {
    // ---- layout
    int* dout;
    hipMalloc(&dout, 64 * 16 * 4);
    k_layout<<<1, 64>>>(dout);
    std::vector<int> h(64 * 16);
    hipMemcpy(h.data(), dout, h.size() * 4, hipMemcpyDeviceToHost);
    auto A = [](int l, int j) { return (int)(int8_t)(((l * 7 + j * 13) % 23) - 11); };
    auto B = [](int l, int j) { return (int)(int8_t)(((l * 5 + j * 3 + 1) % 19) - 9); };
    // hypothesis: D[a][b] = sum_{h,j} A(a + 32h, j) * B(b + 32h, j); lane l reg r holds
    // D[row = (r&3) + 8(r>>2) + 4(l>>5)][col = l&31]
    int bad = 0;
    for (int l = 0; l < 64; ++l)
        for (int r = 0; r < 16; ++r) {
            const int row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5), col = l & 31;
            long ref = 0;
            for (int hh = 0; hh < 2; ++hh)
                for (int j = 0; j < 16; ++j) ref += A(row + 32 * hh, j) * B(col + 32 * hh, j);
            if (ref != h[l * 16 + r]) ++bad;
        }
    printf("i8 32x32x32 symmetric-K / f16-style C map hypothesis: %d mismatches of 1024\n", bad);
    // ---- rates
    double* out;
    hipMalloc(&out, 4096 * 256 * 8);
    const int iters = 20000;
    for (int wps : {1, 2}) {
        const int blocks = 256 * wps;
        const double per = 1e-3 / ((double)iters) * 2.4e9;
        printf("waves/SIMD=%d  cycles/iter per wave (2.4GHz nominal)\n", wps);
        printf("  i8 MFMA x4 only         : %.1f\n", run<1, 0>(out, blocks, iters) * per);
        printf("  f64 FMA 32 only         : %.1f\n", run<2, 32>(out, blocks, iters) * per);
        printf("  f64 FMA 64 only         : %.1f\n", run<2, 64>(out, blocks, iters) * per);
        printf("  f64 MUL 64 only         : %.1f\n", run<16, 64>(out, blocks, iters) * per);
        printf("  f32 FMA 64 only         : %.1f\n", run<4, 64>(out, blocks, iters) * per);
        printf("  int add+xor 64 (128 op) : %.1f\n", run<8, 64>(out, blocks, iters) * per);
        printf("  i8 MFMA x4 + f64 FMA 32 : %.1f\n", run<3, 32>(out, blocks, iters) * per);
        printf("  i8 MFMA x4 + f64 FMA 64 : %.1f\n", run<3, 64>(out, blocks, iters) * per);
        printf("  i8 MFMA x4 + int 64     : %.1f\n", run<9, 64>(out, blocks, iters) * per);
    }
    return 0;
}

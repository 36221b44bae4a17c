// Microbenchmark: does a wave's VALU work overlap the f32 / f16 MFMA pipe on gfx950?
// Each wave runs `iters` iterations of {4 MFMAs on 2 accumulators} and/or {V independent fp32 FMAs}.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

template <int MODE, int V>
__global__ __launch_bounds__(256) void k(float* out, int iters) {
    f32x16 a0 = {}, a1 = {};
    float x = threadIdx.x * 1e-3f, y = 1.0f - x;
    f16x8 hx, hy;
    for (int i = 0; i < 8; ++i) { hx[i] = (_Float16)(x + i); hy[i] = (_Float16)(y - i); }
    float v[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = x * (j + 1);
    for (int it = 0; it < iters; ++it) {
        if (MODE & 1) {
            a0 = __builtin_amdgcn_mfma_f32_32x32x2f32(x, y, a0, 0, 0, 0);
            a1 = __builtin_amdgcn_mfma_f32_32x32x2f32(y, x, a1, 0, 0, 0);
            a0 = __builtin_amdgcn_mfma_f32_32x32x2f32(x, x, a0, 0, 0, 0);
            a1 = __builtin_amdgcn_mfma_f32_32x32x2f32(y, y, a1, 0, 0, 0);
        }
        if (MODE & 4) {
            a0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(hx, hy, a0, 0, 0, 0);
            a1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(hy, hx, a1, 0, 0, 0);
            a0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(hx, hx, a0, 0, 0, 0);
            a1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(hy, hy, a1, 0, 0, 0);
        }
        if (MODE & 2) {
#pragma unroll
            for (int r = 0; r < V / 16; ++r)
#pragma unroll
                for (int j = 0; j < 16; ++j) v[j] = __builtin_fmaf(v[j], 0.999f, 1e-4f);
        }
    }
    float s = 0;
    for (int j = 0; j < 16; ++j) s += a0[j] + a1[j] + v[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int MODE, int V>
double run(float* out, int blocks, int iters) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    k<MODE, V><<<blocks, 256>>>(out, 10);
    hipEventRecord(e0);
    k<MODE, V><<<blocks, 256>>>(out, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    return ms;
}

int main() {
    float* out; hipMalloc(&out, 4096 * 256 * 4);
    const int iters = 20000;
    for (int wps : {1, 2}) {  // waves per SIMD
        const int blocks = 256 * wps;  // 256-thread blocks = 4 waves = 1 per SIMD
        double per = 1e-3 / ((double)iters) * 2.4e9;  // cycles per iteration (at 2.4 GHz)
        printf("waves/SIMD=%d  cycles/iter per wave (2.4GHz)\n", wps);
        printf("  f32 MFMA x4 only      : %.1f\n", run<1, 0>(out, blocks, iters) * per);
        printf("  VALU 32 only          : %.1f\n", run<2, 32>(out, blocks, iters) * per);
        printf("  VALU 64 only          : %.1f\n", run<2, 64>(out, blocks, iters) * per);
        printf("  f32 MFMA x4 + VALU 32 : %.1f\n", run<3, 32>(out, blocks, iters) * per);
        printf("  f32 MFMA x4 + VALU 64 : %.1f\n", run<3, 64>(out, blocks, iters) * per);
        printf("  f16 MFMA x4 only      : %.1f\n", run<4, 0>(out, blocks, iters) * per);
        printf("  f16 MFMA x4 + VALU 32 : %.1f\n", run<6, 32>(out, blocks, iters) * per);
        printf("  f16 MFMA x4 + VALU 64 : %.1f\n", run<6, 64>(out, blocks, iters) * per);
    }
    return 0;
}

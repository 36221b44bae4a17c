// Do MFMA and VALU work of DIFFERENT waves on one SIMD overlap on gfx950? One block of 8 waves per CU (2 per
// SIMD): mode 0 = all waves run the MFMA loop, 1 = all run the VALU loop, 2 = waves 0-3 MFMA and 4-7 VALU
// (one of each per SIMD), 3 = only waves 0-3 run MFMA (4-7 idle), 4 = only waves 4-7 run VALU.
// build: hipcc --offload-arch=gfx950 -O3 -o build/mb_overlap tools/mb_overlap.hip
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));

__global__ __launch_bounds__(512, 1) void k_overlap(int mode, int iters, int* out) {
    const int wv = threadIdx.x >> 6;
    const bool mfma_wave = (mode == 0) || ((mode == 2 || mode == 3) && wv < 4);
    const bool valu_wave = (mode == 1) || ((mode == 2 || mode == 4) && wv >= 4);
    int r = 0;
    if (mfma_wave) {
        i32x4 a = {(int)threadIdx.x, 1, 2, 3}, b = {3, 2, 1, (int)threadIdx.x};
        i32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
        for (int i = 0; i < iters; ++i) {
            c0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c1, 0, 0, 0);
            c2 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c2, 0, 0, 0);
            c3 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c3, 0, 0, 0);
        }
        for (int k = 0; k < 16; ++k) r += c0[k] + c1[k] + c2[k] + c3[k];
    }
    if (valu_wave) {
        float x0 = threadIdx.x, x1 = 1.f, x2 = 2.f, x3 = 3.f, x4 = 4.f, x5 = 5.f, x6 = 6.f, x7 = 7.f;
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {  // 64 independent-ish fp32 FMAs per iteration
                x0 = __builtin_fmaf(x0, 1.0001f, 0.5f); x1 = __builtin_fmaf(x1, 1.0001f, 0.5f);
                x2 = __builtin_fmaf(x2, 1.0001f, 0.5f); x3 = __builtin_fmaf(x3, 1.0001f, 0.5f);
                x4 = __builtin_fmaf(x4, 1.0001f, 0.5f); x5 = __builtin_fmaf(x5, 1.0001f, 0.5f);
                x6 = __builtin_fmaf(x6, 1.0001f, 0.5f); x7 = __builtin_fmaf(x7, 1.0001f, 0.5f);
            }
        }
        r += (int)(x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7);
    }
    if (mode >= 5 && ((mode == 5) || wv >= 4)) {  // integer VALU (not packable): 64 adds/xors per iteration
        unsigned u0 = threadIdx.x, u1 = 1, u2 = 2, u3 = 3, u4 = 4, u5 = 5, u6 = 6, u7 = 7;
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                u0 = (u0 + 0x9e3779b9u) ^ u1; u1 = (u1 + 0x9e3779b9u) ^ u2; u2 = (u2 + 0x9e3779b9u) ^ u3;
                u3 = (u3 + 0x9e3779b9u) ^ u4; u4 = (u4 + 0x9e3779b9u) ^ u5; u5 = (u5 + 0x9e3779b9u) ^ u6;
                u6 = (u6 + 0x9e3779b9u) ^ u7; u7 = (u7 + 0x9e3779b9u) ^ u0;
            }
        }
        r += (int)(u0 + u1 + u2 + u3 + u4 + u5 + u6 + u7);
    }
    if ((mode == 7 || mode == 8) && wv < 4) {  // MFMA accumulating in AGPRs
        i32x4 a = {(int)threadIdx.x, 1, 2, 3}, b = {3, 2, 1, (int)threadIdx.x};
        i32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
        asm volatile("s_nop 7" : "+a"(c0), "+a"(c1), "+a"(c2), "+a"(c3));
        for (int i = 0; i < iters; ++i) {
            asm volatile(
                "v_mfma_i32_32x32x32_i8 %0, %4, %5, %0\n"
                "v_mfma_i32_32x32x32_i8 %1, %4, %5, %1\n"
                "v_mfma_i32_32x32x32_i8 %2, %4, %5, %2\n"
                "v_mfma_i32_32x32x32_i8 %3, %4, %5, %3\n"
                : "+a"(c0), "+a"(c1), "+a"(c2), "+a"(c3)
                : "v"(a), "v"(b));
        }
        asm volatile("s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7" : "+a"(c0), "+a"(c1), "+a"(c2), "+a"(c3));
        for (int k = 0; k < 16; ++k) r += c0[k] + c1[k] + c2[k] + c3[k];
    }
    if (mode == 7 && wv >= 4) {
        float x0 = threadIdx.x, x1 = 1.f, x2 = 2.f, x3 = 3.f, x4 = 4.f, x5 = 5.f, x6 = 6.f, x7 = 7.f;
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                x0 = __builtin_fmaf(x0, 1.0001f, 0.5f); x1 = __builtin_fmaf(x1, 1.0001f, 0.5f);
                x2 = __builtin_fmaf(x2, 1.0001f, 0.5f); x3 = __builtin_fmaf(x3, 1.0001f, 0.5f);
                x4 = __builtin_fmaf(x4, 1.0001f, 0.5f); x5 = __builtin_fmaf(x5, 1.0001f, 0.5f);
                x6 = __builtin_fmaf(x6, 1.0001f, 0.5f); x7 = __builtin_fmaf(x7, 1.0001f, 0.5f);
            }
        }
        r += (int)(x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7);
    }
    if (mode == 6 && wv < 4) {
        i32x4 a = {(int)threadIdx.x, 1, 2, 3}, b = {3, 2, 1, (int)threadIdx.x};
        i32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
        for (int i = 0; i < iters; ++i) {
            c0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c1, 0, 0, 0);
            c2 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c2, 0, 0, 0);
            c3 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c3, 0, 0, 0);
        }
        for (int k = 0; k < 16; ++k) r += c0[k] + c1[k] + c2[k] + c3[k];
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

int main() {
    int* d;
    hipMalloc(&d, 256 * 512 * sizeof(int));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const char* names[9] = {"all MFMA (8 waves)", "all VALU (8 waves)", "4 MFMA + 4 VALU waves", "4 MFMA waves only",
                            "4 VALU waves only", "int VALU, 8 waves", "4 MFMA + 4 int VALU waves",
                            "4 AGPR-MFMA + 4 VALU waves", "4 AGPR-MFMA waves only"};
    for (int rep = 0; rep < 2; ++rep)
        for (int mode = 0; mode < 9; ++mode) {
            const int iters = 20000;
            hipLaunchKernelGGL(k_overlap, dim3(256), dim3(512), 0, 0, mode, iters, d);
            hipEventRecord(e0);
            hipLaunchKernelGGL(k_overlap, dim3(256), dim3(512), 0, 0, mode, iters, d);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            printf("%-26s %8.3f ms\n", names[mode], ms);
        }
    return 0;
}

#include <hip/hip_runtime.h>
#include <cstdio>
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));
template <int NACC>
__global__ __launch_bounds__(256, 1) void k_mfma(int iters, int* out) {
    i32x4 a = {(int)threadIdx.x, 1, 2, 3}, b = {3, 2, 1, (int)threadIdx.x};
    i32x16 c[NACC];
    for (int j = 0; j < NACC; ++j) c[j] = i32x16{};
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int j = 0; j < NACC; ++j) c[j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c[j], 0, 0, 0);
    }
    int r = 0;
    for (int j = 0; j < NACC; ++j)
        for (int k = 0; k < 16; ++k) r += c[j][k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
int main() {
    int* d;
    (void)hipMalloc(&d, 256 * 256 * sizeof(int));
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int rep = 0; rep < 2; ++rep) {
        float ms;
        hipLaunchKernelGGL(k_mfma<4>, dim3(256), dim3(256), 0, 0, 20000, d);
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(k_mfma<4>, dim3(256), dim3(256), 0, 0, 20000, d);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        (void)hipEventElapsedTime(&ms, e0, e1);
        printf("4 acc (VGPR?)  %.3f ms per 80000 MFMAs/SIMD\n", ms);
        hipLaunchKernelGGL(k_mfma<16>, dim3(256), dim3(256), 0, 0, 5000, d);
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(k_mfma<16>, dim3(256), dim3(256), 0, 0, 5000, d);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        (void)hipEventElapsedTime(&ms, e0, e1);
        printf("16 acc (256 regs) %.3f ms per 80000 MFMAs/SIMD\n", ms);
    }
    return 0;
}

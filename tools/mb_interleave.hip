// How much VALU work hides beside v_mfma_i32_32x32x32_i8 on gfx950?  Each loop slot is one MFMA followed by N
// independent vector instructions (inline asm, so the stream is exactly that); 8 slots per iteration on 8
// independent accumulators. Modes:
//   same  : every wave runs the interleaved stream (1 or 2 waves per SIMD)
//   split : 2 waves per SIMD, waves 0-3 MFMA only, waves 4-7 the N VALU only (cross-wave overlap)
//   valu  : the VALU stream alone (no MFMA), 1 wave per SIMD
// VALU kinds: 0 = v_xor_b32, 1 = v_fma_f64, 2 = v_fma_f32, 3 = v_lshrrev_b32 + v_add_u32 alternated.
// build: hipcc --offload-arch=gfx950 -O3 -o build/mb_interleave tools/mb_interleave.hip
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));

template <int KIND>
__device__ __forceinline__ void valu1(unsigned& x, unsigned y, double& d, double e, float& f, int j) {
    if (KIND == 0) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x) : "v"(y));
    if (KIND == 1) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(d) : "v"(e));
    if (KIND == 2) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(f) : "v"(__uint_as_float(y)));
    if (KIND == 3) {
        if (j & 1) asm volatile("v_lshrrev_b32 %0, 8, %0" : "+v"(x));
        else asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(y));
    }
}

template <int N, int KIND>
__device__ __forceinline__ void valu_n(unsigned* x, unsigned y, double* d, double e, float* f) {
#pragma unroll
    for (int j = 0; j < N; ++j) valu1<KIND>(x[j], y, d[j], e, f[j], j);
}

// mode 0 = same, 1 = split, 2 = valu only
template <int N, int KIND>
__global__ __launch_bounds__(512, 1) void k_mb(int mode, int iters, int* out) {
    const int wv = threadIdx.x >> 6;
    const bool do_mfma = __builtin_amdgcn_readfirstlane(mode == 0 || (mode == 1 && wv < 4));
    const bool do_valu = __builtin_amdgcn_readfirstlane(mode == 0 || mode == 2 || (mode == 1 && wv >= 4));
    i32x4 a = {(int)threadIdx.x, 1, 2, 3}, b = {3, 2, 1, (int)threadIdx.x};
    i32x16 c[8];
#pragma unroll
    for (int m = 0; m < 8; ++m) c[m] = i32x16{} + m;
    unsigned x[N > 0 ? N : 1];
    double d[N > 0 ? N : 1];
    float f[N > 0 ? N : 1];
#pragma unroll
    for (int j = 0; j < (N > 0 ? N : 1); ++j) {
        x[j] = threadIdx.x + j;
        d[j] = 1.0 + j;
        f[j] = 1.0f + j;
    }
    const unsigned y = 0x9e3779b9u ^ threadIdx.x;
    const double e = 0.999999;
    // wave-uniform branches outside the loops: the loop bodies are exactly the asm streams
    if (do_mfma && do_valu) {
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int m = 0; m < 8; ++m) {
                asm volatile("v_mfma_i32_32x32x32_i8 %0, %1, %2, %0" : "+v"(c[m]) : "v"(a), "v"(b));
                valu_n<N, KIND>(x, y, d, e, f);
            }
        }
    } else if (do_mfma) {
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int m = 0; m < 8; ++m)
                asm volatile("v_mfma_i32_32x32x32_i8 %0, %1, %2, %0" : "+v"(c[m]) : "v"(a), "v"(b));
        }
    } else if (do_valu) {
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int m = 0; m < 8; ++m) valu_n<N, KIND>(x, y, d, e, f);
        }
    }
    asm volatile("s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7");
    int r = 0;
#pragma unroll
    for (int m = 0; m < 8; ++m)
#pragma unroll
        for (int k = 0; k < 16; ++k) r += c[m][k];
#pragma unroll
    for (int j = 0; j < (N > 0 ? N : 1); ++j) r += (int)x[j] + (int)d[j] + (int)f[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

// back-to-back 2:4-sparse i8 MFMA (K = 64 per instruction) on 8 accumulators, 1 or 2 waves per SIMD
__global__ __launch_bounds__(512, 1) void k_smf(int iters, int idx, int* out) {
    typedef int i32x8 __attribute__((ext_vector_type(8)));
    i32x4 a = {(int)threadIdx.x, 1, 2, 3};
    i32x8 b = {3, 2, 1, (int)threadIdx.x, 5, 6, 7, 8};
    i32x16 c[8];
#pragma unroll
    for (int m = 0; m < 8; ++m) c[m] = i32x16{} + m;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int m = 0; m < 8; ++m)
            asm volatile("v_smfmac_i32_32x32x64_i8 %0, %1, %2, %3" : "+v"(c[m]) : "v"(a), "v"(b), "v"(idx));
    }
    asm volatile("s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7");
    int r = 0;
#pragma unroll
    for (int m = 0; m < 8; ++m)
#pragma unroll
        for (int k = 0; k < 16; ++k) r += c[m][k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

static int* g_out;
static hipEvent_t e0, e1;

template <int N, int KIND>
static void run(int mode, int threads, const char* tag) {
    const int iters = 4000;
    hipLaunchKernelGGL((k_mb<N, KIND>), dim3(256), dim3(threads), 0, 0, mode, iters, g_out);
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
        hipEventRecord(e0);
        hipLaunchKernelGGL((k_mb<N, KIND>), dim3(256), dim3(threads), 0, 0, mode, iters, g_out);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        best = ms < best ? ms : best;
    }
    // slots per SIMD: iters * 8 per wave, waves per SIMD = threads / 256
    const double slots = (double)iters * 8 * (threads / 256);
    printf("%-6s kind=%d N=%2d waves/SIMD=%d  %8.3f ms  %7.2f ns/slot/SIMD\n", tag, KIND, N, threads / 256, best,
           best * 1e6 / slots);
}

template <int KIND>
static void sweep() {
    run<0, KIND>(0, 256, "same");
    run<2, KIND>(0, 256, "same");
    run<4, KIND>(0, 256, "same");
    run<5, KIND>(0, 256, "same");
    run<6, KIND>(0, 256, "same");
    run<7, KIND>(0, 256, "same");
    run<8, KIND>(0, 256, "same");
    run<10, KIND>(0, 256, "same");
    run<4, KIND>(2, 256, "valu");
    run<8, KIND>(2, 256, "valu");
    run<0, KIND>(0, 512, "same");
    run<4, KIND>(0, 512, "same");
    run<6, KIND>(0, 512, "same");
    run<8, KIND>(0, 512, "same");
    run<4, KIND>(1, 512, "split");
    run<8, KIND>(1, 512, "split");
    run<16, KIND>(1, 512, "split");
}

int main() {
    hipMalloc(&g_out, 256 * 512 * sizeof(int));
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int threads = 256; threads <= 512; threads += 256) {
        const int iters = 4000;
        hipLaunchKernelGGL(k_smf, dim3(256), dim3(threads), 0, 0, iters, 0x44, g_out);
        hipEventRecord(e0);
        hipLaunchKernelGGL(k_smf, dim3(256), dim3(threads), 0, 0, iters, 0x44, g_out);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        printf("smfmac_i32_32x32x64_i8 waves/SIMD=%d %8.3f ms %7.2f ns/instr/SIMD\n", threads / 256, ms,
               ms * 1e6 / ((double)iters * 8 * (threads / 256)));
    }
    sweep<0>();
    sweep<1>();
    sweep<2>();
    sweep<3>();
    return 0;
}

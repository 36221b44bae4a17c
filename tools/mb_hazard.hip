// Micro-test of the v_mfma_i32_32x32x32_i8 operand/result timing on gfx950 (one wave, hand-placed registers,
// so that the compiler adds no padding). For each distance N (wait states after the MFMA):
//   RAW: read the 16 result registers (last row first) N wait states after the MFMA;
//   WAR-A / WAR-B: overwrite the A (or B) operand registers with zero N wait states after the MFMA, then
//         wait long and read the results.
// A and B are all-ones bytes, so every D element is 32 when the MFMA saw its operands and finished.
// build: hipcc --offload-arch=gfx950 -O2 -o build/mb_hazard tools/mb_hazard.hip ; run: build/mb_hazard
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>

#define NOP1 "s_nop 0\n"
#define NOP8 "s_nop 7\n"
#define NOP64 NOP8 NOP8 NOP8 NOP8 NOP8 NOP8 NOP8 NOP8
#define LONGWAIT NOP64 NOP64

#define SETUP                                                                                             \
    "v_mov_b32 v0, 0x01010101\n v_mov_b32 v1, 0x01010101\n v_mov_b32 v2, 0x01010101\n v_mov_b32 v3, 0x01010101\n" \
    "v_mov_b32 v4, 0x01010101\n v_mov_b32 v5, 0x01010101\n v_mov_b32 v6, 0x01010101\n v_mov_b32 v7, 0x01010101\n" \
    "v_mov_b32 v8, 0\n v_mov_b32 v9, 0\n v_mov_b32 v10, 0\n v_mov_b32 v11, 0\n v_mov_b32 v12, 0\n"                  \
    "v_mov_b32 v13, 0\n v_mov_b32 v14, 0\n v_mov_b32 v15, 0\n v_mov_b32 v16, 0\n v_mov_b32 v17, 0\n"                \
    "v_mov_b32 v18, 0\n v_mov_b32 v19, 0\n v_mov_b32 v20, 0\n v_mov_b32 v21, 0\n v_mov_b32 v22, 0\n"                \
    "v_mov_b32 v23, 0\n" NOP64

#define READOUT                                                                                           \
    "v_mov_b32 %15, v23\n v_mov_b32 %14, v22\n v_mov_b32 %13, v21\n v_mov_b32 %12, v20\n"                    \
    "v_mov_b32 %11, v19\n v_mov_b32 %10, v18\n v_mov_b32 %9, v17\n v_mov_b32 %8, v16\n"                      \
    "v_mov_b32 %7, v15\n v_mov_b32 %6, v14\n v_mov_b32 %5, v13\n v_mov_b32 %4, v12\n"                        \
    "v_mov_b32 %3, v11\n v_mov_b32 %2, v10\n v_mov_b32 %1, v9\n v_mov_b32 %0, v8\n"

#define OUTS                                                                                              \
    "=v"(r[0]), "=v"(r[1]), "=v"(r[2]), "=v"(r[3]), "=v"(r[4]), "=v"(r[5]), "=v"(r[6]), "=v"(r[7]), "=v"(r[8]), \
        "=v"(r[9]), "=v"(r[10]), "=v"(r[11]), "=v"(r[12]), "=v"(r[13]), "=v"(r[14]), "=v"(r[15])
#define CLOB                                                                                              \
    "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15", "v16",  \
        "v17", "v18", "v19", "v20", "v21", "v22", "v23"

#define MFMA "v_mfma_i32_32x32x32_i8 v[8:23], v[0:3], v[4:7], v[8:23]\n"
#define ONES_A "v_mov_b32 v0, 0x01010101\n v_mov_b32 v1, 0x01010101\n v_mov_b32 v2, 0x01010101\n v_mov_b32 v3, 0x01010101\n"
#define ONES_B "v_mov_b32 v4, 0x01010101\n v_mov_b32 v5, 0x01010101\n v_mov_b32 v6, 0x01010101\n v_mov_b32 v7, 0x01010101\n"
#define ZA "v_mov_b32 v0, 0\n v_mov_b32 v1, 0\n v_mov_b32 v2, 0\n v_mov_b32 v3, 0\n"
#define ZB "v_mov_b32 v4, 0\n v_mov_b32 v5, 0\n v_mov_b32 v6, 0\n v_mov_b32 v7, 0\n"

// background MFMA stream of the other waves (independent accumulator v[24:39]) before the measured MFMA
#define BG8 "v_mfma_i32_32x32x32_i8 v[24:39], v[0:3], v[4:7], v[24:39]\n"
#define BG BG8 BG8 BG8 BG8 BG8 BG8 BG8 BG8
#define CLOB2 CLOB, "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31", "v32", "v33", "v34", "v35", "v36", "v37", \
              "v38", "v39"

// fp64 VALU stream (64 dependent-free FMAs on v[40:47]) for the odd waves of the VALU-loaded case
#define F8 "v_fma_f64 v[40:41], v[42:43], v[44:45], v[40:41]\n v_fma_f64 v[46:47], v[42:43], v[44:45], v[46:47]\n" \
           "v_fma_f64 v[40:41], v[42:43], v[44:45], v[40:41]\n v_fma_f64 v[46:47], v[42:43], v[44:45], v[46:47]\n" \
           "v_fma_f64 v[40:41], v[42:43], v[44:45], v[40:41]\n v_fma_f64 v[46:47], v[42:43], v[44:45], v[46:47]\n" \
           "v_fma_f64 v[40:41], v[42:43], v[44:45], v[40:41]\n v_fma_f64 v[46:47], v[42:43], v[44:45], v[46:47]\n"
#define F64 F8 F8 F8 F8 F8 F8 F8 F8
#define CLOB3 CLOB2, "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47"

// W = wait string between the MFMA and the action
#define KERNELS(TAG, W)                                                                                   \
    __global__ void k_raw_##TAG(int* out) {                                                               \
        int r[16];                                                                                        \
        asm volatile(SETUP MFMA W READOUT : OUTS : : CLOB);                                               \
        for (int i = 0; i < 16; ++i) out[threadIdx.x * 16 + i] = r[i];                                    \
    }                                                                                                     \
    __global__ void k_wara_##TAG(int* out) {                                                              \
        int r[16];                                                                                        \
        asm volatile(SETUP MFMA W ZA LONGWAIT READOUT : OUTS : : CLOB);                                   \
        for (int i = 0; i < 16; ++i) out[threadIdx.x * 16 + i] = r[i];                                    \
    }                                                                                                     \
    __global__ void k_rawl_##TAG(int* out) {                                                              \
        int r[16];                                                                                        \
        asm volatile(SETUP "v_mov_b32 v24, 0\n" BG MFMA W READOUT : OUTS : : CLOB2);                        \
        for (int i = 0; i < 16; ++i) out[(blockIdx.x * blockDim.x + threadIdx.x) * 16 + i] = r[i];         \
    }                                                                                                     \
    __global__ void k_opwa_##TAG(int* out) {                                                              \
        int r[16];                                                                                        \
        asm volatile(SETUP ZA NOP64 "v_mov_b32 v24, 0\n" BG ONES_A W MFMA LONGWAIT READOUT : OUTS : : CLOB2);    \
        for (int i = 0; i < 16; ++i) out[(blockIdx.x * blockDim.x + threadIdx.x) * 16 + i] = r[i];         \
    }                                                                                                     \
    __global__ void k_opwb_##TAG(int* out) {                                                              \
        int r[16];                                                                                        \
        asm volatile(SETUP ZB NOP64 "v_mov_b32 v24, 0\n" BG ONES_B W MFMA LONGWAIT READOUT : OUTS : : CLOB2);    \
        for (int i = 0; i < 16; ++i) out[(blockIdx.x * blockDim.x + threadIdx.x) * 16 + i] = r[i];         \
    }                                                                                                     \
    __global__ void k_chain_##TAG(int* out) {                                                             \
        int r[16];                                                                                        \
        asm volatile(SETUP "v_mov_b32 v24, 0\n" BG MFMA W MFMA LONGWAIT READOUT : OUTS : : CLOB2);            \
        for (int i = 0; i < 16; ++i) out[(blockIdx.x * blockDim.x + threadIdx.x) * 16 + i] = r[i] - 32;    \
    }                                                                                                     \
    __global__ void k_rawv_##TAG(int* out) {                                                              \
        int r[16];                                                                                        \
        if ((threadIdx.x >> 6) & 1) {                                                                     \
            asm volatile("v_mov_b32 v42, 0\n v_mov_b32 v43, 0\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n"       \
                         "v_mov_b32 v40, 0\n v_mov_b32 v41, 0\n v_mov_b32 v46, 0\n v_mov_b32 v47, 0\n"        \
                         F64 F64 F64 F64 ::: CLOB3);                                                      \
            for (int i = 0; i < 16; ++i) r[i] = 32;                                                       \
        } else {                                                                                          \
            asm volatile(SETUP "v_mov_b32 v24, 0\n" BG BG MFMA W READOUT : OUTS : : CLOB2);                 \
        }                                                                                                 \
        for (int i = 0; i < 16; ++i) out[(blockIdx.x * blockDim.x + threadIdx.x) * 16 + i] = r[i];         \
    }                                                                                                     \
    __global__ void k_warqa_##TAG(int* out) {                                                             \
        int r[16];                                                                                        \
        asm volatile(SETUP "v_mov_b32 v24, 0\n" BG8 MFMA W ZA LONGWAIT READOUT : OUTS : : CLOB2);            \
        for (int i = 0; i < 16; ++i) out[(blockIdx.x * blockDim.x + threadIdx.x) * 16 + i] = r[i];         \
    }                                                                                                     \
    __global__ void k_warqb_##TAG(int* out) {                                                             \
        int r[16];                                                                                        \
        asm volatile(SETUP "v_mov_b32 v24, 0\n" BG8 MFMA W ZB LONGWAIT READOUT : OUTS : : CLOB2);            \
        for (int i = 0; i < 16; ++i) out[(blockIdx.x * blockDim.x + threadIdx.x) * 16 + i] = r[i];         \
    }                                                                                                     \
    __global__ void k_warb_##TAG(int* out) {                                                              \
        int r[16];                                                                                        \
        asm volatile(SETUP MFMA W ZB LONGWAIT READOUT : OUTS : : CLOB);                                   \
        for (int i = 0; i < 16; ++i) out[threadIdx.x * 16 + i] = r[i];                                    \
    }

KERNELS(0, "")
KERNELS(1, NOP1)
KERNELS(2, NOP1 NOP1)
KERNELS(4, "s_nop 3\n")
KERNELS(8, NOP8)
KERNELS(12, NOP8 "s_nop 3\n")
KERNELS(16, NOP8 NOP8)
KERNELS(24, NOP8 NOP8 NOP8)
KERNELS(32, NOP8 NOP8 NOP8 NOP8)
KERNELS(48, NOP8 NOP8 NOP8 NOP8 NOP8 NOP8)
KERNELS(64, NOP64)
KERNELS(96, NOP64 NOP8 NOP8 NOP8 NOP8)
KERNELS(128, NOP64 NOP64)

typedef void (*kfn)(int*);
struct Case {
    int n;
    kfn raw, wara, warb, rawl, opwa, opwb, chain, rawv, warqa, warqb;
};
#define CASE(T) \
    {T, k_raw_##T, k_wara_##T, k_warb_##T, k_rawl_##T, k_opwa_##T, k_opwb_##T, k_chain_##T, k_rawv_##T, k_warqa_##T, k_warqb_##T}

static void report(const char* what, int n, const int* h, int nw = 1) {
    int bad = 0, badrow[32] = {0}, badreg[16] = {0};
    for (int l = 0; l < 64 * nw; ++l)
        for (int i = 0; i < 16; ++i)
            if (h[l * 16 + i] != 32) {
                ++bad;
                badreg[i]++;
                badrow[(i & 3) + 8 * (i >> 2) + 4 * ((l & 63) >> 5)]++;
            }
    printf("%-6s N=%3d  wrong %6d / %d", what, n, bad, 1024 * nw);
    if (bad) {
        printf("  rows:");
        for (int a = 0; a < 32; ++a)
            if (badrow[a]) printf(" %d", a);
        printf("  sample %d", h[63 * 16 + 15]);
    }
    printf("\n");
}

int main() {
    Case cases[] = {CASE(0), CASE(1), CASE(2), CASE(4), CASE(8), CASE(12), CASE(16), CASE(24), CASE(32), CASE(48),
                    CASE(64), CASE(96), CASE(128)};
    const int nw = 16 * 256;  // 256 blocks of 16 waves: 4 waves per SIMD on every CU
    int* d;
    hipMalloc(&d, (size_t)64 * 16 * nw * sizeof(int));
    static int h[64 * 16 * 16 * 256];
    for (int rep = 0; rep < 2; ++rep)
        for (const Case& c : cases) {
            kfn fs[5] = {c.raw, c.wara, c.warb, c.warqa, c.warqb};
            const char* names[5] = {"RAW", "WAR-A", "WAR-B", "WARQ-A", "WARQ-B"};
            for (int k = 0; k < 5; ++k) {
                hipMemset(d, 0xff, 64 * 16 * sizeof(int));
                hipLaunchKernelGGL(fs[k], dim3(1), dim3(64), 0, 0, d);
                hipMemcpy(h, d, 64 * 16 * sizeof(int), hipMemcpyDeviceToHost);
                report(names[k], c.n, h);
            }
            kfn ls[7] = {c.rawl, c.opwa, c.opwb, c.chain, c.rawv, c.warqa, c.warqb};
            const char* lnames[7] = {"RAW-4w", "OPWA4w", "OPWB4w", "CHN-4w", "RAW-VA", "WARQA4", "WARQB4"};
            for (int k = 0; k < 7; ++k) {
                hipMemset(d, 0xff, sizeof(h));
                hipLaunchKernelGGL(ls[k], dim3(256), dim3(1024), 0, 0, d);
                hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
                report(lnames[k], c.n, h, nw);
            }
        }
    hipFree(d);
    return 0;
}

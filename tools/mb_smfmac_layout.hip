// Operand layout of v_smfmac_i32_32x32x64_i8 on gfx950, found by probing: B's byte j of lane l holds the code
// 1 + j + 32 (l >> 5) in every column; A is zero except one compressed byte = 1 in one lane, with the given index
// word, so every nonzero output names the B byte the A byte met, and the output's row names A's row.
// Then a random full check of the model the probes give.
// build: hipcc --offload-arch=gfx950 -O3 -o build/mb_smfmac_layout tools/mb_smfmac_layout.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef int i32x16 __attribute__((ext_vector_type(16)));

__global__ void k_sm(const int* a, const int* b, const int* idx, int* d) {
    const int l = threadIdx.x;
    i32x4 A = {a[4 * l], a[4 * l + 1], a[4 * l + 2], a[4 * l + 3]};
    i32x8 B;
    for (int k = 0; k < 8; ++k) B[k] = b[8 * l + k];
    i32x16 D = {};
    D = __builtin_amdgcn_smfmac_i32_32x32x64_i8(A, B, D, idx[l], 0, 0);
    for (int i = 0; i < 16; ++i) d[16 * l + i] = D[i];
}

static int ha[64 * 4], hb[64 * 8], hi[64], hd[64 * 16];
static int *da, *db, *di, *dd;
static void run() {
    hipMemcpy(da, ha, sizeof ha, hipMemcpyHostToDevice);
    hipMemcpy(db, hb, sizeof hb, hipMemcpyHostToDevice);
    hipMemcpy(di, hi, sizeof hi, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_sm, dim3(1), dim3(64), 0, 0, da, db, di, dd);
    hipMemcpy(hd, dd, sizeof hd, hipMemcpyDeviceToHost);
}

int main() {
    hipMalloc(&da, sizeof ha);
    hipMalloc(&db, sizeof hb);
    hipMalloc(&di, sizeof hi);
    hipMalloc(&dd, sizeof hd);
    for (int l = 0; l < 64; ++l)
        for (int j = 0; j < 32; ++j) {
            const int code = 1 + j + 32 * (l >> 5);
            hb[8 * l + j / 4] = (int)(((uint32_t)hb[8 * l + j / 4] & ~(0xffu << (8 * (j % 4)))) | ((uint32_t)code << (8 * (j % 4))));
        }
    for (int la = 0; la < 64; la += 32)  // lanes 0 and 32 (row 0, both halves)
        for (int jb = 0; jb < 16; ++jb)
            for (int ixv = 0; ixv < 2; ++ixv) {
                for (int i = 0; i < 64 * 4; ++i) ha[i] = 0;
                ha[4 * la + jb / 4] = 1 << (8 * (jb % 4));
                const uint32_t word = ixv == 0 ? 0x44444444u : 0xEEEEEEEEu;  // groups (0,1) or (2,3)
                for (int l = 0; l < 64; ++l) hi[l] = (int)word;
                run();
                printf("A lane %2d byte %2d idx %08x ->", la, jb, word);
                int shown = 0;
                for (int l = 0; l < 64 && shown < 4; ++l)
                    for (int i = 0; i < 16; ++i)
                        if (hd[16 * l + i] != 0 && shown < 4) {
                            const int row = 8 * (i >> 2) + 4 * (l >> 5) + (i & 3), col = l & 31;
                            const int code = hd[16 * l + i] - 1;
                            printf("  D[%d][%d]=B(h%d,byte %d)", row, col, code / 32, code % 32);
                            ++shown;
                        }
                printf("\n");
            }
    return 0;
}

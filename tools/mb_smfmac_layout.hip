// Operand layout of v_smfmac_i32_32x32x64_i8 on gfx950, checked against host models: D (32x32) += A (32x64,
// 2:4 sparse, compressed to 32x32) x B (64x32). Lane l, row/col = l & 31, half h = l >> 5.
//   model 0: A's 16 compressed bytes of lane l cover logical K = 32h .. 32h+31 (group g = bytes 2g, 2g+1 at the
//            positions of index bits [4g+1:4g], [4g+3:4g+2]); B's 32 bytes of lane l are K = 32h .. 32h+31.
//   model 1: as 0, but lane l's bytes are K = 16h .. 16h+15 (first half) and 32+16h .. 32+16h+15 (second half).
// D layout as the dense 32x32 MFMA: register i of lane l is row 8 (i >> 2) + 4 h + (i & 3), column l & 31.
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

static int8_t byte_of(const int* w, int i) { return (int8_t)((uint32_t)w[i / 4] >> (8 * (i % 4))); }

int main() {
    int ha[64 * 4], hb[64 * 8], hi[64], hd[64 * 16];
    srand(12345);
    for (int i = 0; i < 64 * 4; ++i) ha[i] = rand() ^ (rand() << 16);
    for (int i = 0; i < 64 * 8; ++i) hb[i] = rand() ^ (rand() << 16);
    for (int l = 0; l < 64; ++l) {  // random valid index pairs (i0 < i1) per group
        uint32_t w = 0;
        for (int g = 0; g < 8; ++g) {
            int i0 = rand() % 3, i1 = i0 + 1 + rand() % (3 - i0);
            w |= (uint32_t)(i0 | (i1 << 2)) << (4 * g);
        }
        hi[l] = (int)w;
    }
    int *da, *db, *di, *dd;
    hipMalloc(&da, sizeof ha);
    hipMalloc(&db, sizeof hb);
    hipMalloc(&di, sizeof hi);
    hipMalloc(&dd, sizeof hd);
    hipMemcpy(da, ha, sizeof ha, hipMemcpyHostToDevice);
    hipMemcpy(db, hb, sizeof hb, hipMemcpyHostToDevice);
    hipMemcpy(di, hi, sizeof hi, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_sm, dim3(1), dim3(64), 0, 0, da, db, di, dd);
    hipMemcpy(hd, dd, sizeof hd, hipMemcpyDeviceToHost);
    for (int model = 0; model < 2; ++model) {
        // dense logical A[32][64], B[64][32]
        static int LA[32][64], LB[64][32];
        for (int r = 0; r < 32; ++r)
            for (int k = 0; k < 64; ++k) LA[r][k] = 0;
        for (int l = 0; l < 64; ++l) {
            const int r = l & 31, h = l >> 5;
            for (int g = 0; g < 8; ++g) {
                const uint32_t ix = (uint32_t)hi[l] >> (4 * g);
                const int p0 = ix & 3, p1 = (ix >> 2) & 3;
                int kbase;
                if (model == 0) kbase = 32 * h + 4 * g;
                else kbase = (g < 4 ? 16 * h : 32 + 16 * h) + 4 * (g % 4);
                LA[r][kbase + p0] = byte_of(&ha[4 * l], 2 * g);
                LA[r][kbase + p1] = byte_of(&ha[4 * l], 2 * g + 1);
            }
            for (int j = 0; j < 32; ++j) {
                int k;
                if (model == 0) k = 32 * h + j;
                else k = (j < 16 ? 16 * h : 32 + 16 * h) + (j % 16);
                LB[k][r] = byte_of(&hb[8 * l], j);
            }
        }
        long bad = 0;
        for (int l = 0; l < 64; ++l)
            for (int i = 0; i < 16; ++i) {
                const int row = 8 * (i >> 2) + 4 * (l >> 5) + (i & 3), col = l & 31;
                long s = 0;
                for (int k = 0; k < 64; ++k) s += (long)LA[row][k] * LB[k][col];
                bad += s != hd[16 * l + i];
            }
        printf("model %d: %ld of 1024 outputs differ\n", model, bad);
    }
    return 0;
}

// Accuracy of the f16 hi/lo split complex product on v_mfma_f32_32x32x16_f16 vs the f32-input MFMA,
// against an fp64 host sum of the same fp32 operands. One wave: a 32x32 tile, P photon pairs.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <random>
#include <vector>
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
__device__ inline uint32_t pk16(_Float16 a, _Float16 b) { f16x2 v = {a, b}; return __builtin_bit_cast(uint32_t, v); }
__device__ inline f16x8 frag(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    typedef uint32_t u4 __attribute__((ext_vector_type(4))); u4 v = {a, b, c, d}; return __builtin_bit_cast(f16x8, v);
}
// mode 0: f32 MFMA; 1: f16 4-term split; 2: f16 split with hi only (no lo); 3: 4-term, lo scaled in separate acc
__global__ void k(const float* U, const float* V, int P, int mode, float scale, int sq, float* out) {
    const int l = threadIdx.x, a = l & 31, h = l >> 5;
    f32x16 re = {}, im = {}, re2 = {}, im2 = {};
    for (int q = 0; q < P; ++q) {
        const int ph = 2 * q + h;
        float uc = U[(ph * 32 + a) * 2] * scale, us = U[(ph * 32 + a) * 2 + 1] * scale;
        float vc = V[(ph * 32 + a) * 2] * scale, vs = V[(ph * 32 + a) * 2 + 1] * scale;
        if (sq) {  // harmonic 2 by squaring, as the search kernel forms it
            const float inv = 1.0f / scale;
            const float c2u = __builtin_fmaf(uc, uc * inv, -(us * inv) * us), s2u = (2.0f * inv * uc) * us;
            const float c2v = __builtin_fmaf(vc, vc * inv, -(vs * inv) * vs), s2v = (2.0f * inv * vc) * vs;
            uc = c2u; us = s2u; vc = c2v; vs = s2v;
        }
        if (mode == 0) {
            re = __builtin_amdgcn_mfma_f32_32x32x2f32(uc, vc, re, 0, 0, 0);
            im = __builtin_amdgcn_mfma_f32_32x32x2f32(us, vc, im, 0, 0, 0);
            re = __builtin_amdgcn_mfma_f32_32x32x2f32(us, -vs, re, 0, 0, 0);
            im = __builtin_amdgcn_mfma_f32_32x32x2f32(uc, vs, im, 0, 0, 0);
        } else {
            _Float16 uch = (_Float16)uc, ush = (_Float16)us, vch = (_Float16)vc, vsh = (_Float16)vs;
            _Float16 ucl = (_Float16)(uc - (float)uch), usl = (_Float16)(us - (float)ush);
            _Float16 vcl = (_Float16)(vc - (float)vch), vsl = (_Float16)(vs - (float)vsh);
            if (mode == 2) ucl = usl = vcl = vsl = (_Float16)0.0f;
            uint32_t a0 = pk16(uch, uch), a1 = pk16(ucl, ucl), a2 = pk16(ush, ush), a3 = pk16(usl, usl);
            uint32_t bc = pk16(vch, vcl), bs = pk16(vsh, vsl), bn = bs ^ 0x80008000u;
            re = __builtin_amdgcn_mfma_f32_32x32x16_f16(frag(a0, a1, a2, a3), frag(bc, bc, bn, bn), re, 0, 0, 0);
            im = __builtin_amdgcn_mfma_f32_32x32x16_f16(frag(a2, a3, a0, a1), frag(bc, bc, bs, bs), im, 0, 0, 0);
        }
    }
    for (int r = 0; r < 16; ++r) {
        const int row = (r & 3) + 8 * (r >> 2) + 4 * h;   // a
        const int col = a;                                 // b
        out[(row * 32 + col) * 2] = re[r] / (scale * scale);
        out[(row * 32 + col) * 2 + 1] = im[r] / (scale * scale);
    }
}
int main() {
    const int P = 16;  // 32 photons
    std::mt19937_64 g(1);
    std::uniform_real_distribution<double> u(0, 1);
    std::vector<float> U(2 * P * 32 * 2), V(2 * P * 32 * 2);
    for (int i = 0; i < 2 * P * 32; ++i) {
        double t = 2 * M_PI * u(g), s = 2 * M_PI * u(g);
        U[2 * i] = (float)cos(t); U[2 * i + 1] = (float)sin(t);
        V[2 * i] = (float)cos(s); V[2 * i + 1] = (float)sin(s);
    }
    float *dU, *dV, *dO;
    (void)hipMalloc(&dU, U.size() * 4); (void)hipMalloc(&dV, V.size() * 4); (void)hipMalloc(&dO, 32 * 32 * 2 * 4);
    (void)hipMemcpy(dU, U.data(), U.size() * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(dV, V.data(), V.size() * 4, hipMemcpyHostToDevice);
    const char* names[] = {"f32 mfma", "f16 split 4-term", "f16 hi only"};
    for (int sq = 0; sq < 2; ++sq) {
        printf("---- %s\n", sq ? "harmonic 2 (squared operands)" : "harmonic 1");
        std::vector<double> ref(32 * 32 * 2, 0.0);
        for (int a = 0; a < 32; ++a)
            for (int b = 0; b < 32; ++b)
                for (int p = 0; p < 2 * P; ++p) {
                    // reference from the fp32 operands the kernel squares (fp64 arithmetic)
                    double uc = U[(p * 32 + a) * 2], us = U[(p * 32 + a) * 2 + 1];
                    double vc = V[(p * 32 + b) * 2], vs = V[(p * 32 + b) * 2 + 1];
                    if (sq) {
                        double c2u = uc * uc - us * us, s2u = 2 * uc * us, c2v = vc * vc - vs * vs, s2v = 2 * vc * vs;
                        uc = c2u; us = s2u; vc = c2v; vs = s2v;
                    }
                    ref[(a * 32 + b) * 2] += uc * vc - us * vs;
                    ref[(a * 32 + b) * 2 + 1] += us * vc + uc * vs;
                }
        for (int mode = 0; mode < 3; ++mode)
            for (float sc : {1.0f, 4096.0f}) {
                k<<<1, 64>>>(dU, dV, P, mode, sc, sq, dO);
                std::vector<float> o(32 * 32 * 2);
                (void)hipMemcpy(o.data(), dO, o.size() * 4, hipMemcpyDeviceToHost);
                double mx = 0, rms = 0, bias = 0;
                for (size_t i = 0; i < o.size(); ++i) {
                    double e = o[i] - ref[i];
                    mx = fmax(mx, fabs(e)); rms += e * e; bias += e;
                }
                printf("%-18s scale %6.0f: max abs err %.3e  rms %.3e  mean %.3e\n", names[mode], sc, mx,
                       sqrt(rms / o.size()), bias / o.size());
            }
    }
    return 0;
}

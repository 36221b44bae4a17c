// search_mfma16.h -- factorised periodicity search on the f16 matrix cores, fp32-exact via hi/lo split.
//
// Same factorisation as search_mfma.h: a 1024-trial tile j = c0 + a + 32*b of an arithmetic-progression
// grid has exp(2*pi*i*k*f_j*dt) = U_a * V_b, so the harmonic sums are complex matrix products over
// photons. Here every fp32 operand x is carried as two f16 values, hi = RN_f16(x), lo = RN_f16(x - hi)
// (|x - hi - lo| <= 2^-22 |x|; f16 denormals are honoured by the conversions and the MFMA), and the four
// exact products hi.hi + hi.lo + lo.hi + lo.lo of each real product fill the K = 16 of one
// v_mfma_f32_32x32x16_f16 together with the complex structure:
//   lane (a, h) holds the 8 K-values of photon 2q+h;
//   A (U side, shared by both MFMAs) = [uc_h us_h | uc_l us_l | uc_l us_l | uc_h us_h]
//   B_re = [vc_h -vs_h | vc_l -vs_l | vc_h -vs_h | vc_l -vs_l]  -> Re += uc.vc - us.vs
//   B_im = [vs_h  vc_h | vs_l  vc_l | vs_h  vc_h | vs_l  vc_l]  -> Im += uc.vs + us.vc
//   (every K pair is one dword, so A costs one conversion and two fma_mix; CRIMP_SPLIT_DUP builds the
//   earlier [uc_h uc_h | uc_l uc_l | ...] layout)
// so one photon pair and harmonic costs two 32-cycle MFMAs (the f32-input form needs four 64-cycle
// ones), the products are exact in the fp32 accumulator, and the result matches the f32 path.
//
// TILES > 1: one wave owns TILES tiles that share the V_b factors (one sin/cos of V per photon for
// TILES tiles); the extra accumulators need the whole register file, so such waves run one per SIMD.
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// sin/cos(2*pi*r), |r| <= 1/2 turn: quarter-turn reduction r = q/4 + y (|y| <= 1/8), minimax
// polynomials (degree 7 / 8, fit error 1.2e-9 / 5e-11, fp32 evaluation 9e-8 / 6e-8), then the exact
// rotation by i^q with cos(q pi/2) = 1 - |q|, sin(q pi/2) = q (2 - |q|) for q in {-2..2}.
__device__ __forceinline__ void sincos_turn(float r, float& s, float& c) {
    const float q = __builtin_rintf(4.0f * r);
    const float y = __builtin_fmaf(-0.25f, q, r);
    const float y2 = y * y;
    float sp = __builtin_fmaf(y2, -75.24005889892578f, 81.58812713623047f);
    sp = __builtin_fmaf(y2, sp, -41.34162902832031f);
    sp = __builtin_fmaf(y2, sp, 6.283185005187988f);
    sp *= y;
    float cp = __builtin_fmaf(y2, 59.220401763916016f, -85.4428482055664f);
    cp = __builtin_fmaf(y2, cp, 64.93931579589844f);
    cp = __builtin_fmaf(y2, cp, -19.739208221435547f);
    cp = __builtin_fmaf(y2, cp, 1.0f);
    const float aq = __builtin_fabsf(q);
    const float cq = 1.0f - aq, sq = q * (2.0f - aq);
    s = __builtin_fmaf(sp, cq, cp * sq);
    c = __builtin_fmaf(cp, cq, -(sp * sq));
}

__device__ __forceinline__ float frac_turn(double ph) { return (float)(ph - rint(ph)); }

// Splits in explicit instructions (the compiler's own choice re-derives hi for every use and, left
// alone, may fuse the producing multiply into one conversion but not the other, so that hi + lo != x).
// P(h, h) = cvt_pk(x, x) and P(l, l) with l = RN_f16(x - h) straight from v_fma_mix (f32 x, f16 h).
__device__ __forceinline__ void split_aa(float x, uint32_t& dh, uint32_t& dl) {
    asm volatile(
        "v_cvt_pk_f16_f32 %0, %2, %2\n\t"
        "v_fma_mixlo_f16 %1, %2, 1.0, -%0 op_sel_hi:[0,0,1]\n\t"
        "v_fma_mixhi_f16 %1, %2, 1.0, -%0 op_sel_hi:[0,0,1]"
        : "=&v"(dh), "=&v"(dl)
        : "v"(x));
}
// P(h, l)
__device__ __forceinline__ uint32_t split_b(float x) {
    uint32_t d;
    asm volatile(
        "v_cvt_pk_f16_f32 %0, %1, %1\n\t"
        "v_fma_mixhi_f16 %0, %1, 1.0, -%0 op_sel_hi:[0,0,1]"
        : "=&v"(d)
        : "v"(x));
    return d;
}

// Two values at once: hi = (RN(x), RN(y)) in one conversion, lo = (RN(x - hi.x), RN(y - hi.y)); NEGY splits -y
// (the sign rides on the instructions' source modifiers, no extra negation).
template <bool NEGY>
__device__ __forceinline__ void split_xy(float x, float y, uint32_t& dh, uint32_t& dl) {
    if (NEGY)
        asm volatile(
            "v_cvt_pk_f16_f32 %0, %2, -%3\n\t"
            "v_fma_mixlo_f16 %1, %2, 1.0, -%0 op_sel_hi:[0,0,1]\n\t"
            "v_fma_mixhi_f16 %1, -%3, 1.0, -%0 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
            : "=&v"(dh), "=&v"(dl)
            : "v"(x), "v"(y));
    else
        asm volatile(
            "v_cvt_pk_f16_f32 %0, %2, %3\n\t"
            "v_fma_mixlo_f16 %1, %2, 1.0, -%0 op_sel_hi:[0,0,1]\n\t"
            "v_fma_mixhi_f16 %1, %3, 1.0, -%0 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
            : "=&v"(dh), "=&v"(dl)
            : "v"(x), "v"(y));
}

struct AFrag {
    f16x8 v;
};
struct BFrag {
    f16x8 re, im;
};

#ifdef CRIMP_SPLIT_DUP
// previous layout: A = [uc_h uc_h | uc_l uc_l | us_h us_h | us_l us_l] (6 instructions for A, 5 for B)
__device__ __forceinline__ AFrag make_a(float uc, float us) {
    uint32_t ch, cl, sh, sl;
    split_aa(uc, ch, cl);
    split_aa(us, sh, sl);
    return AFrag{__builtin_bit_cast(f16x8, u32x4{ch, cl, sh, sl})};
}
__device__ __forceinline__ BFrag make_b(float vc, float vs) {
    const uint32_t bc = split_b(vc), bs = split_b(vs), bn = bs ^ 0x80008000u;
    return BFrag{__builtin_bit_cast(f16x8, u32x4{bc, bc, bn, bn}), __builtin_bit_cast(f16x8, u32x4{bs, bs, bc, bc})};
}
#else
// Interleaved layout (3 instructions for A, 5 for B; A is built once per tile and harmonic, B once per photon pair).
// Dwords h = (uc_h, us_h), l = (uc_l, us_l), e_h = (vc_h, -vs_h), e_l = (vc_l, -vs_l), f_h = (vs_h, vc_h), f_l = (vs_l, vc_l):
//   A    = [h | l | l | h]
//   B_re = [e_h | e_l | e_h | e_l]   -> Re += uc.vc - us.vs (the four hi/lo products h.e_h, l.e_l, l.e_h, h.e_l)
//   B_im = [f_h | f_l | f_h | f_l]   -> Im += uc.vs + us.vc
__device__ __forceinline__ AFrag make_a(float uc, float us) {
    uint32_t h, l;
    split_xy<false>(uc, us, h, l);
    return AFrag{__builtin_bit_cast(f16x8, u32x4{h, l, l, h})};
}
// (a, -b) -> (b, a) in one packed multiply by (1, 1): halves swapped by op_sel, the sign by neg_lo (exact)
__device__ __forceinline__ uint32_t swap_neg_lo(uint32_t e) {
    uint32_t d;
    asm volatile("v_pk_mul_f16 %0, %1, %2 op_sel:[1,0] op_sel_hi:[0,1] neg_lo:[1,0]" : "=v"(d) : "v"(e), "v"(0x3C003C00u));
    return d;
}
__device__ __forceinline__ BFrag make_b(float vc, float vs) {
    uint32_t eh, el;
    split_xy<true>(vc, vs, eh, el);
    const uint32_t fh = swap_neg_lo(eh), fl = swap_neg_lo(el);
    return BFrag{__builtin_bit_cast(f16x8, u32x4{eh, el, eh, el}), __builtin_bit_cast(f16x8, u32x4{fh, fl, fh, fl})};
}
#endif

__device__ __forceinline__ void mma(const AFrag& A, const BFrag& B, f32x16& re, f32x16& im) {
    re = __builtin_amdgcn_mfma_f32_32x32x16_f16(A.v, B.re, re, 0, 0, 0);
    im = __builtin_amdgcn_mfma_f32_32x32x16_f16(A.v, B.im, im, 0, 0, 0);
}

// One photon pair: V factors once, then every tile's U factors and MFMAs. SQUARE groups are harmonic
// pairs (ka, 2 ka), the second by squaring the first (unbiased: the sin/cos error is quarter-turn
// periodic); other groups evaluate each of their harmonics (ka, kb) from its own fp64 phase.
// Table sin/cos (CRIMP_SINCOS_TABLE): r = k/1024 + y, |y| <= 1/2048 turn; (cos, sin)(2 pi k/1024) from a
// 1024-entry LDS table held as fp32 hi + lo pairs (tab[k] = hi, tab[1024 + k] = lo), the residual rotation by
// sin(2 pi y) ~ 2 pi y - (2 pi y)^3/6 and cos(2 pi y) - 1 ~ -(2 pi y)^2/2 (truncation < 4e-12), combined so
// that only the final fp32 rounding remains (16 VALU + 2 LDS reads instead of 19 VALU).
__device__ __forceinline__ void sincos_tab(const float2* __restrict__ tab, float r, float& s, float& c) {
    const float kf = __builtin_rintf(1024.0f * r);
    const float y = __builtin_fmaf(-1.0f / 1024.0f, kf, r);  // exact
    const int k = ((int)kf) & 1023;
    const float2 th = tab[k], tl = tab[1024 + k];
    const float y2 = y * y;
    const float sp = y * __builtin_fmaf(y2, -41.341702240399755f, 6.283185307179586f);
    const float cm = y2 * -19.739208802178716f;
    s = th.y + __builtin_fmaf(th.y, cm, __builtin_fmaf(th.x, sp, tl.y));
    c = th.x + __builtin_fmaf(th.x, cm, __builtin_fmaf(-th.y, sp, tl.x));
}

__device__ __forceinline__ void sc_rev(const float2* __restrict__ tab, float r, float& s, float& c) {
#ifdef CRIMP_SINCOS_TABLE
    sincos_tab(tab, r, s, c);
#else
    (void)tab;
    sincos_turn(r, s, c);
#endif
}

template <int G, int TILES, bool SQUARE>
__device__ __forceinline__ void mfma16_pair(const float2* tab, const double (&phu)[TILES], double phv, float live,
                                            int ka, int kb, f32x16 (&re)[TILES][G], f32x16 (&im)[TILES][G]) {
    if (SQUARE) {  // harmonics (ka, 2 ka): phases arrive pre-scaled by ka
        float vs, vc;
        sc_rev(tab, frac_turn(phv), vs, vc);
        BFrag B1 = make_b(vc, vs), B2;
        if (G > 1) B2 = make_b(__builtin_fmaf(vc, vc, -(vs * vs)), (vc + vc) * vs);
#pragma unroll
        for (int t = 0; t < TILES; ++t) {
            float us, uc;
            sc_rev(tab, frac_turn(phu[t]), us, uc);
            uc *= live;
            us *= live;
            mma(make_a(uc, us), B1, re[t][0], im[t][0]);
            if (G > 1) mma(make_a(__builtin_fmaf(uc, uc, -(us * us)), (uc + uc) * us), B2, re[t][1], im[t][1]);
        }
    } else {
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const double kf = (double)(g == 0 ? ka : kb);
            float vs, vc;
            sc_rev(tab, frac_turn(phv * kf), vs, vc);
            const BFrag B = make_b(vc, vs);
#pragma unroll
            for (int t = 0; t < TILES; ++t) {
                float us, uc;
                sc_rev(tab, frac_turn(phu[t] * kf), us, uc);
                mma(make_a(uc * live, us * live), B, re[t][g], im[t][g]);
            }
        }
    }
}

template <int G, bool TWOD, bool SQUARE, int TILES>
__global__ __launch_bounds__(256, TILES == 1 ? 2 : 1) void k_search_mfma16(
    const double* __restrict__ dt, const double* __restrict__ dt2, int64_t n, int64_t chunk,
    const double* __restrict__ freq, int64_t nf, const double* __restrict__ c2row, double delta,
    int64_t tile_first, int64_t ntiles, int64_t tiles_per_row, int64_t first, int64_t count, int ka, int kb,
    int ncomp, double* __restrict__ part) {
    const int lane = threadIdx.x & 63;
    const int64_t T = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
#ifdef CRIMP_SINCOS_TABLE
    __shared__ float2 s_tab[2048];
    for (int i = threadIdx.x; i < 1024; i += 256) {
        double sv, cv;
        sincospi((double)i / 512.0, &sv, &cv);
        const float ch = (float)cv, sh = (float)sv;
        s_tab[i] = make_float2(ch, sh);
        s_tab[1024 + i] = make_float2((float)(cv - (double)ch), (float)(sv - (double)sh));
    }
    __syncthreads();
    const float2* tab = s_tab;
#else
    const float2* tab = nullptr;
#endif
    if (T >= ntiles) return;  // wave-uniform
    const int64_t gt = tile_first + T;
    const int64_t frow = gt / tiles_per_row;
    const int64_t c0 = (gt - frow * tiles_per_row) * (kTile * TILES);
    const int a = lane & 31;
    const int h = lane >> 5;
    // SQUARE groups evaluate harmonic ka directly: scale the phase coefficients once (exact for ka = 1)
    const double ks = SQUARE ? (double)ka : 1.0;
    double fa[TILES];
#pragma unroll
    for (int t = 0; t < TILES; ++t) {
        const int64_t ca = c0 + t * kTile + a;
        fa[t] = freq[ca < nf ? ca : nf - 1] * ks;
    }
    const double gb = (double)(32 * a) * delta * ks;
    const double c2 = TWOD ? c2row[frow] * ks : 0.0;
    const int64_t split = blockIdx.y;
    const int64_t i0 = split * chunk;
    const int64_t i1 = i0 + chunk < n ? i0 + chunk : n;

    double Cr[TILES][G][16], Ci[TILES][G][16];
#pragma unroll
    for (int t = 0; t < TILES; ++t)
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int r = 0; r < 16; ++r) Cr[t][g][r] = Ci[t][g][r] = 0.0;

#ifndef CRIMP_NO_PREFETCH
    // the next chunk's photon times are loaded one chunk ahead (the global-load latency hides behind a chunk)
    double dtn = (i0 + a < i1) ? dt[i0 + a] : 0.0;
    double d2n = TWOD ? ((i0 + a < i1) ? dt2[i0 + a] : 0.0) : 0.0;
#endif
    for (int64_t ib = i0; ib < i1; ib += kMfmaChunk) {
        const int cnt = (int)(i1 - ib < kMfmaChunk ? i1 - ib : kMfmaChunk);
        // the chunk's photon times: one coalesced load; lane (a, h) then fetches photon 2q+h's
#ifndef CRIMP_NO_PREFETCH
        const double dtv = dtn, d2v = d2n;
        {
            const int64_t nb = ib + kMfmaChunk;
            dtn = (nb + a < i1) ? dt[nb + a] : 0.0;
            if (TWOD) d2n = (nb + a < i1) ? dt2[nb + a] : 0.0;
        }
#else
        const double dtv = a < cnt ? dt[ib + a] : 0.0;
        const double d2v = TWOD ? (a < cnt ? dt2[ib + a] : 0.0) : 0.0;
#endif
        f32x16 re[TILES][G], im[TILES][G];
#pragma unroll
        for (int t = 0; t < TILES; ++t)
#pragma unroll
            for (int g = 0; g < G; ++g)
#pragma unroll
                for (int r = 0; r < 16; ++r) re[t][g][r] = im[t][g][r] = 0.0f;
        auto pair = [&](int q, float live) {
            const int src = 2 * q + h;
#ifdef CRIMP_D_GLOBAL  // experiment: each lane loads its photon (L1/L2 hit) instead of a bpermute
            const double d = src < cnt ? dt[ib + src] : 0.0;
            const double d2 = TWOD ? (src < cnt ? dt2[ib + src] : 0.0) : 0.0;
#else
            const double d = bperm_d(dtv, src);
            const double d2 = TWOD ? bperm_d(d2v, src) : 0.0;
#endif
            double phu[TILES];
#pragma unroll
            for (int t = 0; t < TILES; ++t) phu[t] = TWOD ? fma(fa[t], d, c2 * d2) : fa[t] * d;
            mfma16_pair<G, TILES, SQUARE>(tab, phu, gb * d, live, ka, kb, re, im);
        };
        if (cnt == kMfmaChunk) {
#if !defined(CRIMP_NO_PREFETCH) && !defined(CRIMP_D_GLOBAL)
            // photon pair q+1's times are fetched (ds_bpermute) while pair q computes
            double dn = bperm_d(dtv, h), d2nn = TWOD ? bperm_d(d2v, h) : 0.0;
#pragma unroll
            for (int q = 0; q < kMfmaChunk / 2; ++q) {
                const double d = dn, d2 = d2nn;
                if (q + 1 < kMfmaChunk / 2) {
                    dn = bperm_d(dtv, 2 * (q + 1) + h);
                    if (TWOD) d2nn = bperm_d(d2v, 2 * (q + 1) + h);
                }
                __builtin_amdgcn_sched_barrier(0);  // keep the fetch ahead of this pair's arithmetic
                double phu[TILES];
#pragma unroll
                for (int t = 0; t < TILES; ++t) phu[t] = TWOD ? fma(fa[t], d, c2 * d2) : fa[t] * d;
                mfma16_pair<G, TILES, SQUARE>(tab, phu, gb * d, 1.0f, ka, kb, re, im);
            }
#else
#pragma unroll
            for (int q = 0; q < kMfmaChunk / 2; ++q) pair(q, 1.0f);
#endif
        } else {
            for (int q = 0; 2 * q < cnt; ++q) pair(q, 2 * q + h < cnt ? 1.0f : 0.0f);
        }
#pragma unroll
        for (int t = 0; t < TILES; ++t)
#pragma unroll
            for (int g = 0; g < G; ++g)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    Cr[t][g][r] += (double)re[t][g][r];
                    Ci[t][g][r] += (double)im[t][g][r];
                }
    }
    // D[row][col] of each 32x32 tile: col = lane&31 (b), row = (r&3) + 8*(r>>2) + 4*(lane>>5) (a)
#pragma unroll
    for (int t = 0; t < TILES; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int ra = (r & 3) + 8 * (r >> 2) + 4 * h;
            const int64_t c = c0 + t * kTile + ra + 32 * a;
            const int64_t o = frow * nf + c - first;
            if (c < nf && o >= 0 && o < count) {
#pragma unroll
                for (int g = 0; g < G; ++g) {
                    const int comp = 2 * ((g == 0 ? ka : kb) - 1);
                    part[(split * ncomp + comp) * count + o] = Cr[t][g][r];
                    part[(split * ncomp + comp + 1) * count + o] = Ci[t][g][r];
                }
            }
        }
}

template <bool TWOD, int TILES>
static void launch_mfma16(int G, bool square, dim3 grid, hipStream_t s, const double* dt, const double* dt2,
                          int64_t n, int64_t chunk, const double* fr, int64_t nf, const double* c2, double delta,
                          int64_t tf, int64_t nt, int64_t tpr, int64_t first, int64_t count, int ka, int kb, int ncomp,
                          double* part) {
#define CRIMP_LM16(GG, FF)                                                                                      \
    k_search_mfma16<GG, TWOD, FF, TILES><<<grid, 256, 0, s>>>(dt, dt2, n, chunk, fr, nf, c2, delta, tf, nt, tpr, \
                                                              first, count, ka, kb, ncomp, part)
    if (G == 2) {
        if (square) CRIMP_LM16(2, true); else CRIMP_LM16(2, false);
    } else {
        CRIMP_LM16(1, false);
    }
#undef CRIMP_LM16
}

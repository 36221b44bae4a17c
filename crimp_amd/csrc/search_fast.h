// search_fast.h -- the opt-in "fast" periodicity search (CRIMP_FLAG_FAST, PeriodSearch(precision="fast")):
// factorised harmonic sums on the f16 matrix cores, fp32-exact products via a hi/lo split, fp32 sin/cos.
// Accurate to ~1e-6 of the grid's mean power, not per trial (its per-term error is ~1e-7 against ~1e-9 for
// the default exact kernel of search_exact.h); kept for users who trade that for speed.
//
// For an arithmetic-progression grid a 1024-trial tile j = c0 + a + 32*b factorises:
// exp(2*pi*i*k*f_j*dt) = U_a * V_b with U_a = exp(2*pi*i*k*(f_{c0+a} dt + c2 dt^2)), V_b = exp(2*pi*i*k*(32*b*delta)*dt),
// so the harmonic sums are complex matrix products over photons. Every fp32 operand x is carried as two f16
// values, hi = RN_f16(x), lo = RN_f16(x - hi) (|x - hi - lo| <= 2^-22 |x|), and the four exact products
// hi.hi + hi.lo + lo.hi + lo.lo of each real product fill the K = 16 of one v_mfma_f32_32x32x16_f16:
//   lane (a, h) holds the 8 K-values of photon 2q+h;
//   A (U side, shared by both MFMAs) = [uc_h us_h | uc_l us_l | uc_l us_l | uc_h us_h]
//   B_re = [vc_h -vs_h | vc_l -vs_l | vc_h -vs_h | vc_l -vs_l]  -> Re += uc.vc - us.vs
//   B_im = [vs_h  vc_h | vs_l  vc_l | vs_h  vc_h | vs_l  vc_l]  -> Im += uc.vs + us.vc
// One photon pair and harmonic costs two 32-cycle MFMAs; chunks of 32 photons accumulate in fp32, then fold
// into fp64 per-split partial sums that k_search_finalize combines.
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kMfmaChunk = 32;
constexpr int kTile = 1024;

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

// lane-indexed fetch of a double held by lane `src` of the wave (ds_bpermute, LDS crossbar)
__device__ __forceinline__ double bperm_d(double v, int src) {
    const int lo = __builtin_amdgcn_ds_bpermute(src << 2, __double2loint(v));
    const int hi = __builtin_amdgcn_ds_bpermute(src << 2, __double2hiint(v));
    return __hiloint2double(hi, lo);
}

// Two values at once: hi = (RN(x), RN(y)) in one conversion, lo = (RN(x - hi.x), RN(y - hi.y)); NEGY splits -y.
// Explicit instructions: left alone, the compiler may fuse a producing multiply into one conversion but not the
// other, so that hi + lo != x (that bug gave 1e-5 errors on squared harmonics).
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

// A = [h | l | l | h] (3 instructions, once per tile and harmonic), B built once per photon pair (5 instructions).
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

__device__ __forceinline__ void mma(const AFrag& A, const BFrag& B, f32x16& re, f32x16& im) {
    re = __builtin_amdgcn_mfma_f32_32x32x16_f16(A.v, B.re, re, 0, 0, 0);
    im = __builtin_amdgcn_mfma_f32_32x32x16_f16(A.v, B.im, im, 0, 0, 0);
}

// One photon pair. SQUARE groups are harmonic pairs (ka, 2 ka), the second by squaring the first (unbiased: the
// sin/cos error is quarter-turn periodic); other groups evaluate each of their harmonics from its own fp64 phase.
template <int G, bool SQUARE>
__device__ __forceinline__ void fast_pair(double phu, double phv, float live, int ka, int kb, f32x16 (&re)[G],
                                          f32x16 (&im)[G]) {
    static_assert(G == 1 || G == 2, "harmonic groups of one or two");
    // all operands first, then the MFMAs as one group followed by the operand guard (mfma_drain.h)
    AFrag A[G];
    BFrag B[G];
    if (SQUARE) {  // harmonics (ka, 2 ka): phases arrive pre-scaled by ka
        float vs, vc, us, uc;
        sincos_turn(frac_turn(phv), vs, vc);
        B[0] = make_b(vc, vs);
        if (G > 1) B[G - 1] = make_b(__builtin_fmaf(vc, vc, -(vs * vs)), (vc + vc) * vs);
        sincos_turn(frac_turn(phu), us, uc);
        uc *= live;
        us *= live;
        A[0] = make_a(uc, us);
        if (G > 1) A[G - 1] = make_a(__builtin_fmaf(uc, uc, -(us * us)), (uc + uc) * us);
    } else {
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const double kf = (double)(g == 0 ? ka : kb);
            float vs, vc, us, uc;
            sincos_turn(frac_turn(phv * kf), vs, vc);
            B[g] = make_b(vc, vs);
            sincos_turn(frac_turn(phu * kf), us, uc);
            A[g] = make_a(uc * live, us * live);
        }
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int g = 0; g < G; ++g) mma(A[g], B[g], re[g], im[g]);
    mfma_operand_guard();
}

template <int G, bool TWOD, bool SQUARE>
__global__ __launch_bounds__(256, 2) void k_search_fast(
    const double* __restrict__ dt, const double* __restrict__ dt2, int64_t n, int64_t chunk,
    const double* __restrict__ freq, int64_t nf, const double* __restrict__ c2row, const double* __restrict__ apinfo,
    int64_t tile_first, int64_t ntiles, int64_t tiles_per_row, int64_t first, int64_t count, int ka, int kb,
    int ncomp, double* __restrict__ part) {
    const int lane = threadIdx.x & 63;
    const int64_t T = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (T >= ntiles) return;  // wave-uniform
    const int64_t gt = tile_first + T;
    const int64_t frow = gt / tiles_per_row;
    const int64_t c0 = (gt - frow * tiles_per_row) * kTile;
    const int a = lane & 31;
    const int h = lane >> 5;
    const double ks = SQUARE ? (double)ka : 1.0;  // SQUARE groups evaluate harmonic ka directly
    const int64_t ca = c0 + a;
    const double fa = freq[ca < nf ? ca : nf - 1] * ks;
    const double gb = (double)(32 * a) * apinfo[0] * ks;
    const double c2 = TWOD ? c2row[frow] * ks : 0.0;
    const int64_t split = blockIdx.y;
    const int64_t i0 = split * chunk;
    const int64_t i1 = i0 + chunk < n ? i0 + chunk : n;

    double Cr[G][16], Ci[G][16];
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
        for (int r = 0; r < 16; ++r) Cr[g][r] = Ci[g][r] = 0.0;

    // the next chunk's photon times are loaded one chunk ahead (the global-load latency hides behind a chunk)
    double dtn = (i0 + a < i1) ? dt[i0 + a] : 0.0;
    double d2n = TWOD ? ((i0 + a < i1) ? dt2[i0 + a] : 0.0) : 0.0;
    for (int64_t ib = i0; ib < i1; ib += kMfmaChunk) {
        const int cnt = (int)(i1 - ib < kMfmaChunk ? i1 - ib : kMfmaChunk);
        const double dtv = dtn, d2v = d2n;
        {
            const int64_t nb = ib + kMfmaChunk;
            dtn = (nb + a < i1) ? dt[nb + a] : 0.0;
            if (TWOD) d2n = (nb + a < i1) ? dt2[nb + a] : 0.0;
        }
        f32x16 re[G], im[G];
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int r = 0; r < 16; ++r) re[g][r] = im[g][r] = 0.0f;
        if (cnt == kMfmaChunk) {
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
                fast_pair<G, SQUARE>(TWOD ? fma(fa, d, c2 * d2) : fa * d, gb * d, 1.0f, ka, kb, re, im);
            }
        } else {
            for (int q = 0; 2 * q < cnt; ++q) {
                const int src = 2 * q + h;
                const double d = bperm_d(dtv, src);
                const double d2 = TWOD ? bperm_d(d2v, src) : 0.0;
                fast_pair<G, SQUARE>(TWOD ? fma(fa, d, c2 * d2) : fa * d, gb * d, src < cnt ? 1.0f : 0.0f, ka, kb,
                                     re, im);
            }
        }
        mfma_drain();
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                Cr[g][r] += (double)re[g][r];
                Ci[g][r] += (double)im[g][r];
            }
    }
    // D[row][col] of each 32x32 tile: col = lane&31 (b), row = (r&3) + 8*(r>>2) + 4*(lane>>5) (a)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int ra = (r & 3) + 8 * (r >> 2) + 4 * h;
        const int64_t c = c0 + ra + 32 * a;
        const int64_t o = frow * nf + c - first;
        if (c < nf && o >= 0 && o < count) {
#pragma unroll
            for (int g = 0; g < G; ++g) {
                const int comp = 2 * ((g == 0 ? ka : kb) - 1);
                part[(split * ncomp + comp) * count + o] = Cr[g][r];
                part[(split * ncomp + comp + 1) * count + o] = Ci[g][r];
            }
        }
    }
}

// Harmonic groups of the fast kernel: pairs (k, 2k) share one sin/cos evaluation (the second by squaring),
// taken greedily from k = 1 up; the harmonics left over go in pairs (each from its own phase) and a final single.
// m = 2: {(1,2)}; m = 20: six squared pairs + (11,12) (13,15) (16,17) (19,20).
struct HarmGroup {
    int g, ka, kb;
    bool square;
};

static std::vector<HarmGroup> harmonic_groups(int m) {
    std::vector<HarmGroup> out;
    std::vector<char> used((size_t)m + 1, 0);
    for (int k = 1; 2 * k <= m; ++k)
        if (!used[k] && !used[2 * k]) {
            out.push_back({2, k, 2 * k, true});
            used[k] = used[2 * k] = 1;
        }
    std::vector<int> rest;
    for (int k = 1; k <= m; ++k)
        if (!used[k]) rest.push_back(k);
    for (size_t i = 0; i < rest.size(); i += 2)
        out.push_back(i + 1 < rest.size() ? HarmGroup{2, rest[i], rest[i + 1], false}
                                          : HarmGroup{1, rest[i], rest[i], false});
    return out;
}

template <bool TWOD>
static void launch_fast(const HarmGroup& hg, dim3 grid, hipStream_t s, const double* dt, const double* dt2, int64_t n,
                        int64_t chunk, const double* fr, int64_t nf, const double* c2, const double* ap, int64_t tf,
                        int64_t nt, int64_t tpr, int64_t first, int64_t count, int ncomp, double* part) {
#define CRIMP_LF16(GG, FF)                                                                                            \
    k_search_fast<GG, TWOD, FF><<<grid, 256, 0, s>>>(dt, dt2, n, chunk, fr, nf, c2, ap, tf, nt, tpr, first, count, \
                                                     hg.ka, hg.kb, ncomp, part)
    if (hg.g == 2) {
        if (hg.square) CRIMP_LF16(2, true); else CRIMP_LF16(2, false);
    } else {
        CRIMP_LF16(1, false);
    }
#undef CRIMP_LF16
}

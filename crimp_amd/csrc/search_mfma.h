// search_mfma.h -- factorised periodicity search on the fp32 matrix cores (MI355X / gfx950).
//
// For a trial grid that is an arithmetic progression f_j = f_0 + j*delta (within 16 ulp), a tile
// of 1024 consecutive trials j = c0 + a + 32*b (a, b in 0..31) factorises:
//     exp(2*pi*i*k*f_j*dt) = U_a * V_b,  U_a = exp(2*pi*i*k*(f_{c0+a}*dt + c2*dt^2)),
//                                         V_b = exp(2*pi*i*k*(32*b*delta)*dt),
// so the harmonic sums over photons are a complex matrix product
//     C_ab + i S_ab = sum_i U_ai V_bi,
// computed with real 32x32x2 f32 MFMAs whose K=2 index runs over a pair of photons, four per pair
// and harmonic: Re += Ur.Vr + Ui.(-Vi), Im += Ui.Vr + Ur.Vi.
// U and V cost 32+32 sin/cos per photon per wave instead of 1024 for the direct kernel; the phases
// are fp64 and reduced to a centred fractional cycle before the fp32 sin/cos, the MFMA chain
// accumulates kMfmaChunk photons in fp32 (exact fp32 fma chain) before folding into fp64.
// One wave owns one tile and one photon range (split); results go to the same part[] layout as
// the direct kernel, so k_search_finalize forms Z^2 / H.
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kMfmaChunk = 32;
constexpr int kTile = 1024;

// sin/cos(2*pi*r), |r| <= 1/2: quarter-turn reduction + the polynomials of sincos_rev_poly.
__device__ __forceinline__ void sincos_rev_f(float r, float& s, float& c) {
    const float q = __builtin_rintf(4.0f * r);
    const float y = __builtin_fmaf(-0.25f, q, r);
    const float y2 = y * y;
    float sp = __builtin_fmaf(y2, 42.0587782776566f, -76.7058597530613f);
    sp = __builtin_fmaf(y2, sp, 81.6052492760750f);
    sp = __builtin_fmaf(y2, sp, -41.3417022403997f);
    sp = __builtin_fmaf(y2, sp, 6.28318530717958647692f);
    sp *= y;
    float cp = __builtin_fmaf(y2, -26.4262625987960f, 60.2446397079094f);
    cp = __builtin_fmaf(y2, cp, -85.4568172844813f);
    cp = __builtin_fmaf(y2, cp, 64.9393940226683f);
    cp = __builtin_fmaf(y2, cp, -19.7392088021787f);
    cp = __builtin_fmaf(y2, cp, 1.0f);
    const int iq = (int)q & 3;
    const float s_a = (iq & 1) ? cp : sp;
    const float c_a = (iq & 1) ? sp : cp;
    s = (iq & 2) ? -s_a : s_a;
    c = ((iq + 1) & 2) ? -c_a : c_a;
}

__device__ __forceinline__ double readlane_d(double v, int l) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
    return __hiloint2double(hi, lo);
}

// One photon PAIR of one wave's tile: operands of harmonics k0 .. k0+G-1 and their 4G MFMAs.
// The MFMA's K=2 index is the photon of the pair: lane l = (a = l&31, h = l>>5) evaluates U_a and
// V_a of photon 2q+h only (no sin/cos is computed twice), and the complex product is split into
// real MFMAs:  Re += Ur.Vr + Ui.(-Vi),  Im += Ui.Vr + Ur.Vi.  `live` zeroes the missing photon of
// an odd tail. FIRST groups take harmonic 2 by squaring (unbiased: the sin/cos error is quarter-turn
// periodic); later groups evaluate every harmonic from its own fp64 phase.
template <int G>
__device__ __forceinline__ void mfma_pair_ops(float uc, float us, float vc, float vs, int g, f32x16 (&re)[G],
                                              f32x16 (&im)[G]) {
    re[g] = __builtin_amdgcn_mfma_f32_32x32x2f32(uc, vc, re[g], 0, 0, 0);
    im[g] = __builtin_amdgcn_mfma_f32_32x32x2f32(us, vc, im[g], 0, 0, 0);
    re[g] = __builtin_amdgcn_mfma_f32_32x32x2f32(us, -vs, re[g], 0, 0, 0);
    im[g] = __builtin_amdgcn_mfma_f32_32x32x2f32(uc, vs, im[g], 0, 0, 0);
}

template <int G, bool FIRST>
__device__ __forceinline__ void mfma_pair(double phu, double phv, float live, int k0, f32x16 (&re)[G],
                                          f32x16 (&im)[G]) {
    if (FIRST) {
        float us, uc, vs, vc;
        sincos_rev_f((float)(phu - rint(phu)), us, uc);
        sincos_rev_f((float)(phv - rint(phv)), vs, vc);
        us *= live;
        uc *= live;
        if (G > 1) {
            const float c2u = __builtin_fmaf(uc, uc, -us * us), s2u = 2.0f * uc * us;
            const float c2v = __builtin_fmaf(vc, vc, -vs * vs), s2v = 2.0f * vc * vs;
            re[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(uc, vc, re[0], 0, 0, 0);
            im[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(us, vc, im[0], 0, 0, 0);
            re[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(c2u, c2v, re[1], 0, 0, 0);
            im[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(s2u, c2v, im[1], 0, 0, 0);
            re[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(us, -vs, re[0], 0, 0, 0);
            im[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(uc, vs, im[0], 0, 0, 0);
            re[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(s2u, -s2v, re[1], 0, 0, 0);
            im[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(c2u, s2v, im[1], 0, 0, 0);
        } else {
            mfma_pair_ops<G>(uc, us, vc, vs, 0, re, im);
        }
    } else {
        float us[G], uc[G], vs[G], vc[G];
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const double kf = (double)(k0 + g);
            const double pu = phu * kf, pv = phv * kf;
            sincos_rev_f((float)(pu - rint(pu)), us[g], uc[g]);
            sincos_rev_f((float)(pv - rint(pv)), vs[g], vc[g]);
            us[g] *= live;
            uc[g] *= live;
        }
        if (G > 1) {
#pragma unroll
            for (int g = 0; g < G; ++g) {
                re[g] = __builtin_amdgcn_mfma_f32_32x32x2f32(uc[g], vc[g], re[g], 0, 0, 0);
                im[g] = __builtin_amdgcn_mfma_f32_32x32x2f32(us[g], vc[g], im[g], 0, 0, 0);
            }
#pragma unroll
            for (int g = 0; g < G; ++g) {
                re[g] = __builtin_amdgcn_mfma_f32_32x32x2f32(us[g], -vs[g], re[g], 0, 0, 0);
                im[g] = __builtin_amdgcn_mfma_f32_32x32x2f32(uc[g], vs[g], im[g], 0, 0, 0);
            }
        } else {
            mfma_pair_ops<G>(uc[0], us[0], vc[0], vs[0], 0, re, im);
        }
    }
}

// lane-indexed fetch of a double held by lane `src` of the wave (ds_bpermute, LDS crossbar)
__device__ __forceinline__ double bperm_d(double v, int src) {
    const int lo = __builtin_amdgcn_ds_bpermute(src << 2, __double2loint(v));
    const int hi = __builtin_amdgcn_ds_bpermute(src << 2, __double2hiint(v));
    return __hiloint2double(hi, lo);
}

template <int G, bool TWOD, bool FIRST>
__global__ __launch_bounds__(256, 2) void k_search_mfma(
    const double* __restrict__ dt, const double* __restrict__ dt2, int64_t n, int64_t chunk,
    const double* __restrict__ freq, int64_t nf, const double* __restrict__ c2row, double delta,
    int64_t tile_first, int64_t ntiles, int64_t tiles_per_row, int64_t first, int64_t count, int k0, int ncomp,
    double* __restrict__ part) {
    const int lane = threadIdx.x & 63;
    const int64_t T = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (T >= ntiles) return;  // wave-uniform
    const int64_t gt = tile_first + T;
    const int64_t frow = gt / tiles_per_row;
    const int64_t c0 = (gt - frow * tiles_per_row) * kTile;
    const int a = lane & 31;
    const int h = lane >> 5;
    int64_t ca = c0 + a;
    ca = ca < nf ? ca : nf - 1;
    const double fa = freq[ca];
    const double gb = (double)(32 * a) * delta;
    const double c2 = TWOD ? c2row[frow] : 0.0;
    const int64_t split = blockIdx.y;
    const int64_t i0 = split * chunk;
    const int64_t i1 = i0 + chunk < n ? i0 + chunk : n;

    double Cr[G][16], Ci[G][16];
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
        for (int r = 0; r < 16; ++r) Cr[g][r] = Ci[g][r] = 0.0;

    for (int64_t ib = i0; ib < i1; ib += kMfmaChunk) {
        const int cnt = (int)(i1 - ib < kMfmaChunk ? i1 - ib : kMfmaChunk);
        // the chunk's photon times: one coalesced load; lane (a, h) then fetches photon 2q+h's
        const double dtv = a < cnt ? dt[ib + a] : 0.0;
        const double d2v = TWOD ? (a < cnt ? dt2[ib + a] : 0.0) : 0.0;
        f32x16 re[G], im[G];
#pragma unroll
        for (int g = 0; g < G; ++g) {
#pragma unroll
            for (int r = 0; r < 16; ++r) re[g][r] = im[g][r] = 0.0f;
        }
        if (cnt == kMfmaChunk) {
#pragma unroll
            for (int q = 0; q < kMfmaChunk / 2; ++q) {
                const int src = 2 * q + h;
                const double d = bperm_d(dtv, src);
                const double phu = TWOD ? fma(fa, d, c2 * bperm_d(d2v, src)) : fa * d;
                mfma_pair<G, FIRST>(phu, gb * d, 1.0f, k0, re, im);
            }
        } else {
            for (int q = 0; 2 * q < cnt; ++q) {
                const int src = 2 * q + h;
                const double d = bperm_d(dtv, src);
                const double phu = TWOD ? fma(fa, d, c2 * bperm_d(d2v, src)) : fa * d;
                mfma_pair<G, FIRST>(phu, gb * d, src < cnt ? 1.0f : 0.0f, k0, re, im);
            }
        }
#pragma unroll
        for (int g = 0; g < G; ++g) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                Cr[g][r] += (double)re[g][r];
                Ci[g][r] += (double)im[g][r];
            }
        }
    }
    // D[row][col] of the 32x32 tile: col = lane&31 (b), row = (r&3) + 8*(r>>2) + 4*(lane>>5) (a)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int ra = (r & 3) + 8 * (r >> 2) + 4 * h;
        const int64_t c = c0 + ra + 32 * a;
        const int64_t t = frow * nf + c - first;
        if (c < nf && t >= 0 && t < count) {
#pragma unroll
            for (int g = 0; g < G; ++g) {
                const int comp = 2 * (k0 - 1 + g);
                part[(split * ncomp + comp) * count + t] = Cr[g][r];
                part[(split * ncomp + comp + 1) * count + t] = Ci[g][r];
            }
        }
    }
}

#include "search_mfma16.h"

// Uniform-grid check on the host copy of freq: |f_j - (f_0 + j*delta)| <= 16 ulp(max|f|).
static bool freq_is_progression(const std::vector<double>& f, double* delta) {
    const int64_t nf = (int64_t)f.size();
    if (nf < 2) return false;
    const double d = (f[nf - 1] - f[0]) / (double)(nf - 1);
    double fmax = 0.0;
    for (double v : f) fmax = std::max(fmax, std::fabs(v));
    const double tol = 16.0 * 2.220446049250313e-16 * fmax;
    for (int64_t j = 0; j < nf; ++j)
        if (std::fabs(f[j] - (f[0] + (double)j * d)) > tol) return false;
    *delta = d;
    return true;
}


template <bool TWOD>
static void launch_mfma(int G, bool firstk, dim3 grid, hipStream_t s, const double* dt, const double* dt2, int64_t n,
                        int64_t chunk, const double* fr, int64_t nf, const double* c2, double delta, int64_t tf,
                        int64_t nt, int64_t tpr, int64_t first, int64_t count, int k0, int ncomp, double* part) {
#define CRIMP_LM(GG, FF)                                                                                           \
    k_search_mfma<GG, TWOD, FF><<<grid, 256, 0, s>>>(dt, dt2, n, chunk, fr, nf, c2, delta, tf, nt, tpr, first, count, \
                                                     k0, ncomp, part)
    if (G == 2) {
        if (firstk) CRIMP_LM(2, true); else CRIMP_LM(2, false);
    } else {
        if (firstk) CRIMP_LM(1, true); else CRIMP_LM(1, false);
    }
#undef CRIMP_LM
}

// Harmonic groups of the f16 kernel: pairs (k, 2k) share one sin/cos evaluation (the second by
// squaring), taken greedily from k = 1 up; the harmonics left over go in pairs (each from its own
// phase) and a final single. m = 2: {(1,2)}; m = 20: six squared pairs + (11,12) (13,15) (16,17) (19,20),
// 14 sin/cos evaluations per photon and trial instead of 20.
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

// Returns 1 when the factorised kernel produced `out`, 0 when it declines, <0 on error.
static int mfma_search(Scratch& sc, hipStream_t s, const double* dt, const double* dt2, int64_t n,
                       const double* freq, int64_t nf, const double* c2, bool twod, int nharm, int stat,
                       int64_t first, int64_t count, double* out, uint32_t flags) {
    if (count < 256 && !(flags & CRIMP_FLAG_FORCE_MFMA)) return 0;
    std::vector<double> fh((size_t)nf);
    hipError_t e = d2h(s, fh.data(), freq, nf * sizeof(double));
    if (e != hipSuccess) return set_err(CRIMP_ERR_HIP, std::string("mfma_search freq copy: ") + hipGetErrorString(e));
    double delta = 0.0;
    if (!freq_is_progression(fh, &delta)) return 0;

    // variant: f16 hi/lo split on the f16 MFMA (default; one or two tiles per wave) or f32-input MFMA
    const int variant = (flags & CRIMP_FLAG_MFMA_F32) ? 0 : ((flags & CRIMP_FLAG_MFMA_T2) ? 2 : 1);
    const int64_t wtile = kTile * (variant == 2 ? 2 : 1);
    const int64_t tpr = cdiv(nf, wtile);
    // photon splits depend on the photon count alone, so that every trial's value is bit-identical
    // however the grid is partitioned (tiles are already aligned to absolute trial indices): a
    // sharded search returns exactly what one unsharded call returns. Up to 64 splits of >= 64k photons:
    // the last round of resident waves is then a small part of the launch (config 3: 977 tiles x 64 splits
    // = 30.5 rounds of the 2048 wave slots, 98.5 % filled, against 7.6 of 8 rounds = 95.4 % with 16).
#ifndef CRIMP_MAX_SPLITS
#define CRIMP_MAX_SPLITS 64
#endif
    const int64_t best_s = std::min<int64_t>(CRIMP_MAX_SPLITS, std::max<int64_t>(1, n / 65536));
    int64_t chunk = cdiv(cdiv(n, best_s), kMfmaChunk) * kMfmaChunk;
    const int64_t splits = cdiv(n, chunk);
    const int ncomp = 2 * nharm;
    // per-split partial sums are fp64 [splits][ncomp][trials]; a trial range whose partials would pass
    // kPartBudget bytes (of the 288 GB HBM) is searched in equal blocks of trials, so that no block is a
    // sliver that leaves most wave slots idle (tiles straddling a block edge run twice)
    const int64_t kPartBudget = int64_t(16) << 30;
    const int64_t cbmax = std::max<int64_t>(wtile, kPartBudget / (8 * splits * ncomp));
    const int64_t nblk = cdiv(count, cbmax);
    const int64_t cb = std::min<int64_t>(count, cdiv(cdiv(count, nblk), wtile) * wtile);
    double* part = nullptr;
    e = sc.alloc(&part, (size_t)(splits * ncomp * cb));
    if (e != hipSuccess) return set_err(CRIMP_ERR_HIP, std::string("mfma_search alloc: ") + hipGetErrorString(e));
    KernelTimer kt(s, flags & CRIMP_FLAG_TIME_KERNELS);
    kt.start();
    for (int64_t b0 = 0; b0 < count; b0 += cb) {
        const int64_t bfirst = first + b0, bcount = std::min<int64_t>(cb, count - b0);
        const int64_t last = bfirst + bcount - 1;
        const int64_t tf = (bfirst / nf) * tpr + (bfirst % nf) / wtile;
        const int64_t tl = (last / nf) * tpr + (last % nf) / wtile;
        const int64_t nt = tl - tf + 1;
        dim3 grid((unsigned)cdiv(nt, 4), (unsigned)splits);
        if (variant == 0) {
            for (int k0 = 1; k0 <= nharm;) {
                // groups {1,2}, {3,4}, {5,6}, ...: harmonic 2 by squaring, later ones from exact phases
                const int G = (nharm - k0 + 1) >= 2 ? 2 : 1;
                if (twod)
                    launch_mfma<true>(G, k0 == 1, grid, s, dt, dt2, n, chunk, freq, nf, c2, delta, tf, nt, tpr, bfirst,
                                      bcount, k0, ncomp, part);
                else
                    launch_mfma<false>(G, k0 == 1, grid, s, dt, dt2, n, chunk, freq, nf, c2, delta, tf, nt, tpr, bfirst,
                                       bcount, k0, ncomp, part);
                e = hipGetLastError();
                if (e != hipSuccess) return set_err(CRIMP_ERR_HIP, std::string("k_search_mfma: ") + hipGetErrorString(e));
                k0 += G;
            }
        } else {
            for (const HarmGroup& hg : harmonic_groups(nharm)) {
#define CRIMP_ARGS hg.g, hg.square, grid, s, dt, dt2, n, chunk, freq, nf, c2, delta, tf, nt, tpr, bfirst, bcount, hg.ka, \
                       hg.kb, ncomp, part
                if (variant == 1) {
                    if (twod) launch_mfma16<true, 1>(CRIMP_ARGS); else launch_mfma16<false, 1>(CRIMP_ARGS);
                } else {
                    if (twod) launch_mfma16<true, 2>(CRIMP_ARGS); else launch_mfma16<false, 2>(CRIMP_ARGS);
                }
#undef CRIMP_ARGS
                e = hipGetLastError();
                if (e != hipSuccess) return set_err(CRIMP_ERR_HIP, std::string("k_search_mfma16: ") + hipGetErrorString(e));
            }
        }
        if (b0 + cb >= count) kt.stop();  // the last block's harmonic-sum kernels end the timed span
        k_search_finalize<<<(unsigned)cdiv(bcount, 256), 256, 0, s>>>(part, bcount, (int)splits, nharm, stat, (double)n,
                                                                    out + b0);
        e = hipGetLastError();
        if (e != hipSuccess) return set_err(CRIMP_ERR_HIP, std::string("finalize: ") + hipGetErrorString(e));
    }
    return 1;
}

// toa_fit.h -- measureToA_* fits on the device, one workgroup per ToA interval (included by crimp_hip.hip).
//
// crimp_amd/toafit.py drives the same iterations from the host, where every likelihood evaluation is a
// k_toa_points launch and a host round trip. Here an interval's whole fit (measureToAs.py:285-376) runs
// inside one 512-thread workgroup: an evaluation is one pass over the interval's photons and a workgroup
// reduction that every thread reads back, so the workgroup iterates the reference driver itself, with
// toafit.py's constants and stopping rules:
//   start   the brute-grid maximum (k_toa_grid partial sums -> k_toa_grid_best) or (norm0, 0);
//   ascent  damped 2-D Newton in (norm, phShift) with a backtracking line search, the last step below 1e-6 taken
//           on the quadratic model without a pass (toafit.maximise, the same rule);
//   1 sigma phShift = best -/+ k*2pi/phShiftRes with lmfit's clip-to-bound semantics, the norm re-profiled at every
//           step -- from one pass of the moments sum (n0 + h_i)^-p (fit_profile_mom), or by 1-D Newton
//           (toafit.profile_norm) where that series does not apply; stop at the first LLmax - LL > 0.5*chi2.ppf(0.6827,1)
//           or once k + 1 > phShiftRes/2 (measureToAs.py:331-376, toafit.error_scan).
// The evaluation repeats k_toa_points' per-photon arithmetic (tpl_terms), thread striding and reduction
// order, so its sums equal the host-driven path's (the moment profile is device-only: its LL agrees with the
// iterative profile's to ~1e-10, and the scan compares it with a 0.5 threshold).

constexpr int kFitBlock = kPtsBlock;
// the photon phases through a global address-space pointer: the fit's helpers take generic pointers (they are called
// out of line), whose loads hipcc would issue as flat loads -- counted against the LDS counter too, so every wait for
// a sin/cos table read would also wait for the next photon's load (measured neutral: 2.90 vs 2.90 ms per 1250
// config-5 fits, profiles/r04/ab_toa_gld.log -- the prefetch one photon ahead already hides it; CRIMP_FIT_GLD=0: the
// generic loads)
#ifndef CRIMP_FIT_GLD
#define CRIMP_FIT_GLD 1
#endif
typedef const double __attribute__((address_space(1))) GDouble;
__device__ __forceinline__ double gld(const double* p, int64_t i) { return CRIMP_FIT_GLD ? ((GDouble*)p)[i] : p[i]; }
// fit_moments2 fills the second phShift's coefficients from threads 64 .. 64 + K - 1 (the first wave fills the first's)
static_assert(kFitBlock >= 64 + CRIMP_MAX_COMP, "fit_moments2: the block must cover threads 64 .. 64 + CRIMP_MAX_COMP");
constexpr double kHalfChi2OneSigma = 0.500021713558733;  // 0.5 * chi2.ppf(0.6827, 1)   (measureToAs.py:324)
constexpr double kTwoPi = 6.283185307179586476925286766559;

struct FitCfg {
    double lo, hi;   // norm bounds [norm0/100, 500]                           (measureToAs.py:715-716, :757-758)
    double pb;       // phShift bound: pi (fourier), 1.5 pi (cauchy, vonmises)   (:722, :767)
    double step;     // 2 pi / phShiftRes                                       (:320)
    double kcap;     // phShiftRes / 2                                          (:348, :373)
    double sum_amp;  // sum_j amp_j: cauchy / von Mises normalisation F = 2 pi norm + sum_amp
    double amp_lo, amp_hi;  // ampShift bounds when varied: [0.01, 100] fourier (:308), [0, inf) cauchy (:461),
                            // [0, 500] von Mises (:605)
    double mom_r;           // fit_profile_mom's largest |d| / min m (kMomR; test hook CRIMP_FIT_MOM_R, 0: iterative)
};

struct FitEval {
    double ll, gn, gp, hnn, hnp, hpp;
};

struct FitShared {
    double red[kFitBlock / 64][8];
    double coef[2][CRIMP_MAX_COMP];
    double coef2[2][CRIMP_MAX_COMP];       // the second phShift of a joint moment pass (fit_moments2)
    double red2[kFitBlock / 64][8];
#if CRIMP_FIT_TABLE
    double2 tab[kSinTab];  // photon_sincos_tab (filled once per workgroup)
#endif
};
__device__ __forceinline__ void fit_sincos(int model, FitShared& sh, double xv, double& s1, double& c1) {
#if CRIMP_FIT_TABLE
    photon_sincos_tab(model, sh.tab, xv, s1, c1);
#else
    photon_sincos(model, xv, s1, c1);
#endif
}
__device__ __forceinline__ void fit_shared_init(FitShared& sh) {
#if CRIMP_FIT_TABLE
    sintab_fill(sh.tab);
#endif
}

// np.clip semantics (a NaN stays NaN)
__device__ __forceinline__ double clipd(double v, double lo, double hi) { return v < lo ? lo : (v > hi ? hi : v); }
// the 1-sigma bound kk * step + step / 2 (measureToAs.py:351, :376) rounded as numpy does: multiply, then add
// (hipcc would otherwise fuse it into one fma and differ in the last bit)
__device__ __forceinline__ double sigma_bound(int kk, double step) {
#pragma clang fp contract(off)
    return (double)kk * step + step / 2;
}

// Template-part cache modes of fit_eval: the norm profile of the 1-sigma scan evaluates one phShift at several
// norms, and the template part h(x_i; phShift) of the model norm + h does not depend on the norm. The profile's
// first pass stores each photon's h (the thread that computes it is the one that reads it back: same striding),
// later passes read it instead of recomputing sin/cos and the template terms. The stored value is the
// recomputed one bit for bit, so the sums are unchanged.
enum : int { kHNone = 0, kHStore = 1, kHLoad = 2 };
// model values per fp64 log: 8 (12.03 -> 11.33 ms per 1250 config-5 fits, profiles/r03/ab_fit_store_prod8.log);
// exact for model values in (1e-38, 1e38), where no product of 8 leaves the fp64 range
#ifndef CRIMP_FIT_PROD
#define CRIMP_FIT_PROD 8
#endif
constexpr int kFitProd = CRIMP_FIT_PROD;  // model values per fp64 log in fit_eval
// 16 model values per log where that provably stays in the fp64 range: a compile-time Fourier template, whose template
// part |h| <= sum_j |amp_j| = H, at a pass norm n with n - H >= 2^-60 and n + H <= 2^60 -- a product of 16 model
// values n + h then lies in [2^-960, 2^960] (2.82 -> 2.70 ms per 1250 config-5 fits, profiles/r06/ab_toa_prod16.log);
// kFitProd elsewhere. Chosen per pass from (n, template) alone, so a record does not depend on its batch.
// CRIMP_FIT_PROD16=0: kFitProd everywhere.
#ifndef CRIMP_FIT_PROD16
#define CRIMP_FIT_PROD16 1
#endif
template <int MODEL, int KF>
__device__ __forceinline__ int fit_prodlen(const TplDev* __restrict__ T, double n) {
    if constexpr (CRIMP_FIT_PROD16 && MODEL == CRIMP_MODEL_FOURIER && KF > 0) {
        double H = 0.0;
#pragma unroll
        for (int j = 0; j < KF; ++j) H += fabs(T->amp[j]);
        if (n - H >= 0x1p-60 && n + H <= 0x1p60) return 16;
    }
    return kFitProd;
}
// the photon loops load the next photon's time (or cached template part) one iteration ahead, so the load's
// latency overlaps the current photon's arithmetic (CRIMP_FIT_PREFETCH=0: load at the top of each iteration)
#ifndef CRIMP_FIT_PREFETCH
#define CRIMP_FIT_PREFETCH 1
#endif
constexpr bool kFitPrefetch = CRIMP_FIT_PREFETCH != 0;

// Reference extended LL (templatemodels.py:109-121, :213-226, :318-329) with its (norm, phShift) gradient and
// Hessian at (n, phi), from one pass over photons x[a, b) (as toafit.ToAFitter.evaluate assembles them).
// kHStore and kHLoad passes return the LL and the norm derivatives only (gp, hnp, hpp are 0). MODEL and (Fourier) the template
// size KF are compile-time (KF = 0: K from the template at run time), as in k_toa_grid.
template <int MODEL, int KF, int PL>  // PL: model values per log (fit_prodlen)
__device__ FitEval fit_eval_pl(const double* __restrict__ x, int64_t a, int64_t b, const TplDev* __restrict__ T,
                               double n, double phi, double E, const FitCfg& C, FitShared& sh, double* __restrict__ hc,
                               int hmode) {
    const int tid = threadIdx.x;
    constexpr int model = MODEL;
    const int K = KF > 0 ? KF : T->K;
    __syncthreads();  // the previous evaluation's readers are done with sh
    if (tid < K) tpl_coef(T, tid, phi, sh.coef[0][tid], sh.coef[1][tid]);
    __syncthreads();
    double acc[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    double mn = INFINITY;
    // sum of ln(model) as ln of products of kFitProd consecutive (per thread) model values: one fp64 log per
    // kFitProd photons; a product of <= 8 model values in (1e-38, 1e38) stays in the fp64 range and adds <= 7
    // roundings (~8e-16 relative). A non-positive model makes the LL -inf through min(model) below.
    double pr = 1.0;
    int np = 0;
    auto lnacc = [&](double mv) {
        pr *= mv;
        if (++np == PL) {
            acc[0] += log(pr);
            pr = 1.0;
            np = 0;
        }
    };
    if (hmode == kHLoad) {
        double hn = a + tid < b ? hc[a + tid] : 0.0;
        for (int64_t i = a + tid; i < b; i += kFitBlock) {
            const double hv = hn;
            if (kFitPrefetch && i + kFitBlock < b) hn = hc[i + kFitBlock];
            const double mv = n + (kFitPrefetch ? hv : hc[i]);
            const double q = lk_rcp(mv);
            lnacc(mv);
            acc[1] += q;
            acc[3] -= q * q;
            mn = fmin(mn, mv);
        }
    } else {
      [[maybe_unused]] double al[KF > 0 ? KF : 1], be[KF > 0 ? KF : 1];
      if constexpr (MODEL == CRIMP_MODEL_FOURIER && KF > 0) {
#pragma unroll
          for (int j = 0; j < KF; ++j) {
              al[j] = sh.coef[0][j];
              be[j] = sh.coef[1][j];
          }
      }
      if (hmode == kHStore) {
        // the first pass of a norm profile: the profile reads only LL, dLL/dnorm and d2LL/dnorm2, so the phShift
        // derivatives h', h'' are not formed (the Fourier template: 5 instead of 9 operations per harmonic); h and
        // the sums are formed exactly as in the full pass
        double xn = a + tid < b ? gld(x, a + tid) : 0.0;
        for (int64_t i = a + tid; i < b; i += kFitBlock) {
            double s1, c1, h;
            const double xv = kFitPrefetch ? xn : gld(x, i);
            if (kFitPrefetch && i + kFitBlock < b) xn = gld(x, i + kFitBlock);
            fit_sincos(model, sh, xv, s1, c1);
            if constexpr (MODEL == CRIMP_MODEL_FOURIER && KF > 0) {
                tpl_value_fourier<KF>(al, be, s1, c1, h);
            } else {
                double h1, h2;
                tpl_terms(T, model, K, sh.coef[0], sh.coef[1], s1, c1, h, h1, h2);
            }
            hc[i] = h;
            const double mv = n + h;
            const double q = lk_rcp(mv);
            lnacc(mv);
            acc[1] += q;
            acc[3] -= q * q;
            mn = fmin(mn, mv);
        }
      } else {
       double xn = a + tid < b ? gld(x, a + tid) : 0.0;
       for (int64_t i = a + tid; i < b; i += kFitBlock) {
        double s1, c1, h, h1, h2;
        const double xv = kFitPrefetch ? xn : gld(x, i);
        if (kFitPrefetch && i + kFitBlock < b) xn = gld(x, i + kFitBlock);
        fit_sincos(model, sh, xv, s1, c1);
        if constexpr (MODEL == CRIMP_MODEL_FOURIER && KF > 0)
            tpl_terms_fourier<KF>(al, be, s1, c1, h, h1, h2);
        else
            tpl_terms(T, model, K, sh.coef[0], sh.coef[1], s1, c1, h, h1, h2);
        const double mv = n + h;
        const double q = lk_rcp(mv);
        lnacc(mv);
        acc[1] += q;
        acc[2] += h1 * q;
        acc[3] -= q * q;
        acc[4] -= h1 * q * q;
        acc[5] += h2 * q - h1 * h1 * q * q;
        mn = fmin(mn, mv);
       }
      }
    }
    if (np) acc[0] += log(pr);
    const int w = tid >> 6, lane = tid & 63;
#pragma unroll
    for (int q = 0; q < 6; ++q) {
        const double v = wave_sum(acc[q]);
        if (lane == 0) sh.red[w][q] = v;
    }
    const double vm = wave_min(mn);
    if (lane == 0) sh.red[w][6] = vm;
    __syncthreads();
    double S[7];
#pragma unroll
    for (int q = 0; q < 7; ++q) {
        double v = sh.red[0][q];
        for (int ww = 1; ww < kFitBlock / 64; ++ww) v = (q == 6) ? fmin(v, sh.red[ww][q]) : v + sh.red[ww][q];
        S[q] = v;
    }
    const double N = (double)(b - a);
    FitEval r;
    double F;
    if (model == CRIMP_MODEL_FOURIER) {
        F = n;
        r.ll = -n * E + N * log(n * E) + (S[0] - N * log(n));
    } else {
        F = kTwoPi * n + C.sum_amp;
        r.ll = -F * E / kTwoPi + N * log(F * E / kTwoPi) + (S[0] - N * log(F));
    }
    if (!(S[6] / F > 0)) r.ll = -INFINITY;  // min(model / normalisation) <= 0 (:113-115, :220-222, :324-326)
    r.gn = -E + S[1];
    r.gp = S[2];
    r.hnn = S[3];
    r.hnp = S[4];
    r.hpp = S[5];
    return r;
}
template <int MODEL, int KF>
__device__ FitEval fit_eval(const double* __restrict__ x, int64_t a, int64_t b, const TplDev* __restrict__ T, double n,
                            double phi, double E, const FitCfg& C, FitShared& sh, double* __restrict__ hc = nullptr,
                            int hmode = kHNone) {
    if (fit_prodlen<MODEL, KF>(T, n) == 16) return fit_eval_pl<MODEL, KF, 16>(x, a, b, T, n, phi, E, C, sh, hc, hmode);
    return fit_eval_pl<MODEL, KF, kFitProd>(x, a, b, T, n, phi, E, C, sh, hc, hmode);
}

// toafit._newton_step: Levenberg-shifted Newton direction with a trust region (0.05 rad, half the norm). Projected:
// a coordinate on its bound whose gradient points out of the box is held there and the other takes its own 1-D Newton
// step, so that when phShift stops on -+bound (a maximum beyond it) the norm is still maximised exactly -- the
// reference's lmfit fit, and the oracle's bounded search, profile it there; a joint step whose phShift part is clipped
// away would leave the norm wherever the clipped line search stalls (redChi2 off by ~1e-5).
__device__ void fit_newton_dir(double n, double p, const FitCfg& C, const FitEval& e, double& dn, double& dp,
                               bool* pure = nullptr) {
    const bool pfix = (p <= -C.pb && e.gp < 0.0) || (p >= C.pb && e.gp > 0.0);
    const bool nfix = (n <= C.lo && e.gn < 0.0) || (n >= C.hi && e.gn > 0.0);
    if (pfix || nfix) {
        dn = nfix ? 0.0 : (e.hnn < 0.0 ? -e.gn / e.hnn : (e.gn > 0.0 ? 0.1 : -0.1) * fabs(n));
        dp = pfix ? 0.0 : (e.hpp < 0.0 ? -e.gp / e.hpp : (e.gp > 0.0 ? 0.05 : -0.05));
        double sc = fmin(1.0, 0.05 / fmax(fabs(dp), 1e-300));
        sc = fmin(sc, 0.5 * fabs(n) / fmax(fabs(dn), 1e-300));
        if (pure) *pure = sc == 1.0 && (nfix || e.hnn < 0.0) && (pfix || e.hpp < 0.0);
        dn *= sc;
        dp *= sc;
        return;
    }
    const double hnn = e.hnn, hnp = e.hnp, hpp = e.hpp;
    const double tr = hnn + hpp;
    const double det = hnn * hpp - hnp * hnp;
    const double disc = 0.25 * tr * tr - det;
    const double lam_max = 0.5 * tr + sqrt(disc != disc ? disc : (disc > 0.0 ? disc : 0.0));
    const double shift = lam_max < 0 ? 0.0 : lam_max * 1.5 + 1e-6 * (fabs(hnn) + fabs(hpp)) + 1e-12;
    const double aa = hnn - shift, cc = hpp - shift;
    const double det2 = aa * cc - hnp * hnp;
    dn = -(cc * e.gn - hnp * e.gp) / det2;
    dp = -(aa * e.gp - hnp * e.gn) / det2;
    double sc = fmin(1.0, 0.05 / fmax(fabs(dp), 1e-300));
    sc = fmin(sc, 0.5 * fabs(n) / fmax(fabs(dn), 1e-300));
    if (pure) *pure = shift == 0.0 && sc == 1.0;  // the plain Newton step of a negative definite Hessian
    dn *= sc;
    dp *= sc;
}

// Final Newton step without a likelihood pass (toafit.maximise does the same): once the plain Newton step of a
// negative definite Hessian is below kFitModelStep (rad, and relative in the norm) and inside the bounds, the
// ascent takes it and reports the LL of the local quadratic model, LL + g.d + d.H.d / 2. Newton's quadratic
// convergence leaves the point ~C d^2 (~1e-11 rad) from the maximum, and the model's LL error is third order in d
// (~N (h' d / m)^3 ~ 1e-13 for 1e5 photons) -- instead of one more pass to find a step below 1e-12.
#ifndef CRIMP_FIT_MODEL_STEP
#define CRIMP_FIT_MODEL_STEP 1
#endif
#ifndef CRIMP_FIT_MODEL_STEP_TOL
#define CRIMP_FIT_MODEL_STEP_TOL 1e-6
#endif
constexpr double kFitModelStep = CRIMP_FIT_MODEL_STEP_TOL;

// toafit.profile_norm: max over norm in [lo, hi] of LL(norm, phi) at fixed phi (1-D Newton, concave)
// hc: per-photon template-part cache (nullptr: recompute every pass).
template <int MODEL, int KF>
__device__ __noinline__ double fit_profile(const double* __restrict__ x, int64_t a, int64_t b, const TplDev* __restrict__ T,
                              double phi, double n_start, double E, const FitCfg& C, FitShared& sh, int& nev,
                              double* __restrict__ hc = nullptr, int* ncached = nullptr) {
    double n = clipd(n_start, C.lo, C.hi);
    const int hm = hc ? kHLoad : kHNone;
    FitEval e = fit_eval<MODEL, KF>(x, a, b, T, n, phi, E, C, sh, hc, hc ? kHStore : kHNone);
    ++nev;
    for (int it = 0; it < 30; ++it) {
        const bool bad = !isfinite(e.ll);
        double step = e.hnn < 0 ? -e.gn / e.hnn : 0.1 * n;
        step = clipd(step, -0.5 * n, 0.5 * n);
        if (bad) step = 0.5 * n;  // infeasible: model <= 0 somewhere, raise the norm
        double nn = clipd(n + step, C.lo, C.hi);
        // converged: the next pass would move the norm by <= 1e-13 of it, so its LL equals this one's to ~1e-26
        // relative; stop without it (toafit.profile_norm does the same)
        if (isfinite(e.ll) && fabs(nn - n) <= 1e-13 * fmax(1.0, n)) break;
        FitEval e2 = fit_eval<MODEL, KF>(x, a, b, T, nn, phi, E, C, sh, hc, hm);
        ++nev;
        if (ncached && hc) ++*ncached;
        const bool worse = isfinite(e.ll) && (!isfinite(e2.ll) || e2.ll < e.ll - 1e-12 * fabs(e.ll));
        if (worse) {  // damp an overshoot
            nn = clipd(n + 0.25 * step, C.lo, C.hi);
            e2 = fit_eval<MODEL, KF>(x, a, b, T, nn, phi, E, C, sh, hc, hm);
            ++nev;
            if (ncached && hc) ++*ncached;
        }
        const bool conv = fabs(nn - n) <= 1e-13 * fmax(1.0, n);
        n = nn;
        e = e2;
        if (conv) break;
    }
    return e.ll;
}

// toafit.profile_norm from one photon pass (the 1-sigma scan's norm profiles). At fixed phShift the extended LL is
// -nE + sum_i ln(n + h_i) + const, so with m_i = n0 + h_i at the start n0 and the moments S_p = sum_i m_i^-p, for
// n = n0 + d:   sum_i ln(n + h_i) = S_0 + sum_{p>=1} (-1)^(p+1) d^p S_p / p,   dLL/dn = -E + sum_{p>=1} (-d)^(p-1) S_p.
// One pass returns S_0 = sum ln m_i (as fit_eval forms it: one log per kFitProd values), S_1..S_5 and min m_i; the
// root of the degree-4 derivative polynomial is the profile optimum and the series at it the profile LL. With
// r = |d| / min m_i <= kMomR the dropped terms are <= N r^6 / 6 in the LL (1e5 photons: ~1e-12) and move the root by
// ~r^5 of the norm, below the iterative profile's own 1e-13 stopping step; the scan needs the profile LL only for the
// 0.5 chi2 threshold. Otherwise (start infeasible, root outside the bounds, r larger) the iterative profile runs.
// This replaces the iterative profile's cached-template passes (store h, then ~2 passes over the cache) by one pass
// without the h store: config 5, 4 scan profiles per interval.
#ifndef CRIMP_FIT_MOMENTS
#define CRIMP_FIT_MOMENTS 1
#endif
constexpr double kMomR = 2e-3;
// the scan's two sides in one moment pass per step (fit_moments2; CRIMP_FIT_JOINT=0: one pass per side and step)
#ifndef CRIMP_FIT_JOINT
#define CRIMP_FIT_JOINT 1
#endif
struct FitMom {
    double s[6];  // S_0 .. S_5
    double mn;
};
template <int MODEL, int KF, int PL>
__device__ FitMom fit_moments_pl(const double* __restrict__ x, int64_t a, int64_t b, const TplDev* __restrict__ T,
                                 double n, double phi, FitShared& sh) {
    const int tid = threadIdx.x;
    constexpr int model = MODEL;
    const int K = KF > 0 ? KF : T->K;
    __syncthreads();  // the previous evaluation's readers are done with sh
    if (tid < K) tpl_coef(T, tid, phi, sh.coef[0][tid], sh.coef[1][tid]);
    __syncthreads();
    double acc[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    double mn = INFINITY;
    double pr = 1.0;
    int np = 0;
    [[maybe_unused]] double al[KF > 0 ? KF : 1], be[KF > 0 ? KF : 1];
    if constexpr (MODEL == CRIMP_MODEL_FOURIER && KF > 0) {
#pragma unroll
        for (int j = 0; j < KF; ++j) {
            al[j] = sh.coef[0][j];
            be[j] = sh.coef[1][j];
        }
    }
    double xn = a + tid < b ? gld(x, a + tid) : 0.0;
    for (int64_t i = a + tid; i < b; i += kFitBlock) {
        double s1, c1, h;
        const double xv = xn;
        if (i + kFitBlock < b) xn = gld(x, i + kFitBlock);
        fit_sincos(model, sh, xv, s1, c1);
        if constexpr (MODEL == CRIMP_MODEL_FOURIER && KF > 0) {
            tpl_value_fourier<KF>(al, be, s1, c1, h);
        } else {
            double h1, h2;
            tpl_terms(T, model, K, sh.coef[0], sh.coef[1], s1, c1, h, h1, h2);
        }
        const double mv = n + h;
        const double q = lk_rcp(mv);
        pr *= mv;
        if (++np == PL) {
            acc[0] += log(pr);
            pr = 1.0;
            np = 0;
        }
        const double q2 = q * q;
        acc[1] += q;
        acc[2] += q2;
        acc[3] += q2 * q;
        acc[4] += q2 * q2;
        acc[5] += q2 * q2 * q;
        mn = fmin(mn, mv);
    }
    if (np) acc[0] += log(pr);
    const int w = tid >> 6, lane = tid & 63;
#pragma unroll
    for (int q = 0; q < 6; ++q) {
        const double v = wave_sum(acc[q]);
        if (lane == 0) sh.red[w][q] = v;
    }
    const double vm = wave_min(mn);
    if (lane == 0) sh.red[w][6] = vm;
    __syncthreads();
    FitMom r;
#pragma unroll
    for (int q = 0; q < 7; ++q) {
        double v = sh.red[0][q];
        for (int ww = 1; ww < kFitBlock / 64; ++ww) v = (q == 6) ? fmin(v, sh.red[ww][q]) : v + sh.red[ww][q];
        if (q < 6) r.s[q] = v; else r.mn = v;
    }
    return r;
}
template <int MODEL, int KF>
__device__ FitMom fit_moments(const double* __restrict__ x, int64_t a, int64_t b, const TplDev* __restrict__ T,
                              double n, double phi, FitShared& sh) {
    if (fit_prodlen<MODEL, KF>(T, n) == 16) return fit_moments_pl<MODEL, KF, 16>(x, a, b, T, n, phi, sh);
    return fit_moments_pl<MODEL, KF, kFitProd>(x, a, b, T, n, phi, sh);
}

// the profile optimum and LL from one phShift's moments (fit_profile_mom); false where the series does not apply
template <int MODEL>
__device__ bool mom_solve(const FitMom& m, double n0, double E, double N, const FitCfg& C, double& ll) {
    const double* S = m.s;
    if (!(m.mn > 0 && isfinite(S[0]) && S[2] > 0)) return false;
    // Newton on g(d) = -E + S1 - d S2 + d^2 S3 - d^3 S4 + d^4 S5 (strictly decreasing near 0: g' ~ -S2)
    double d = 0.0;
    bool ok = false;
    for (int it = 0; it < 12; ++it) {
        const double g = -E + S[1] + d * (-S[2] + d * (S[3] + d * (-S[4] + d * S[5])));
        const double gp = -S[2] + d * (2.0 * S[3] + d * (-3.0 * S[4] + d * 4.0 * S[5]));
        if (!(gp < 0)) break;
        const double st = -g / gp;
        d += st;
        if (!(fabs(d) <= C.mom_r * m.mn)) break;
        if (fabs(st) <= 1e-15 * n0) {
            ok = true;
            break;
        }
    }
    const double nn = n0 + d;
    if (!(ok && nn >= C.lo && nn <= C.hi)) return false;
    const double s0 = S[0] + d * (S[1] + d * (-S[2] / 2 + d * (S[3] / 3 + d * (-S[4] / 4 + d * (S[5] / 5)))));
    if (MODEL == CRIMP_MODEL_FOURIER) {
        ll = -nn * E + N * log(nn * E) + (s0 - N * log(nn));
    } else {
        const double F = kTwoPi * nn + C.sum_amp;
        ll = -F * E / kTwoPi + N * log(F * E / kTwoPi) + (s0 - N * log(F));
    }
    return true;
}

template <int MODEL, int KF>
__device__ double fit_profile_mom(const double* __restrict__ x, int64_t a, int64_t b, const TplDev* __restrict__ T,
                                  double phi, double n_start, double E, const FitCfg& C, FitShared& sh, int& nev) {
    const double n0 = clipd(n_start, C.lo, C.hi);
    const FitMom m = fit_moments<MODEL, KF>(x, a, b, T, n0, phi, sh);
    ++nev;
    double ll;
    if (mom_solve<MODEL>(m, n0, E, (double)(b - a), C, ll)) return ll;
    return fit_profile<MODEL, KF>(x, a, b, T, phi, n_start, E, C, sh, nev);  // iterative, recomputing h
}

// Two phShifts' moments in one pass (the 1-sigma scan's step k on both sides, Fourier templates of compile-time
// size): the photon's sin/cos and harmonic recurrence are formed once, and each phShift's sums repeat
// fit_moments' per-photon operations, striding and reduction order, so they equal two fit_moments passes.
template <int KF, int PL>
__device__ __noinline__ void fit_moments2_pl(const double* __restrict__ x, int64_t a, int64_t b,
                                             const TplDev* __restrict__ T, double n, double phi0, double phi1,
                                             FitShared& sh, FitMom& m0, FitMom& m1) {
    static_assert(KF > 0, "compile-time template size");
    const int tid = threadIdx.x;
    __syncthreads();  // the previous evaluation's readers are done with sh
    if (tid < KF) tpl_coef(T, tid, phi0, sh.coef[0][tid], sh.coef[1][tid]);
    else if (tid >= 64 && tid < 64 + KF) tpl_coef(T, tid - 64, phi1, sh.coef2[0][tid - 64], sh.coef2[1][tid - 64]);
    __syncthreads();
    double al0[KF], be0[KF], al1[KF], be1[KF];
#pragma unroll
    for (int j = 0; j < KF; ++j) {
        al0[j] = sh.coef[0][j];
        be0[j] = sh.coef[1][j];
        al1[j] = sh.coef2[0][j];
        be1[j] = sh.coef2[1][j];
    }
    double acc0[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0}, acc1[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    double mn0 = INFINITY, mn1 = INFINITY, pr0 = 1.0, pr1 = 1.0;
    int np = 0;
    double xn = a + tid < b ? gld(x, a + tid) : 0.0;
    for (int64_t i = a + tid; i < b; i += kFitBlock) {
        double s1, c1;
        const double xv = xn;
        if (i + kFitBlock < b) xn = gld(x, i + kFitBlock);
        fit_sincos(CRIMP_MODEL_FOURIER, sh, xv, s1, c1);
        // tpl_value_fourier for both coefficient rows on one recurrence (the same h, operation by operation)
        double h0 = 0.0, h1 = 0.0;
        {
            const double tc = c1 + c1;
            double cj = c1, sj = s1, cp = 1.0, sp = 0.0;
#pragma unroll
            for (int j = 0; j < KF; ++j) {
                const double t0j = fma(al0[j], cj, be0[j] * sj), t1j = fma(al1[j], cj, be1[j] * sj);
                h0 = j == 0 ? t0j : h0 + t0j;
                h1 = j == 0 ? t1j : h1 + t1j;
                if (j + 1 < KF) {
                    const double cn = fma(tc, cj, -cp), sn = fma(tc, sj, -sp);
                    cp = cj;
                    sp = sj;
                    cj = cn;
                    sj = sn;
                }
            }
        }
        const double mv0 = n + h0, mv1 = n + h1;
        const double q0 = lk_rcp(mv0), q1 = lk_rcp(mv1);
        pr0 *= mv0;
        pr1 *= mv1;
        if (++np == PL) {
            acc0[0] += log(pr0);
            acc1[0] += log(pr1);
            pr0 = 1.0;
            pr1 = 1.0;
            np = 0;
        }
        const double r0 = q0 * q0, r1 = q1 * q1;
        acc0[1] += q0;
        acc0[2] += r0;
        acc0[3] += r0 * q0;
        acc0[4] += r0 * r0;
        acc0[5] += r0 * r0 * q0;
        acc1[1] += q1;
        acc1[2] += r1;
        acc1[3] += r1 * q1;
        acc1[4] += r1 * r1;
        acc1[5] += r1 * r1 * q1;
        mn0 = fmin(mn0, mv0);
        mn1 = fmin(mn1, mv1);
    }
    if (np) {
        acc0[0] += log(pr0);
        acc1[0] += log(pr1);
    }
    const int w = tid >> 6, lane = tid & 63;
#pragma unroll
    for (int q = 0; q < 6; ++q) {
        const double v0 = wave_sum(acc0[q]);
        const double v1 = wave_sum(acc1[q]);
        if (lane == 0) {
            sh.red[w][q] = v0;
            sh.red2[w][q] = v1;
        }
    }
    const double vm0 = wave_min(mn0), vm1 = wave_min(mn1);
    if (lane == 0) {
        sh.red[w][6] = vm0;
        sh.red2[w][6] = vm1;
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 7; ++q) {
        double v0 = sh.red[0][q], v1 = sh.red2[0][q];
        for (int ww = 1; ww < kFitBlock / 64; ++ww) {
            v0 = (q == 6) ? fmin(v0, sh.red[ww][q]) : v0 + sh.red[ww][q];
            v1 = (q == 6) ? fmin(v1, sh.red2[ww][q]) : v1 + sh.red2[ww][q];
        }
        if (q < 6) {
            m0.s[q] = v0;
            m1.s[q] = v1;
        } else {
            m0.mn = v0;
            m1.mn = v1;
        }
    }
}
template <int KF>
__device__ __forceinline__ void fit_moments2(const double* __restrict__ x, int64_t a, int64_t b,
                                             const TplDev* __restrict__ T, double n, double phi0, double phi1,
                                             FitShared& sh, FitMom& m0, FitMom& m1) {
    if (fit_prodlen<CRIMP_MODEL_FOURIER, KF>(T, n) == 16)
        fit_moments2_pl<KF, 16>(x, a, b, T, n, phi0, phi1, sh, m0, m1);
    else
        fit_moments2_pl<KF, kFitProd>(x, a, b, T, n, phi0, phi1, sh, m0, m1);
}

// ---------------------------------------------------------------- varyAmps (measureToAs.py:305-312)
// With ampShift A free the model is norm + A*h, and the extended LL, its gradient and Hessian in
// (norm, phShift, A) follow from 11 photon sums; ampShift is bounded by the model's [C.amp_lo, C.amp_hi].

struct FitEval3 {
    double ll, g[3], H[6];  // H = {nn, np, nA, pp, pA, AA}
};

struct FitShared3 {
    double red[kFitBlock / 64][12];
};

__device__ FitEval3 fit_eval3(const double* __restrict__ x, int64_t a, int64_t b, const TplDev* __restrict__ T,
                              double n, double phi, double A, double E, const FitCfg& C, FitShared& sh,
                              FitShared3& s3) {
    const int tid = threadIdx.x;
    const int model = T->model, K = T->K;
    __syncthreads();
    if (tid < K) tpl_coef(T, tid, phi, sh.coef[0][tid], sh.coef[1][tid]);
    __syncthreads();
    // sums: ln mv, q, h q, h1 q, h2 q, q^2, h q^2, h1 q^2, h^2 q^2, h h1 q^2, h1^2 q^2 ; min mv
    double acc[11];
#pragma unroll
    for (int q = 0; q < 11; ++q) acc[q] = 0.0;
    double mn = INFINITY;
    for (int64_t i = a + tid; i < b; i += kFitBlock) {
        double s1, c1, h, h1, h2;
        fit_sincos(model, sh, gld(x, i), s1, c1);
        tpl_terms(T, model, K, sh.coef[0], sh.coef[1], s1, c1, h, h1, h2);
        const double mv = n + A * h;
        const double q = lk_rcp(mv);
        const double q2 = q * q;
        acc[0] += log(mv);
        acc[1] += q;
        acc[2] += h * q;
        acc[3] += h1 * q;
        acc[4] += h2 * q;
        acc[5] += q2;
        acc[6] += h * q2;
        acc[7] += h1 * q2;
        acc[8] += h * h * q2;
        acc[9] += h * h1 * q2;
        acc[10] += h1 * h1 * q2;
        mn = fmin(mn, mv);
    }
    const int w = tid >> 6, lane = tid & 63;
#pragma unroll
    for (int q = 0; q < 11; ++q) {
        const double v = wave_sum(acc[q]);
        if (lane == 0) s3.red[w][q] = v;
    }
    const double vm = wave_min(mn);
    if (lane == 0) s3.red[w][11] = vm;
    __syncthreads();
    double S[12];
#pragma unroll
    for (int q = 0; q < 12; ++q) {
        double v = s3.red[0][q];
        for (int ww = 1; ww < kFitBlock / 64; ++ww) v = (q == 11) ? fmin(v, s3.red[ww][q]) : v + s3.red[ww][q];
        S[q] = v;
    }
    const double N = (double)(b - a);
    FitEval3 r;
    double F;
    if (model == CRIMP_MODEL_FOURIER) {
        F = n;
        r.ll = -n * E + N * log(n * E) + (S[0] - N * log(n));
        r.g[2] = S[2];
    } else {
        F = kTwoPi * n + A * C.sum_amp;
        r.ll = -F * E / kTwoPi + N * log(F * E / kTwoPi) + (S[0] - N * log(F));
        r.g[2] = S[2] - C.sum_amp * E / kTwoPi;
    }
    if (!(S[11] / F > 0)) r.ll = -INFINITY;
    r.g[0] = -E + S[1];
    r.g[1] = A * S[3];
    r.H[0] = -S[5];
    r.H[1] = -A * S[7];
    r.H[2] = -S[6];
    r.H[3] = A * S[4] - A * A * S[10];
    r.H[4] = S[3] - A * S[9];
    r.H[5] = -S[8];
    return r;
}

// Newton direction for the free coordinates (mask bits: 1 norm, 2 phShift, 4 ampShift) of a 3-parameter
// ascent: plain Newton where H is negative definite, else a Levenberg shift by a Gershgorin bound of the largest
// eigenvalue; then a trust region (0.05 rad
// in phShift, half the current norm and ampShift).
__device__ void fit_newton_dir3(const double* v, const FitEval3& e, int mask, double* d) {
    double H[3][3] = {{e.H[0], e.H[1], e.H[2]}, {e.H[1], e.H[3], e.H[4]}, {e.H[2], e.H[4], e.H[5]}};
    double g[3] = {e.g[0], e.g[1], e.g[2]};
    for (int i = 0; i < 3; ++i)
        if (!(mask & (1 << i))) {
            for (int j = 0; j < 3; ++j) H[i][j] = H[j][i] = 0.0;
            H[i][i] = -1.0;
            g[i] = 0.0;
        }
    double lam = -INFINITY, diag = 0.0;
    for (int i = 0; i < 3; ++i) {
        double r = H[i][i];
        for (int j = 0; j < 3; ++j)
            if (j != i) r += fabs(H[i][j]);
        lam = fmax(lam, r);
        diag += fabs(H[i][i]);
    }
    // no shift when H is negative definite (leading principal minors alternate in sign): the Gershgorin bound
    // over-estimates the largest eigenvalue of a badly scaled H (norm vs ampShift entries) and a shift from it
    // shrank every ampShift step to ~2 % of the distance to the optimum
    const double m2 = H[0][0] * H[1][1] - H[0][1] * H[1][0];
    const double m3 = H[0][0] * (H[1][1] * H[2][2] - H[1][2] * H[2][1]) -
                      H[0][1] * (H[1][0] * H[2][2] - H[1][2] * H[2][0]) +
                      H[0][2] * (H[1][0] * H[2][1] - H[1][1] * H[2][0]);
    const bool negdef = H[0][0] < 0.0 && m2 > 0.0 && m3 < 0.0;
    const double shift = (lam < 0 || negdef) ? 0.0 : lam * 1.5 + 1e-6 * diag + 1e-12;
    for (int i = 0; i < 3; ++i) H[i][i] -= shift;
    // solve H d = -g (symmetric 3x3, Cramer)
    const double c00 = H[1][1] * H[2][2] - H[1][2] * H[2][1];
    const double c01 = H[1][2] * H[2][0] - H[1][0] * H[2][2];
    const double c02 = H[1][0] * H[2][1] - H[1][1] * H[2][0];
    const double det = H[0][0] * c00 + H[0][1] * c01 + H[0][2] * c02;
    const double inv[3][3] = {
        {c00 / det, (H[0][2] * H[2][1] - H[0][1] * H[2][2]) / det, (H[0][1] * H[1][2] - H[0][2] * H[1][1]) / det},
        {c01 / det, (H[0][0] * H[2][2] - H[0][2] * H[2][0]) / det, (H[0][2] * H[1][0] - H[0][0] * H[1][2]) / det},
        {c02 / det, (H[0][1] * H[2][0] - H[0][0] * H[2][1]) / det, (H[0][0] * H[1][1] - H[0][1] * H[1][0]) / det}};
    for (int i = 0; i < 3; ++i) d[i] = -(inv[i][0] * g[0] + inv[i][1] * g[1] + inv[i][2] * g[2]);
    double sc = 1.0;
    sc = fmin(sc, 0.5 * fabs(v[0]) / fmax(fabs(d[0]), 1e-300));
    sc = fmin(sc, 0.05 / fmax(fabs(d[1]), 1e-300));
    sc = fmin(sc, 0.5 * fabs(v[2]) / fmax(fabs(d[2]), 1e-300));
    for (int i = 0; i < 3; ++i) d[i] *= sc;
}

// Damped Newton ascent over the free coordinates of v = (norm, phShift, ampShift) within the bounds.
__device__ FitEval3 fit_ascent3(const double* __restrict__ x, int64_t a, int64_t b, const TplDev* __restrict__ T,
                                double* v, int mask, int max_iter, double E, const FitCfg& C, FitShared& sh,
                                FitShared3& s3, int& nev) {
    const double lo[3] = {C.lo, -C.pb, C.amp_lo}, hi[3] = {C.hi, C.pb, C.amp_hi};
    FitEval3 e = fit_eval3(x, a, b, T, v[0], v[1], v[2], E, C, sh, s3);
    ++nev;
    for (int it = 0; it < max_iter; ++it) {
        double d[3];
        int m = mask;  // projected: a coordinate on its bound with the gradient pointing out is held (fit_newton_dir)
        for (int i = 0; i < 3; ++i)
            if ((v[i] <= lo[i] && e.g[i] < 0.0) || (v[i] >= hi[i] && e.g[i] > 0.0)) m &= ~(1 << i);
        fit_newton_dir3(v, e, m, d);
        double t = 1.0, tv[3] = {v[0], v[1], v[2]};
        FitEval3 e2 = e;
        bool ok = false;
        for (int ls = 0; ls < 40; ++ls) {
            for (int i = 0; i < 3; ++i) tv[i] = clipd(v[i] + t * d[i], lo[i], hi[i]);
            e2 = fit_eval3(x, a, b, T, tv[0], tv[1], tv[2], E, C, sh, s3);
            ++nev;
            if (isfinite(e2.ll) && e2.ll >= e.ll - 1e-12 * fabs(e.ll)) {
                ok = true;
                break;
            }
            t *= 0.5;
        }
        if (!ok) break;
        bool moved = false;
        for (int i = 0; i < 3; ++i) {
            const double tol = (i == 1) ? 1e-12 : 1e-12 * fmax(1.0, fabs(tv[i]));
            moved |= fabs(tv[i] - v[i]) >= tol;
            v[i] = tv[i];
        }
        e = e2;
        if (!moved) break;
    }
    return e;
}

// varyAmps fit of one interval: the (norm, phShift) ascent with ampShift = 1, then all three free from there
// (:306-312), then the 1-sigma scan with norm and ampShift re-profiled at each phShift step.
__global__ __launch_bounds__(kFitBlock) void k_toa_fit_amp(const double* __restrict__ x,
                                                           const int64_t* __restrict__ offsets,
                                                           const TplDev* __restrict__ T, const double* __restrict__ expo,
                                                           const double* __restrict__ start, FitCfg C,
                                                           double* __restrict__ out) {
    __shared__ FitShared sh;
    __shared__ FitShared3 s3;
    fit_shared_init(sh);
    const int64_t iv = blockIdx.x;
    const int64_t a = offsets[iv], b = offsets[iv + 1];
    const double E = expo[iv];
    int nev = 0;
    double v[3] = {start[2 * iv], start[2 * iv + 1], 1.0};
    fit_ascent3(x, a, b, T, v, 1 | 2, 60, E, C, sh, s3, nev);
    const FitEval3 em = fit_ascent3(x, a, b, T, v, 1 | 2 | 4, 100, E, C, sh, s3, nev);
    const double nhat = v[0], phat = v[1], ahat = v[2], llmax = em.ll;
    double sig[2];
    for (int s = 0; s < 2; ++s) {
        const int side = s == 0 ? -1 : 1;
        bool past = false;
        int kk = 0;
        for (int k = 1;; ++k) {
            const double target = phat + (double)(side * k) * C.step;
            double ph;
            if (T->model == CRIMP_MODEL_FOURIER) {
                const bool beyond = side < 0 ? (target <= -M_PI) : (target >= M_PI);
                if (beyond && !past) {
                    ph = side < 0 ? -M_PI : M_PI;
                    past = true;
                } else {
                    ph = target;
                }
            } else {
                ph = clipd(target, -C.pb, C.pb);
            }
            double w[3] = {nhat, ph, ahat};
            const FitEval3 ek = fit_ascent3(x, a, b, T, w, 1 | 4, 30, E, C, sh, s3, nev);
            const double diff = llmax - ek.ll;
            if (diff > kHalfChi2OneSigma || (double)(k + 1) > C.kcap) {
                kk = k + 1;
                break;
            }
        }
        sig[s] = sigma_bound(kk, C.step);
    }
    if (threadIdx.x == 0) {
        double* o = out + iv * 8;
        o[0] = nhat;
        o[1] = phat;
        o[2] = llmax;
        o[3] = sig[0];
        o[4] = sig[1];
        o[5] = (double)nev;
        o[6] = ahat;
        o[7] = 0.0;
    }
}

// One workgroup per interval: ascent from start[iv], then the 1-sigma scan on both sides.
// out[iv*8 + 0..7] = norm, phShift, LLmax, phShift_LL, phShift_UL, likelihood evaluations, ampShift (1), and how
// many of those evaluations read the cached template part (bench.py's algorithmic work count).
// Waves per SIMD of the fit kernel: 4 (two 512-thread workgroups per CU, 66 KB of LDS each) holds it to 128 VGPRs;
// hipcc then calls fit_eval out of line and spills only around those calls (once per likelihood pass), and the
// photon loops run at twice the occupancy: 14.9 -> 13.2 ms per 1250 config-5 fits, records bit-identical
// (profiles/r03/ab_fit_tmpl.log; CRIMP_FIT_WPE=2 is the all-inline 221-VGPR build)
#ifndef CRIMP_FIT_WPE
#define CRIMP_FIT_WPE 4
#endif
template <int MODEL, int KF>
__global__ __launch_bounds__(kFitBlock) __attribute__((amdgpu_waves_per_eu(CRIMP_FIT_WPE))) void k_toa_fit(const double* __restrict__ x, const int64_t* __restrict__ offsets,
                                                       const TplDev* __restrict__ T, const double* __restrict__ expo,
                                                       const double* __restrict__ start, FitCfg C,
                                                       double* __restrict__ out, double* __restrict__ hcache) {
    __shared__ FitShared sh;
    fit_shared_init(sh);
    const int64_t iv = blockIdx.x;
    const int64_t a = offsets[iv], b = offsets[iv + 1];
    const double E = expo[iv];
    int nev = 0, ncached = 0;
    double n = start[2 * iv], p = start[2 * iv + 1];
    FitEval e = fit_eval<MODEL, KF>(x, a, b, T, n, p, E, C, sh);
    ++nev;
    for (int it = 0; it < 60; ++it) {  // toafit.maximise
        double dn, dp;
        bool pure = false;
        fit_newton_dir(n, p, C, e, dn, dp, &pure);
        {   // converged: even the full step moves less than the stopping tolerance, so the pass that would confirm
            // it is skipped (toafit.maximise does the same)
            const double fn = clipd(n + dn, C.lo, C.hi), fp = clipd(p + dp, -C.pb, C.pb);
            if (isfinite(e.ll) && fabs(fp - p) < 1e-12 && fabs(fn - n) < 1e-12 * fmax(1.0, fabs(fn))) break;
            if (CRIMP_FIT_MODEL_STEP && pure && isfinite(e.ll) && fn == n + dn && fp == p + dp &&
                fabs(dp) < kFitModelStep && fabs(dn) < kFitModelStep * fmax(1.0, fabs(n))) {
#pragma clang fp contract(off)
                const double q = e.hnn * dn * dn + 2.0 * e.hnp * dn * dp + e.hpp * dp * dp;
                e.ll = e.ll + (e.gn * dn + e.gp * dp + 0.5 * q);
                n = fn;
                p = fp;
                break;
            }
        }
        double t = 1.0, tn = n, tp = p;
        FitEval e2 = e;
        bool ok = false;
        for (int ls = 0; ls < 40; ++ls) {
            tn = clipd(n + t * dn, C.lo, C.hi);
            tp = clipd(p + t * dp, -C.pb, C.pb);
            e2 = fit_eval<MODEL, KF>(x, a, b, T, tn, tp, E, C, sh);
            ++nev;
            if (isfinite(e2.ll) && e2.ll >= e.ll - 1e-12 * fabs(e.ll)) {
                ok = true;
                break;
            }
            t *= 0.5;
        }
        if (!ok) break;  // line search exhausted: at the (numerical) optimum
        const double mvn = fabs(tn - n), mvp = fabs(tp - p);
        n = tn;
        p = tp;
        e = e2;
        if (mvp < 1e-12 && mvn < 1e-12 * fmax(1.0, fabs(tn))) break;
    }
    const double nhat = n, phat = p, llmax = e.ll;
    // toafit.error_scan, measureToAs.py:331-376: both sides step k = 1, 2, ... in lockstep (each side's sequence of
    // phShifts, profiles and stopping rule is its own, so the order of evaluation cannot change a bound); with the
    // moment profile of a compile-time Fourier template a step of both sides is one joint pass (fit_moments2)
    double sig[2];
    int kk[2] = {0, 0};
    bool past[2] = {false, false};
    for (int k = 1; kk[0] == 0 || kk[1] == 0; ++k) {
        double ph[2] = {0.0, 0.0};
        for (int s = 0; s < 2; ++s) {
            if (kk[s]) continue;
            const int side = s == 0 ? -1 : 1;
            const double target = phat + (double)(side * k) * C.step;
            if (MODEL == CRIMP_MODEL_FOURIER) {
                // the first step past +-pi is clipped to the bound; later ones move the bound (:332-334, :357-359)
                const bool beyond = side < 0 ? (target <= -M_PI) : (target >= M_PI);
                if (beyond && !past[s]) {
                    ph[s] = side < 0 ? -M_PI : M_PI;
                    past[s] = true;
                } else {
                    ph[s] = target;
                }
            } else {
                ph[s] = clipd(target, -C.pb, C.pb);
            }
        }
        double llk[2] = {0.0, 0.0};
        bool have[2] = {kk[0] != 0, kk[1] != 0};
        bool iter[2] = {!CRIMP_FIT_MOMENTS, !CRIMP_FIT_MOMENTS};  // the iterative profile (no moment pass first)
        if constexpr (CRIMP_FIT_MOMENTS && CRIMP_FIT_JOINT && MODEL == CRIMP_MODEL_FOURIER && KF > 0) {
            if (!have[0] && !have[1]) {
                const double n0 = clipd(nhat, C.lo, C.hi);
                FitMom m[2];
                fit_moments2<KF>(x, a, b, T, n0, ph[0], ph[1], sh, m[0], m[1]);
                nev += 2;
                for (int s = 0; s < 2; ++s) {
                    have[s] = mom_solve<MODEL>(m[s], n0, E, (double)(b - a), C, llk[s]);
                    iter[s] = true;
                }
            }
        }
        for (int s = 0; s < 2; ++s) {
            if (have[s]) continue;
            if (!iter[s])
                llk[s] = fit_profile_mom<MODEL, KF>(x, a, b, T, ph[s], nhat, E, C, sh, nev);
            else
                llk[s] = fit_profile<MODEL, KF>(x, a, b, T, ph[s], nhat, E, C, sh, nev,
                                                CRIMP_FIT_MOMENTS ? nullptr : hcache, &ncached);
        }
        for (int s = 0; s < 2; ++s) {
            if (kk[s]) continue;
            const double diff = llmax - llk[s];
            if (diff > kHalfChi2OneSigma || (double)(k + 1) > C.kcap) kk[s] = k + 1;
        }
    }
    sig[0] = sigma_bound(kk[0], C.step);
    sig[1] = sigma_bound(kk[1], C.step);
    if (threadIdx.x == 0) {
        double* o = out + iv * 8;
        o[0] = nhat;
        o[1] = phat;
        o[2] = llmax;
        o[3] = sig[0];
        o[4] = sig[1];
        o[5] = (double)nev;
        o[6] = 1.0;
        o[7] = (double)ncached;
    }
}

// lmfit brute maximum per interval from k_toa_grid's per-split partial sums (toafit.brute): splits combined in
// a fixed order, the reference LL formed for every (norm, phShift) lattice point, -inf where the model is not
// positive, first maximum in norm-outer order (scipy.optimize.brute / np.argmax). ``norm`` holds each interval's
// candidate norms (a contiguous run of the grid, in grid order: crimp_toa_fit's pruning), so the order is kept.
__global__ __launch_bounds__(256) void k_toa_grid_best(const double* __restrict__ pl, const double* __restrict__ ph,
                                                       const double* __restrict__ norm, const double* __restrict__ phi,
                                                       const int64_t* __restrict__ offsets,
                                                       const double* __restrict__ expo, int nnorm, int nphi, int nint,
                                                       int splits, int model, double sum_amp, double norm_first,
                                                       double lo, double hi, int plain, double hconst,
                                                       double prod8_scale, int nlazy, int* __restrict__ unsafe,
                                                       const uint64_t* __restrict__ lzmask,
                                                       const int* __restrict__ lzrow,
                                                       const unsigned long long* __restrict__ cnt, int nbins,
                                                       double* __restrict__ start) {
    __shared__ double bv[4];
    __shared__ int bi[4];
    const int64_t iv = blockIdx.x;
    const double N = (double)(offsets[iv + 1] - offsets[iv]);
    const double E = expo[iv];
    double best = -INFINITY;
    int bidx = 0x7fffffff;
    auto lattice_ll = [&](int ai, int bj) -> double {  // the reference LL of lattice point (norm ai, phShift bj)
        if (ai < nlazy) {  // a lazy norm (not evaluated): -inf where the min h invalidates it, else the grid reruns
            if (lzmask) {  // kGridCert: a photon-holding bin whose template bound at this phShift is <= -norm
                const uint64_t m = lzmask[(int64_t)lzrow[iv * nlazy + ai] * nphi + bj];
                bool inv = false;
                for (int b = 0; b < nbins; ++b) inv = inv || (((m >> b) & 1ull) != 0 && cnt[iv * nbins + b] > 0);
                if (!inv) atomicOr(unsafe, 1);
                return (double)-INFINITY;
            }
            double hm = INFINITY;
            for (int sp = 0; sp < splits; ++sp) hm = fmin(hm, ph[((int64_t)sp * nint + iv) * nphi + bj]);
            if ((hm + norm[iv * nnorm + ai]) > 0) atomicOr(unsafe, 1);
            return (double)-INFINITY;
        }
        double v = 0.0;
        for (int sp = 0; sp < splits; ++sp) v += pl[(((int64_t)sp * nint + iv) * nnorm + ai) * nphi + bj];
        const double ln = v * 0.69314718055994530942;  // log2 sums -> ln
        double hm = ph ? INFINITY : hconst;  // no per-phShift min: the host's lower bound of h (crimp_toa_fit)
        if (ph)
            for (int sp = 0; sp < splits; ++sp) hm = fmin(hm, ph[((int64_t)sp * nint + iv) * nphi + bj]);
        const double nn = norm[iv * nnorm + ai];
        double ll;
        if (model == CRIMP_MODEL_FOURIER) {
            ll = -nn * E + N * log(nn * E) + (ln - N * log(nn));
        } else {
            const double F = kTwoPi * nn + sum_amp;
            ll = -F * E / kTwoPi + N * log(F * E / kTwoPi) + (ln - N * log(F));
        }
        if (!((hm + nn) > 0) || !isfinite(ll)) {
            ll = -INFINITY;
        } else if (prod8_scale > 0.0 && (hm + nn) * prod8_scale < 0x1p-15) {
            atomicOr(unsafe, 1);  // a product of eight factors could have underflowed: the host reruns with four
        }
        return ll;
    };
    for (int idx = threadIdx.x; idx < nnorm * nphi; idx += 256) {
        const double ll = lattice_ll(idx / nphi, idx % nphi);
        if (ll > best || (ll == best && idx < bidx)) {
            best = ll;
            bidx = idx;
        }
    }
    // (value, index) argmax, ties -> lowest index
    for (int o = 32; o > 0; o >>= 1) {
        const double ov = __shfl_xor(best, o);
        const int oi = __shfl_xor(bidx, o);
        if (ov > best || (ov == best && oi < bidx)) {
            best = ov;
            bidx = oi;
        }
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        bv[w] = best;
        bi[w] = bidx;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int ww = 1; ww < 4; ++ww)
            if (bv[ww] > best || (bv[ww] == best && bi[ww] < bidx)) {
                best = bv[ww];
                bidx = bi[ww];
            }
        if (bidx == 0x7fffffff) {  // no finite point: the full lattice's first point (norm_first, phi[0])
            start[2 * iv] = norm_first;
            start[2 * iv + 1] = phi[0];
        } else {
            // the ascent starts at the lattice phShift with the norm at the photon rate N/E (the profile optimum
            // solves sum_i 1/(n + h_i) = E, so n* ~ N/E - <h>: within a few % where the lattice is one 26-unit norm
            // step away), unless that is outside the bounds or makes the model non-positive at this phShift; the
            // lattice norm otherwise. Same basin, same maximum, two fewer Newton passes (toafit.fit_host does the same)
            // (plain: the test hook CRIMP_TOA_LATTICE_START, the lattice point itself, as lmfit hands it on)
            const double r = N / E;
            double hmx = ph ? INFINITY : hconst;
            const int bj = bidx % nphi;
            if (ph)
                for (int sp = 0; sp < splits; ++sp) hmx = fmin(hmx, ph[((int64_t)sp * nint + iv) * nphi + bj]);
            const bool use_rate = !plain && r >= lo && r <= hi && hmx + r > 0.0;
            start[2 * iv] = use_rate ? r : norm[iv * nnorm + bidx / nphi];
            // and the phShift at the vertex of the parabola through the maximum and its two lattice neighbours (at
            // the maximum's norm; within half a lattice step), where the model stays well positive
            double ps = phi[bj];
            if (use_rate && hmx + r > 0.5 * r && bj >= 1 && bj + 1 < nphi) {
                const int ai = bidx / nphi;
                const double lm = lattice_ll(ai, bj - 1), l0 = best, lp = lattice_ll(ai, bj + 1);
                const double den = lm - 2.0 * l0 + lp;
                if (isfinite(lm) && isfinite(lp) && den < 0.0) {
                    const double d = fmin(0.5, fmax(-0.5, 0.5 * (lm - lp) / den));
                    ps = phi[bj] + d * (phi[bj + 1] - phi[bj]);
                }
            }
            start[2 * iv + 1] = ps;
        }
    }
}

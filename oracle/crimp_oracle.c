/*
 * crimp_oracle.c -- CPU restatement of CRIMP's photon hot path (TEST INFRASTRUCTURE).
 *
 * This file is the parity CHECKER, never the product: only tests/, the
 * __graft_entry__.smoke() check and bench.py's cpu_baseline leg may load it.
 * The shipped path (crimp_amd/, libcrimp_hip.so) must never link or call it.
 *
 * Plain fp64 C, one function per reference routine, each citing the reference
 * file:line it restates (paths relative to georgeyounes/CRIMP v2.3.0, src/crimp/).
 * Pinned against the reference's own outputs: tests/golden/ fixtures were produced
 * by importing the reference (tests/golden/gen_golden.py) and the worked-example
 * table data/ToAs_2259.txt rows 35-41.
 *
 * OpenMP parallelises the trial axis of the periodicity searches (the CPU
 * baseline timed by bench.py); every per-trial sum is computed serially in
 * photon order, so results do not depend on the thread count.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

#define ORC_PI 3.141592653589793238462643383279502884

/* The search sums use fma() and rint() on every term: built for FMA3 hosts (hardware fma, roundsd via AVX) with a baseline
 * clone selected at load time on older hosts (the library is built here and runs on the GPU box's host too). */
#if defined(__x86_64__) && defined(__GNUC__)
#define ORC_CLONES __attribute__((target_clones("fma", "default")))
#else
#define ORC_CLONES
#endif

/* ------------------------------------------------------------------------ */
/* Timing model (values of the .par dictionary, readtimingmodel.py:212-233)  */
/* ------------------------------------------------------------------------ */
typedef struct {
    double pepoch;
    double f[13];              /* F0..F12, missing ones are 0 (readtimingmodel.py:64-65) */
    int32_t n_glitch;
    double glitch[32][7];      /* GLEP, GLPH, GLF0, GLF1, GLF2, GLF0D, GLTD (calcphase.py:99-110) */
    int32_t n_wave;            /* number of WAVEj harmonics used (calcphase.py:135,142) */
    double wave_epoch, wave_om;
    double wave_ab[64][2];
} orc_model;

int orc_max_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

void orc_set_threads(int n) {
#ifdef _OPENMP
    if (n > 0) omp_set_num_threads(n);
#else
    (void)n;
#endif
}

/* calcphase.py:73-85  phases_te = sum_{n=1..13} (1/n!) F_{n-1} dt^n, dt=(t-PEPOCH)*86400,
 * summed in increasing n with dt**n as in the reference (pow). */
static double te_phase(const orc_model* m, double t) {
    double dt = (t - m->pepoch) * 86400.0;
    double acc = 0.0, fact = 1.0;
    for (int n = 1; n <= 13; ++n) {
        fact *= (double)n;
        acc += (1.0 / fact) * m->f[n - 1] * pow(dt, (double)n);
    }
    return acc;
}

/* calcphase.py:87-126 (glitches): mask t >= GLEP; GLTD == 0 disables the exp term (:115). */
static double gl_phase(const orc_model* m, double t) {
    double acc = 0.0;
    for (int j = 0; j < m->n_glitch; ++j) {
        const double* g = m->glitch[j];
        if (!(t >= g[0])) continue;
        double dts = (t - g[0]) * 86400.0;
        double ex = (g[6] == 0.0) ? 0.0 : (g[6] * 86400.0) * (1.0 - exp(-(t - g[0]) / g[6]));
        acc += g[1] + g[2] * dts + 0.5 * g[3] * dts * dts + (1.0 / 6.0) * g[4] * dts * dts * dts + g[5] * ex;
    }
    return acc;
}

/* calcphase.py:128-149 (waves): F0 * sum_j (A_j sin(j*om*(t-EPOCH)) + B_j cos(...)). */
static double wave_phase(const orc_model* m, double t) {
    if (m->n_wave <= 0) return 0.0;
    double acc = 0.0;
    for (int j = 1; j <= m->n_wave; ++j) {
        double arg = j * m->wave_om * (t - m->wave_epoch);
        acc += m->wave_ab[j - 1][0] * sin(arg) + m->wave_ab[j - 1][1] * cos(arg);
    }
    return acc * m->f[0];
}

/* calcphase.py:152-176: total = te + gl + wav; folded = total - floor(total).
 * parts: bit0 te, bit1 glitches, bit2 waves (Phases.taylorexpansion/.glitches/.waves). */
void orc_calcphase(const double* t, int64_t n, const orc_model* m, int parts, double* total, double* folded) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
        double te = (parts & 1) ? te_phase(m, t[i]) : 0.0;
        double gl = (parts & 2) ? gl_phase(m, t[i]) : 0.0;
        double wv = (parts & 4) ? wave_phase(m, t[i]) : 0.0;
        double tot = te + gl + wv;
        total[i] = tot;
        if (folded) folded[i] = tot - floor(tot);
    }
}

/* periodsearch.py:57-71 (ztest), :73-106 (twod_ztest), :109-125 (htest).
 * The argument is built exactly as the reference does:
 *   1-D: 2*(kk+1)*pi*f*(t-t0)
 *   2-D: 2*(kk+1)*pi*(f*(t-t0) + (0.5*(-1*10**fd))*(t-t0)**2)
 * stat 0 = Z^2_m; stat 1 = H (max of cumsum(Z^2_k) - 4*(k-1)).
 * out is [nfd*nf] with fd outer, f inner (periodsearch.py:264-278). nfd==0 => 1-D. */
/* cos(a), sin(a) of the fp64 argument a, as accurate as libm's (a few 1e-16 absolute) but without libm's slow
 * large-argument path (glibc switches to Payne-Hanek reduction above ~1e8 rad, where the config-4 arguments
 * 2 pi k f dt ~ 4e9 rad live: ~110 ns per term). Reduction by 2 pi = P1 + P2 (+ < 6e-33): with k = rint(a / 2 pi),
 * a - k P1 is a multiple of 2^-50 below 4 in magnitude for |a| < 2^40, so the fma is exact; k P2 <= 2^38 x 2.5e-16
 * adds one rounding of the reduced angle. The argument itself is the reference's, unchanged. */
/* sin, cos of |x| <= pi/4 + 1e-9: Taylor series to x^17 / x^18 (truncation < 1e-19), Horner in fp64 (~1 ulp) */
static inline __attribute__((always_inline)) void orc_sincos_small(double x, double* s, double* c) {
    const double x2 = x * x;
    double ps = 1.0 / 355687428096000.0;                 /* 1/17! */
    ps = fma(ps, -x2, 1.0 / 1307674368000.0);            /* 1/15! */
    ps = fma(ps, -x2, 1.0 / 6227020800.0);               /* 1/13! */
    ps = fma(ps, -x2, 1.0 / 39916800.0);                 /* 1/11! */
    ps = fma(ps, -x2, 1.0 / 362880.0);
    ps = fma(ps, -x2, 1.0 / 5040.0);
    ps = fma(ps, -x2, 1.0 / 120.0);
    ps = fma(ps, -x2, 1.0 / 6.0);
    *s = fma(-x * x2, ps, x);
    double pc = 1.0 / 6402373705728000.0;                /* 1/18! */
    pc = fma(pc, -x2, 1.0 / 20922789888000.0);           /* 1/16! */
    pc = fma(pc, -x2, 1.0 / 87178291200.0);              /* 1/14! */
    pc = fma(pc, -x2, 1.0 / 479001600.0);                /* 1/12! */
    pc = fma(pc, -x2, 1.0 / 3628800.0);
    pc = fma(pc, -x2, 1.0 / 40320.0);
    pc = fma(pc, -x2, 1.0 / 720.0);
    pc = fma(pc, -x2, 1.0 / 24.0);
    pc = fma(pc, -x2, 0.5);
    *c = fma(-x2, pc, 1.0);
}

/* cos/sin of r - q pi/2 -> of r by the quadrant q (mod 4) */
static inline __attribute__((always_inline)) void orc_quadrant(double s0, double c0, int64_t q, double* c, double* s) {
    switch ((int)(q & 3)) {
        case 0: *c = c0; *s = s0; break;
        case 1: *c = -s0; *s = c0; break;
        case 2: *c = -c0; *s = -s0; break;
        default: *c = s0; *s = -c0; break;
    }
}

static inline __attribute__((always_inline)) void orc_cossin(double a, double* c, double* s) {
    /* 2 pi = P1 + P2 (+ < 6e-33), pi/2 = H1 + H2 (+ < 2e-33) */
    static const double P1 = 6.283185307179586232, P2 = 2.4492935982947063e-16, INV = 0.15915494309189535;
    static const double H1 = 1.5707963267948966, H2 = 6.123233995736766e-17, INVH = 0.6366197723675814;
    if (!(fabs(a) < 1099511627776.0)) {
        *c = cos(a);
        *s = sin(a);
        return;
    }
    const double k = rint(a * INV);
    const double r = fma(-k, P2, fma(-k, P1, a));   /* |r| <= pi + 1e-15 */
    const double q = rint(r * INVH);                 /* quadrant, |q| <= 2 */
    const double x = fma(-q, H2, fma(-q, H1, r));    /* |x| <= pi/4 + 1e-15; fma(-q, H1, r) exact */
    double s0, c0;
    orc_sincos_small(x, &s0, &c0);
    orc_quadrant(s0, c0, (int64_t)q, c, s);
}

/* Harmonic sums of one trial over photons [i0, i1) (the inner loops of periodsearch.py:66-69,
 * :97-100 and :118-121). */
ORC_CLONES static void trial_sums(const double* time, int64_t i0, int64_t i1, double t0, double f, double c2, int twod,
                       int k, double* sc_out, double* ss_out) {
    double pre = 2.0 * (double)(k + 1) * ORC_PI;
    double sc = 0.0, ss = 0.0, c, s;
    if (twod) {
        for (int64_t i = i0; i < i1; ++i) {
            double dt = time[i] - t0;
            double a = pre * (f * dt + c2 * (dt * dt));
            orc_cossin(a, &c, &s);
            sc += c;
            ss += s;
        }
    } else {
        double pf = pre * f;
        for (int64_t i = i0; i < i1; ++i) {
            double a = pf * (time[i] - t0);
            orc_cossin(a, &c, &s);
            sc += c;
            ss += s;
        }
    }
    *sc_out = sc;
    *ss_out = ss;
}

/* The same sums with the EXACT argument of the given inputs: phase in cycles (k+1)(f dt + c2 dt^2) carried in
 * double-double (error-free products by fma), reduced to a centred fraction before the 2 pi multiply. This is the
 * value the reference's formula has on these fp64 inputs in exact arithmetic -- the reference's own fp64 argument
 * rounds by ~2^-53 of |a| per term (up to ~1e-6 rad at config 4), which this variant measures. Not a restatement
 * of any reference routine: it is the yardstick both the reference and the device kernels are measured against. */
ORC_CLONES static void trial_sums_true(const double* time, int64_t i0, int64_t i1, double t0, double f, double c2, int twod,
                            int k, double* sc_out, double* ss_out) {
    const double kk = (double)(k + 1);
    double sc = 0.0, ss = 0.0, c, s;
    for (int64_t i = i0; i < i1; ++i) {
        const double dt = time[i] - t0;              /* exact: t and t0 within a factor 2 (Sterbenz) */
        double uh = f * dt, ul = fma(f, dt, -uh);    /* f dt = uh + ul exactly */
        if (twod) {
            const double d2h = dt * dt, d2l = fma(dt, dt, -d2h);
            const double wh = c2 * d2h, wl = fma(c2, d2h, -wh) + c2 * d2l;
            const double sh = uh + wh, bb = sh - uh;  /* two-sum of uh + wh */
            const double se = (uh - (sh - bb)) + (wh - bb);
            uh = sh;
            ul = ul + wl + se;
        }
        const double ph = kk * uh, pl = fma(kk, uh, -ph) + kk * ul;
        const double fr = (ph - rint(ph)) + pl;      /* ph - rint(ph) is exact */
        const double q = rint(4.0 * fr);             /* quadrant: fr = q/4 + y, |y| <= 1/8 (+ 1e-9) */
        double s0, c0;
        orc_sincos_small(2.0 * ORC_PI * (fr - 0.25 * q), &s0, &c0);   /* fr - q/4 is exact */
        orc_quadrant(s0, c0, (int64_t)q, &c, &s);
        sc += c;
        ss += s;
    }
    *sc_out = sc;
    *ss_out = ss;
}

typedef void (*orc_sums_fn)(const double*, int64_t, int64_t, double, double, double, int, int, double*, double*);

static double combine(const double* z, int nharm, int stat, int64_t n) {
    if (stat == 0) {
        double s = 0.0;
        for (int k = 0; k < nharm; ++k) s += z[k];
        return s * (2.0 / (double)n);
    }
    double cum = 0.0, best = -INFINITY;
    for (int k = 0; k < nharm; ++k) {
        cum += z[k] * (2.0 / (double)n);
        double v = cum - 4.0 * (double)k;
        if (v > best) best = v;
    }
    return best;
}

/* Few trials over many photons (the full-size parity checks: 1e8 photons, a handful of trials):
 * parallel over (trial, harmonic, photon block) with a FIXED block count, blocks summed in
 * order, so the result does not depend on the thread count either. */
#define ORC_PBLOCKS 256
static void orc_search_photon_blocked(orc_sums_fn sums, const double* time, int64_t n, double t0,
                                      const double* freq, int64_t nf, const double* fd, int64_t nfd, int nharm,
                                      int stat, double* out) {
    int64_t rows = nfd > 0 ? nfd : 1;
    int64_t total = rows * nf;
    int64_t nb = ORC_PBLOCKS, bs = (n + nb - 1) / nb;
    double* part = (double*)malloc(sizeof(double) * 2 * (size_t)(total * nharm * nb));
#pragma omp parallel for collapse(3) schedule(dynamic, 1)
    for (int64_t idx = 0; idx < total; ++idx)
        for (int k = 0; k < nharm; ++k)
            for (int64_t b = 0; b < nb; ++b) {
                int64_t r = idx / nf, j = idx % nf;
                double c2 = nfd > 0 ? 0.5 * (-1.0 * pow(10.0, fd[r])) : 0.0;
                int64_t i0 = b * bs, i1 = i0 + bs < n ? i0 + bs : n;
                double* o = part + 2 * ((idx * nharm + k) * nb + b);
                if (i0 >= i1) { o[0] = o[1] = 0.0; continue; }
                sums(time, i0, i1, t0, freq[j], c2, nfd > 0, k, o, o + 1);
            }
    double* z = (double*)malloc(sizeof(double) * (size_t)nharm);
    for (int64_t idx = 0; idx < total; ++idx) {
        for (int k = 0; k < nharm; ++k) {
            double sc = 0.0, ss = 0.0;
            const double* o = part + 2 * ((idx * nharm + k) * nb);
            for (int64_t b = 0; b < nb; ++b) { sc += o[2 * b]; ss += o[2 * b + 1]; }
            z[k] = sc * sc + ss * ss;
        }
        out[idx] = combine(z, nharm, stat, n);
    }
    free(z);
    free(part);
}

static void orc_search_with(orc_sums_fn sums, const double* time, int64_t n, double t0, const double* freq,
                            int64_t nf, const double* fd, int64_t nfd, int nharm, int stat, double* out) {
    int64_t rows = nfd > 0 ? nfd : 1;
    int64_t total = rows * nf;
    if (total < 64 && n >= (1 << 22)) {
        orc_search_photon_blocked(sums, time, n, t0, freq, nf, fd, nfd, nharm, stat, out);
        return;
    }
#pragma omp parallel
    {
        double* z = (double*)malloc(sizeof(double) * (size_t)(nharm > 0 ? nharm : 1));
#pragma omp for schedule(dynamic, 1)
        for (int64_t idx = 0; idx < total; ++idx) {
            int64_t r = idx / nf, j = idx % nf;
            double c2 = nfd > 0 ? 0.5 * (-1.0 * pow(10.0, fd[r])) : 0.0;
            for (int k = 0; k < nharm; ++k) {
                double sc, ss;
                sums(time, 0, n, t0, freq[j], c2, nfd > 0, k, &sc, &ss);
                z[k] = sc * sc + ss * ss;
            }
            out[idx] = combine(z, nharm, stat, n);
        }
        free(z);
    }
}

void orc_search(const double* time, int64_t n, double t0, const double* freq, int64_t nf,
                const double* fd, int64_t nfd, int nharm, int stat, double* out) {
    orc_search_with(trial_sums, time, n, t0, freq, nf, fd, nfd, nharm, stat, out);
}

/* Same statistic with exact arguments (trial_sums_true): the yardstick for the argument-rounding analysis of the
 * full-size parity tests, not a reference routine. */
void orc_search_true(const double* time, int64_t n, double t0, const double* freq, int64_t nf,
                     const double* fd, int64_t nfd, int nharm, int stat, double* out) {
    orc_search_with(trial_sums_true, time, n, t0, freq, nf, fd, nfd, nharm, stat, out);
}

/* cos/sin of orc_cossin for a vector of arguments (CPU test of the reduction against libm) */
ORC_CLONES void orc_cossin_vec(const double* a, int64_t n, double* c, double* s) {
    for (int64_t i = 0; i < n; ++i) orc_cossin(a[i], c + i, s + i);
}

/* ------------------------------------------------------------------------ */
/* Unbinned extended likelihoods (templatemodels.py:98-121, 201-226, 306-329) */
/* ------------------------------------------------------------------------ */
/* model: 0 fourier (x in cycles), 1 wrapped cauchy, 2 von mises (x in radians).
 * p1 = amp_j, p2 = ph_j (fourier) or cen_j, p3 = wid_j (cauchy/vm), i0k = I0(1/wid^2) for VM.
 *
 * All three reduce to LL(n, phi) = -n*E + sum_i ln(n + a*h_i(phi)) + C(n-independent) with
 * the reference's exact constant terms restored below, so this routine also returns the
 * first and second derivatives in (n, phi) used by the profile fits:
 *   out[0] = LL (reference formula), out[1] = dLL/dn, out[2] = dLL/dphi,
 *   out[3] = d2/dn2, out[4] = d2/dn dphi, out[5] = d2/dphi2, out[6] = min(model/norm-factor)
 * LL is -inf when any model value <= 0 (templatemodels.py:113-115,220-222,324-326). */
static void h_terms(int model, int K, const double* p1, const double* p2, const double* p3, const double* i0k,
                    double amps, double x, double phi, double* h, double* h1, double* h2) {
    double s0 = 0.0, s1 = 0.0, s2 = 0.0;
    for (int j = 0; j < K; ++j) {
        if (model == 0) {
            double jj = (double)(j + 1);
            double arg = jj * 2.0 * ORC_PI * x + p2[j] - jj * phi;
            double a = p1[j] * amps;
            double c = cos(arg), s = sin(arg);
            s0 += a * c;
            s1 += a * jj * s;          /* d/dphi of cos(arg) = +j sin(arg) */
            s2 += -a * jj * jj * c;
        } else if (model == 1) {
            double a = p1[j] * amps / (2.0 * ORC_PI);
            double sh = sinh(p3[j]), ch = cosh(p3[j]);
            double u = x - p2[j] - phi;
            double cu = cos(u), su = sin(u);
            double D = ch - cu;
            double v = a * sh / D;
            /* dv/du = -a sh su / D^2 ; du/dphi = -1 */
            double dvdu = -a * sh * su / (D * D);
            double d2vdu2 = -a * sh * (cu / (D * D) - 2.0 * su * su / (D * D * D));
            s0 += v;
            s1 += -dvdu;
            s2 += d2vdu2;
        } else {
            double kap = 1.0 / (p3[j] * p3[j]);
            double b = p1[j] * amps / (2.0 * ORC_PI * i0k[j]);
            double u = x - p2[j] - phi;
            double cu = cos(u), su = sin(u);
            double v = b * exp(kap * cu);
            double dvdu = -kap * su * v;
            double d2vdu2 = (-kap * cu + kap * kap * su * su) * v;
            s0 += v;
            s1 += -dvdu;
            s2 += d2vdu2;
        }
    }
    *h = s0;
    *h1 = s1;
    *h2 = s2;
}

void orc_toa_eval(const double* x, int64_t n, double exposure, int model, int K, const double* p1,
                  const double* p2, const double* p3, const double* i0k, double amps, double norm, double phi,
                  double* out) {
    double lsum = 0.0, g_n = 0.0, g_p = 0.0, h_nn = 0.0, h_np = 0.0, h_pp = 0.0, mn = INFINITY;
    double atot = 0.0;
    for (int j = 0; j < K; ++j) atot += p1[j] * amps;
    /* normalising factor: fourier -> norm ; cauchy/vm -> 2*pi*norm + sum(amp*ampShift) */
    double F = (model == 0) ? norm : 2.0 * ORC_PI * norm + atot;
    for (int64_t i = 0; i < n; ++i) {
        double h, h1, h2;
        h_terms(model, K, p1, p2, p3, i0k, amps, x[i], phi, &h, &h1, &h2);
        double mv = norm + h;
        double r = mv / F;
        if (r < mn) mn = r;
        lsum += log(r);
        double q = 1.0 / mv;
        g_n += q;
        g_p += h1 * q;
        h_nn -= q * q;
        h_np -= h1 * q * q;
        h_pp += h2 * q - h1 * h1 * q * q;
    }
    double ll;
    if (mn <= 0.0) {
        ll = -INFINITY;
    } else if (model == 0) {
        ll = -norm * exposure + (double)n * log(norm * exposure) + lsum;
    } else {
        ll = -F * exposure / (2.0 * ORC_PI) + (double)n * log(F * exposure / (2.0 * ORC_PI)) + lsum;
    }
    out[0] = ll;
    out[1] = -exposure + g_n;
    out[2] = g_p;
    out[3] = h_nn;
    out[4] = h_np;
    out[5] = h_pp;
    out[6] = mn;
}

/* Batched brute grid (lmfit brute over norm x phShift, measureToAs.py:292-295):
 * ll[a*nphi + b] = LL(norm_grid[a], phi_grid[b]). */
void orc_toa_grid(const double* x, int64_t n, double exposure, int model, int K, const double* p1,
                  const double* p2, const double* p3, const double* i0k, double amps, const double* norms,
                  int64_t nn, const double* phis, int64_t np_, double* ll) {
#pragma omp parallel for collapse(2) schedule(dynamic, 1)
    for (int64_t a = 0; a < nn; ++a)
        for (int64_t b = 0; b < np_; ++b) {
            double o[7];
            orc_toa_eval(x, n, exposure, model, K, p1, p2, p3, i0k, amps, norms[a], phis[b], o);
            ll[a * np_ + b] = o[0];
        }
}

// search_nufft.h -- Z^2_m / H periodicity search by a non-uniform FFT over an arithmetic-progression trial grid
// (CRIMP_FLAG_NUFFT, PeriodSearch(..., precision="nufft")). Included by crimp_hip.hip after the exact path's host
// code (it uses Scratch, grid_is_progression's delta and fixup_search).
//
// The reference (periodsearch.py:67, :93-99, :120-121) evaluates, for every trial f_j and harmonic k,
//   A_k(f_j) = sum_i exp(2 pi i k (f_j dt_i + c2 dt_i^2))        (C_k = Re A_k, S_k = Im A_k)
// photon by photon: O(N M) per harmonic. On an arithmetic progression f_j = fc + jc delta (jc = j - h, h = nf/2,
// fc = f_0 + h delta) the sum over trials is a type-1 non-uniform DFT:
//   A_k(j) = sum_i c_i exp(2 pi i jc u_i / n),   c_i = exp(2 pi i k (fc dt_i + c2 dt_i^2)),   u_i = n k delta dt_i,
// with n a power of two >= nf. Writing u_i = g_i + e_i (g_i = rint(u_i), |e_i| <= 1/2), the sub-cell factor
// exp(2 pi i jc e_i / n) = exp(2 i z e_i), z = pi jc / n (|z| <= pi/2), is expanded in Chebyshev polynomials of
// 2 e_i (Jacobi-Anger; nu_bes): exp(2 i z e) = sum_p eps_p i^p J_p(z) T_p(2e), so with P "moments"
//   A_k(j) = sum_{p<P} eps_p i^p J_p(z) * B_p(jc mod n),   B_p(J) = sum_g b_p[g] exp(2 pi i J g / n),
//   b_p[g] = sum_{i : g_i = g (mod n)} c_i T_p(2 e_i).
// |T_p| <= 1 and |J_p(z)| <= (|z|/2)^p / p!, so |A_k error| <= 2 N sum_{p>=P} (|z|/2)^p / p! < 2.4 N (x/2)^P / P!
// with x = pi |jc| / n; P and n are chosen so that the bound is <= kNuEps at the grid's edge (16 moments at config 3;
// a Taylor expansion in e_i, bound N x^P / P!, needs 20).
// The cost is O(N m P) for the moments plus O(m P n log n) for the FFTs, against O(N M m) for the direct sum.
//
// Kernels (one pass = harmonics k0 .. k0+G-1 of up to 8 trial-grid rows):
//   k_nu_spread   photons -> per-(chunk, cell) moment sums. Each wave owns a chunk of kNuCW time-ordered photons;
//                 4 photons x 16 moments form the A operand and 4 photons x 8 rows x (re, im) of c_i the B operand
//                 of v_mfma_f64_16x16x4_f64, whose accumulator sums the photons of the current cell in fp64 (no
//                 reduction, no atomics). A cell change (photons are sorted, so cells only grow) flushes the 16 x 16
//                 tile to the cell's slot: slot(chunk c, cell G) = G - G_min + c is unique per (c, G).
//   k_nu_merge    slots -> W[batch][g]: every wrapped cell g sums its unwrapped cells G = g (mod n) and, per G, the
//                 chunks that hold it, in chunk order (deterministic), transposed to batch-major rows.
//   k_nu_fft_cols, k_nu_fft_rows   four-step FFT (n = n1 n2, Stockham autosort stages of radix 16/8/4/2 in LDS,
//                 positive exponent); a single row pass for n <= 4096.
//   k_nu_combine  the moments' Bessel-weighted sum at every trial -> (C_k, S_k) (fused into the row pass by
//                 default: k_nu_rows_combine8 / k_nu_fft_rows_combine).
//   k_nu_finalize Z^2 / H in the reference's formula order and the certificate (fix-up list, as the exact path).
#pragma once

typedef double nu_f64x4 __attribute__((ext_vector_type(4)));

constexpr int kNuCW = 1024;        // photons per wave chunk (256 K-groups of 4 photons)
constexpr int kNuWaves = 4;        // chunks per 256-thread block
constexpr int kNuRows = 8;         // trial-grid rows per pass (8 rows x re/im = the 16 MFMA columns)
constexpr int kNuMaxP = 16;        // moments of the MFMA spread (its 16 A rows)
constexpr int kNuGatherMaxP = 24;  // moments of the cell-gather spread (registers)
constexpr int kNuMergeG = 16;      // wrapped cells per merge block
constexpr int kNuMaxWrap = 32;     // unwrapped cells per wrapped cell (span of the photons over n)
constexpr int kNuTile = 4096;      // complex elements per FFT block (64 KB of LDS), 16 per thread
constexpr double kNuEps = 5e-14;   // truncation bound per photon at the grid's edge (below the rounding term kNuRho)
// Z^2_m with m >= 2: 5e-13. The certificate flags a trial when its power's bound exceeds 1e-6 of the power, and Z^2_m's
// bound over its power is sum_k (2 |A_k| E + E^2) / sum_k |A_k|^2 -- at E = N (5e-13 + kNuRho) only trials whose every
// |A_k| is below ~2e-5 N are flagged (none at config 3, P 15 -> 14). Z^2_1 and H keep kNuEps: H = max_m (Z^2_m - 4m + 4)
// cancels to near 0 on noise, where a larger E flags many more trials for the fp64 fix-up (config 4: 55 at kNuEps).
constexpr double kNuEpsZm = 5e-13;
// Rounding bound per photon for the certificate, in units of |A_k|'s scale N: c_i (cis table + fp64 polynomial,
// angle-addition over <= 8 harmonics: ~20 ulp), the MFMA's fp64 accumulation over <= 256 K-groups per cell run
// (<= 256 ulp of the run's sum of |terms|, each <= 1), the merge, the FFT (~3 log2 n ulp) and Horner (e^x ulp):
// < 4e-14 N; kept at 1e-13 N.
constexpr double kNuRho = 1e-13;

constexpr int kNuPassMax = 10;  // harmonics per MFMA spread pass (k_nu_spread<G>, G <= 10)
struct NuPass {          // one spread pass: the slot array of each harmonic k0 + kk
    int64_t gmin[kNuPassMax];   // unwrapped cell of dt[0]
    int64_t ubase[kNuPassMax];  // offset (doubles) of the harmonic's slots in U
};

struct NuTw {            // w_n^t = hi[t >> lbits] * lo[t & (2^lbits - 1)], t in [0, n)
    const double2* lo;
    const double2* hi;
    int lbits;
    int64_t mask;        // n - 1
};

__device__ __forceinline__ double2 nu_cmul(double2 a, double2 b) {
    return make_double2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ double2 nu_add(double2 a, double2 b) { return make_double2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ double2 nu_sub(double2 a, double2 b) { return make_double2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ double2 nu_muli(double2 a) { return make_double2(-a.y, a.x); }  // i * a

__device__ __forceinline__ double2 nu_tw(const NuTw& T, int64_t t) {
    t &= T.mask;
    return nu_cmul(T.hi[t >> T.lbits], T.lo[t & ((int64_t(1) << T.lbits) - 1)]);
}

// e^{2 pi i x}, |x| <= 0.5 (+ a few ulp): 1024-entry table of the coarse angle and the fp64 series of the residual
// angle |theta| <= pi/1024 (omitted terms < 1e-24).
__device__ __forceinline__ double2 nu_cis(const double2* __restrict__ tab, double x) {
    const double t = rint(x * 1024.0);
    const double r = fma(t, -1.0 / 1024.0, x);  // exact
    const double th = r * 6.283185307179586476925286766559;
    const double t2 = th * th;
    const double c = fma(t2, fma(t2, fma(t2, fma(t2, 1.0 / 40320.0, -1.0 / 720.0), 1.0 / 24.0), -0.5), 1.0);
    const double s = th * fma(t2, fma(t2, fma(t2, fma(t2, 1.0 / 362880.0, -1.0 / 5040.0), 1.0 / 120.0), -1.0 / 6.0), 1.0);
    const double2 T = tab[((int)t) & 1023];
    return make_double2(T.x * c - T.y * s, T.x * s + T.y * c);
}

// e^{2 pi i x}, |x| <= 0.5 (+ a few ulp), from a 2048-entry table (the cell gather keeps it in LDS) and the residual
// series to degree 4 / 5 (|theta| <= pi/2048: omitted terms < 2e-20)
__device__ __forceinline__ double2 nu_cis2(const double2* __restrict__ tab, double x) {
    const double t = rint(x * 2048.0);
    const double r = fma(t, -1.0 / 2048.0, x);  // exact
    const double th = r * 6.283185307179586476925286766559;
    const double t2 = th * th;
    const double c = fma(t2, fma(t2, 1.0 / 24.0, -0.5), 1.0);
    const double s = th * fma(t2, fma(t2, 1.0 / 120.0, -1.0 / 6.0), 1.0);
    const double2 T = tab[((int)t) & 2047];
    return make_double2(T.x * c - T.y * s, T.x * s + T.y * c);
}

// frac(a * d) for a = ahi + alo (double-double), as hi part reduced exactly plus the product's rounding error.
// Contraction off: fused into fma(ahi, d, -rint(p)), the reduction would already hold the rounding error that pe
// adds again (a phase error of ulp(a d), ~1e-11 cycles at config-3 arguments).
__device__ __forceinline__ double nu_frac_prod(double ahi, double alo, double d) {
#pragma clang fp contract(off)
    const double p = ahi * d;
    const double pe = fma(ahi, d, -p) + alo * d;
    return (p - rint(p)) + pe;
}

// frac(c2 d^2) with d^2 = d2 + d2e (double-double), contraction off as nu_frac_prod
__device__ __forceinline__ double nu_frac_c2(double c2, double d2, double d2e) {
#pragma clang fp contract(off)
    const double qv = c2 * d2;
    const double qe = fma(c2, d2, -qv) + c2 * d2e;
    return (qv - rint(qv)) + qe;
}

// frac(k phi) for |phi| <= 1/2, the product's rounding error carried (contraction off)
__device__ __forceinline__ double nu_frac_k(double kd, double phi) {
#pragma clang fp contract(off)
    const double hk = kd * phi;
    const double hl = fma(kd, phi, -hk);
    return (hk - rint(hk)) + hl;
}

// Chebyshev-Bessel expansion of the moments' phase factor (Jacobi-Anger): for |e| <= 1/2 and theta = 2 pi jc / n,
//   e^{i theta e} = sum_p eps_p i^p J_p(theta / 2) T_p(2 e),  eps_0 = 1, eps_p = 2,
// so the spread accumulates Chebyshev moments sum c_i T_p(2 e_i) and the combine weights moment p's transform by
// eps_p i^p J_p(z), z = pi jc / n (|z| <= pi / 2). Truncating at P moments errs by <= 2 N sum_{p >= P} (|z|/2)^p / p!
// (< 2.4 N (|z|/2)^P / P! for P >= 4), against N (2|z|)^P / P! for Taylor moments e^p: 20 -> 16 moments at config 3.
// J_p(z) = (z/2)^p sum_{m < kNuBesM} y^m / (m! (m+p)!), y = -(z/2)^2 (|y| <= 0.617: the omitted terms < 4e-18 of
// J_p); the coefficients 1 / (m! (m+p)!) come from the host tables (nu_tables), read at uniform indices.
constexpr int kNuBesP = 26, kNuBesM = 12;
__device__ __forceinline__ double nu_bes_series(const double* __restrict__ bc, int p, double y) {
    const double* c = bc + p * kNuBesM;
    double f = c[kNuBesM - 1];
#pragma unroll
    for (int m = kNuBesM - 2; m >= 0; --m) f = fma(f, y, c[m]);
    return f;  // J_p(z) / (z/2)^p
}
// The combine walks the moments from P-1 down to 0 with J_p by the backward recurrence
// J_p = (2 (p+1) / z) J_p+1 - J_p+2 (stable: J_p is its minimal solution), started from J_P, J_P+1 by the series.
// z = 0 (jc = 0): J_p = 0 for p > 0 (zero start, 2/z taken as 0) and J_0 = 1 (nu_bes_w).
struct NuBes {
    double j1, j2, iz2;  // J_p+1, J_p+2, 2/z
};
__device__ __forceinline__ NuBes nu_bes_start(const double* __restrict__ bc, int P, double zh) {
    double zp = 1.0;
    for (int p = 0; p < P; ++p) zp *= zh;  // (z/2)^P
    const double y = -zh * zh;
    NuBes b;
    b.j1 = zp * nu_bes_series(bc, P, y);
    b.j2 = (zp * zh) * nu_bes_series(bc, P + 1, y);
    b.iz2 = zh != 0.0 ? 1.0 / zh : 0.0;
    return b;
}
// eps_p J_p for moment p (descending calls p = P-1 .. 0), advancing the recurrence
__device__ __forceinline__ double nu_bes_w(NuBes& b, int p, double zh) {
    double j = fma((double)(p + 1) * b.iz2, b.j1, -b.j2);
    b.j2 = b.j1;
    b.j1 = j;
    if (p == 0) return zh != 0.0 ? j : 1.0;
    return 2.0 * j;
}
// acc + w i^p v (p uniform)
__device__ __forceinline__ double2 nu_bes_acc(double2 acc, double w, double2 v, int p) {
    switch (p & 3) {
        case 0: return make_double2(fma(w, v.x, acc.x), fma(w, v.y, acc.y));
        case 1: return make_double2(fma(-w, v.y, acc.x), fma(w, v.x, acc.y));
        case 2: return make_double2(fma(-w, v.x, acc.x), fma(-w, v.y, acc.y));
        default: return make_double2(fma(w, v.y, acc.x), fma(-w, v.x, acc.y));
    }
}
// z/2 = (pi/2) jc / n for an FFT output position holding trial offset jc
__device__ __forceinline__ double nu_zh(int64_t jc, int lnfft) {
    return ldexp((double)jc, -lnfft) * 1.5707963267948966192313216916398;
}
// T_p(u), p < 32, by the doubling ladder (T_2m = 2 T_m^2 - 1, T_2m+1 = 2 T_m T_m+1 - u) -- the MFMA spread's lanes
// each need one p
__device__ __forceinline__ double nu_cheb(double u, int p) {
    double a = 1.0, b = u;  // (T_m, T_m+1), m = 0
#pragma unroll
    for (int bit = 4; bit >= 0; --bit) {
        const double ab = fma(2.0 * a, b, -u);
        if ((p >> bit) & 1) {
            b = fma(2.0 * b, b, -1.0);
            a = ab;
        } else {
            a = fma(2.0 * a, a, -1.0);
            b = ab;
        }
    }
    return a;
}

// T_p(x) = x^(p & 1) Q_p(x^2) with Q_p's monomial coefficients (exact integers), p < 16: the MFMA spread's lane
// evaluates its own T_p by a degree-7 Horner in y = x^2 (9 fp64 operations; the doubling ladder nu_cheb took ~30
// plus selects). |x| <= 1, so the rounding is at most ~sum |c| ulp: 2e-11 absolute for T_15, whose weight in the
// combine is |2 J_15(pi/2)| < 3e-14 (nu_bes); ~1e-15 for the p <= 4 moments that carry the sums.
__constant__ double kNuChebMono[16][8] = {
    {1.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0},
    {1.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0},
    {-1.0, 2.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0},
    {-3.0, 4.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0},
    {1.0, -8.0, 8.0, 0.0, 0.0, 0.0, 0.0, 0.0},
    {5.0, -20.0, 16.0, 0.0, 0.0, 0.0, 0.0, 0.0},
    {-1.0, 18.0, -48.0, 32.0, 0.0, 0.0, 0.0, 0.0},
    {-7.0, 56.0, -112.0, 64.0, 0.0, 0.0, 0.0, 0.0},
    {1.0, -32.0, 160.0, -256.0, 128.0, 0.0, 0.0, 0.0},
    {9.0, -120.0, 432.0, -576.0, 256.0, 0.0, 0.0, 0.0},
    {-1.0, 50.0, -400.0, 1120.0, -1280.0, 512.0, 0.0, 0.0},
    {-11.0, 220.0, -1232.0, 2816.0, -2816.0, 1024.0, 0.0, 0.0},
    {1.0, -72.0, 840.0, -3584.0, 6912.0, -6144.0, 2048.0, 0.0},
    {13.0, -364.0, 2912.0, -9984.0, 16640.0, -13312.0, 4096.0, 0.0},
    {-1.0, 98.0, -1568.0, 9408.0, -26880.0, 39424.0, -28672.0, 8192.0},
    {-15.0, 560.0, -6048.0, 28800.0, -70400.0, 92160.0, -61440.0, 16384.0}};

__device__ __forceinline__ int64_t nu_readlane64(int64_t v, int lane) {
    const int lo = __builtin_amdgcn_readlane((int)(uint32_t)(uint64_t)v, lane);
    const int hi = __builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), lane);
    return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint64_t)(uint32_t)lo);
}

// sortedness of dt (the spread's cells only grow along a chunk)
__global__ __launch_bounds__(256) void k_nu_sorted(const double* __restrict__ tt, double t0, int64_t n, int* __restrict__ bad) {
    int b = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i + 1 < n; i += (int64_t)gridDim.x * blockDim.x)
        b |= !((tt[i] - t0) <= (tt[i + 1] - t0));
    if (__any(b) && (threadIdx.x & 63) == 0) atomicOr(bad, 1);
}

// Moments of harmonics k0 .. k0+G-1 for rows [0, nrow) of the pass (c2row points at the pass's first row).
// Lane l: photon q = l >> 4 of the K-group, A row (moment) p = l & 15, B column col = l & 15 = 2 row + (re/im).
template <int G, bool TWOD>
__global__ __launch_bounds__(256) void k_nu_spread(const double* __restrict__ tt, double t0, int64_t n, int64_t nchunk, double s1,
                                                   double fch, double fcl, const double* __restrict__ c2row, int nrow,
                                                   int k0, int P, const NuPass* __restrict__ ps,
                                                   const double2* __restrict__ tab, double* __restrict__ U,
                                                   int64_t* __restrict__ ctab, const int* __restrict__ bad) {
    if (*bad) return;  // photons out of order or a cached plan that no longer holds (k_ap_final)
    // the cis table in LDS (read twice per photon and K-group: an L2 round trip each, waited for at once), filled
    // before any wave leaves
    __shared__ double2 stab[1024];
    for (int e = threadIdx.x; e < 1024; e += 256) stab[e] = tab[e];
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int64_t c = (int64_t)blockIdx.x * kNuWaves + (threadIdx.x >> 6);
    if (c >= nchunk) return;  // wave-uniform
    const int q = lane >> 4, col = lane & 15, prow = col >> 1, reim = col & 1, pp = lane & 15;
    const bool rowok = prow < nrow, pok = pp < P;
    const double c2 = (TWOD && rowok) ? c2row[prow] : 0.0;
    double cm[8];  // this lane's T_pp in monomials of (2e)^2 (kNuChebMono); rows p >= P of D are never stored
#pragma unroll
    for (int m = 0; m < 8; ++m) cm[m] = kNuChebMono[pp][m];
    const bool odd = pp & 1;
    (void)pok;
    const int64_t i0 = c * kNuCW, i1 = i0 + kNuCW < n ? i0 + kNuCW : n;
    const int64_t SL = 2 * (int64_t)P * nrow;  // doubles per slot: [p][row][re, im]
    nu_f64x4 acc[G];
    int gcur[G];  // cells fit 32 bits (nu_plan: |G| + n < 2^31)
    {
        const double u1 = (tt[i0] - t0) * s1;
#pragma unroll
        for (int kk = 0; kk < G; ++kk) {
            acc[kk] = nu_f64x4{0.0, 0.0, 0.0, 0.0};
            gcur[kk] = (int)rint((double)(k0 + kk) * u1);
            if (lane == 0) ctab[(kk * nchunk + c) * 2] = gcur[kk];  // the chunk's first cell
        }
    }
    auto flush = [&](int kk) {
        const int64_t slot = (int64_t)gcur[kk] - ps->gmin[kk] + c;
        double* const base = U + ps->ubase[kk] + slot * SL;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int p = q + 4 * r;  // D row of register r
            if (p < P && rowok) base[(p * nrow + prow) * 2 + reim] = acc[kk][r];
        }
        acc[kk] = nu_f64x4{0.0, 0.0, 0.0, 0.0};
    };
    // cells the chunk's photons skip (observation gaps): their slots lie inside the chunk's cell range, which the
    // merge reads, so they are written as zeros
    auto zero_gap = [&](int kk, int64_t from, int64_t to) {
        for (int64_t cell = from + 1; cell < to; ++cell) {
            double* const base = U + ps->ubase[kk] + (cell - ps->gmin[kk] + c) * SL;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int p = q + 4 * r;
                if (p < P && rowok) base[(p * nrow + prow) * 2 + reim] = 0.0;
            }
        }
    };
    // past the end: the last photon's time (same cell, zero weight); the next tile's times are loaded (raw) during
    // the current one
    double tn = tt[i0 + lane < n ? i0 + lane : n - 1];
    for (int64_t ib = i0; ib < i1; ib += 64) {
        const double dv = tn - t0;
        const int64_t il = ib + 64 + lane;
        tn = tt[il < n ? il : n - 1];
#pragma unroll 1
        for (int g = 0; g < 16; ++g) {
            if (ib + 4 * g >= i1) break;  // wave-uniform
            const double d = __shfl(dv, 4 * g + q, 64);
            const bool valid = ib + 4 * g + q < i1;
            // premultiplier phase (cycles): frac(fc d) + frac(c2 d^2), in double-double, then harmonic k0
            double phi = nu_frac_prod(fch, fcl, d);
            if (TWOD) {
                const double d2 = d * d, d2e = fma(d, d, -d2);
                phi += nu_frac_c2(c2, d2, d2e);
            }
            phi -= rint(phi);
            const double2 c1 = nu_cis(stab, phi);
            double2 ck = c1;
            if (k0 > 1) ck = nu_cis(stab, nu_frac_k((double)k0, phi));
            // this lane's B column as the real part of cl: c for re lanes, (-i) c for im lanes; zero for a photon
            // past the chunk's end or a row beyond the pass (products by c1 keep it zero, and A needs no mask:
            // its rows p >= P are never stored). One select per K-group instead of per harmonic.
            double2 cl = reim ? make_double2(ck.y, -ck.x) : ck;
            if (!(valid && rowok)) cl = make_double2(0.0, 0.0);
            const double u1 = d * s1;
#pragma unroll
            for (int kk = 0; kk < G; ++kk) {
                if (kk > 0) cl = nu_cmul(cl, c1);
                const double uk = (double)(k0 + kk) * u1;
                const double gk = rint(uk);
                const double e = uk - gk;
                const double x = 2.0 * e, y = x * x;  // T_p(2e) (nu_bes) by Horner in y
                double a = cm[7];
#pragma unroll
                for (int m = 6; m >= 0; --m) a = fma(a, y, cm[m]);
                if (odd) a *= x;
                const double b = cl.x;
                const int G32 = (int)gk;  // 32-bit cells and read-lanes
                const int g0 = __builtin_amdgcn_readlane(G32, 0), g3 = __builtin_amdgcn_readlane(G32, 48);
                if (g0 == gcur[kk] && g3 == gcur[kk]) {
                    acc[kk] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[kk], 0, 0, 0);
                } else {
                    // the K-group crosses cells: photons of the current cell first, then each later cell in turn
                    const int g1 = __builtin_amdgcn_readlane(G32, 16), g2 = __builtin_amdgcn_readlane(G32, 32);
                    for (;;) {
                        if (g0 <= gcur[kk]) {
                            const double am = (G32 == gcur[kk]) ? a : 0.0;
                            acc[kk] = __builtin_amdgcn_mfma_f64_16x16x4f64(am, b, acc[kk], 0, 0, 0);
                        }
                        if (g3 == gcur[kk]) break;
                        flush(kk);
                        const int nx = g0 > gcur[kk] ? g0 : g1 > gcur[kk] ? g1 : g2 > gcur[kk] ? g2 : g3;
                        if (nx > gcur[kk] + 1) zero_gap(kk, gcur[kk], nx);
                        gcur[kk] = nx;
                    }
                }
            }
        }
    }
#pragma unroll
    for (int kk = 0; kk < G; ++kk) {
        flush(kk);
        if (lane == 0) ctab[(kk * nchunk + c) * 2 + 1] = gcur[kk];  // the chunk's last cell
    }
}

// ---- cell-gather spread (a pass of <= kNuGatherRows rows, one harmonic): one lane per wrapped cell ----
// start[G - gmin] = the first photon whose cell (rint(k (dt s1)), the spread's arithmetic) is >= G, for the
// unwrapped cells G in [gmin, gmax + 1]; photons are time-sorted, so cell G holds photons [start[G], start[G+1]).
// Up to kNuCellK harmonics k0 .. k0+nk-1 per launch (one read of the photon times): harmonic k0 + j writes its
// table at start + off[j] for cells gmin[j] .. gmin[j] + span[j] - 1.
constexpr int kNuCellK = 4;
struct NuCellArgs {
    int64_t gmin[kNuCellK], span[kNuCellK], off[kNuCellK];
};
// The cell gather's plans take the photon order from here too (no k_nu_sorted pass): a pair out of order sets *bad
// (the search then takes the default path) and the writes stay inside the tables, which the host zeroes first, so
// every entry is a photon index in [0, n] whatever the order.
// Photon pairs (one 16-byte load when t is 16-byte aligned, VEC), kNuCellU pairs per thread and sweep with their
// loads issued together, over at most 2048 blocks: the predecessor of a pair's first photon is the previous lane's
// second one (a shuffle; lane 0 loads it). One 8-byte load per iteration ran at ~2 TB/s, and one pair per thread
// over a grid covering the photons (19.5k short blocks at config 3) was bound by the workgroup dispatch: 35-43 us per
// 80 MB either way.
// A wave that finds a pair out of order among its photons of a sweep writes nothing for them: on sorted photons
// every wave is clean and the tables complete; on unsorted ones the search is discarded anyway (*bad), and a
// skipped wave cannot run a long write loop for a backward-then-forward jump (the gathers never read the tables).
constexpr int kNuCellU = 4;
template <bool VEC>
__global__ __launch_bounds__(256) void k_nu_cellstart(const double* __restrict__ tt, double t0, int64_t n, double s1,
                                                      int k0, int nk, NuCellArgs a, int64_t* __restrict__ start,
                                                      int* __restrict__ bad, int mode) {
    if (*bad) return;  // a cached plan that no longer holds (k_ap_final): no table is written
    const int64_t npair = (n + 1) / 2, stride = (int64_t)gridDim.x * blockDim.x;
    const int lane = threadIdx.x & 63;
    int b = 0;
    // block-uniform loop bound (the barrier of __syncthreads_or below)
    for (int64_t p0b = (int64_t)blockIdx.x * blockDim.x; p0b < npair; p0b += kNuCellU * stride) {
        double x0[kNuCellU], x1[kNuCellU], xl[kNuCellU];
#pragma unroll
        for (int q = 0; q < kNuCellU; ++q) {
            const int64_t pr = p0b + threadIdx.x + q * stride, i0 = 2 * pr;
            if (VEC && i0 + 1 < n) {
                const double2 v = reinterpret_cast<const double2*>(tt)[pr];
                x0[q] = v.x;
                x1[q] = v.y;
            } else {
                x0[q] = tt[i0 < n ? i0 : n - 1];
                x1[q] = tt[i0 + 1 < n ? i0 + 1 : n - 1];
            }
            xl[q] = 0.0;
            if (lane == 0) xl[q] = tt[i0 > 0 && i0 - 1 < n ? i0 - 1 : 0];  // the wave's first predecessor
        }
#pragma unroll
        for (int q = 0; q < kNuCellU; ++q) {
            const int64_t i0 = 2 * (p0b + threadIdx.x + q * stride);
            double xp = __shfl_up(x1[q], 1, 64);
            if (lane == 0) xp = xl[q];
            const double d0 = x0[q] - t0, d1 = x1[q] - t0;
            const double dp0 = i0 == 0 ? d0 : xp - t0;
            const bool v0 = i0 < n, v1 = i0 + 1 < n;
            const int ooo = (v0 && !(dp0 <= d0)) || (v1 && !(d0 <= d1));
            b |= ooo;
            if (mode == 1) continue;  // A/B probe: loads and order check only (the search is then discarded)
            // a wave that holds a pair out of order writes nothing for its photons (a vote, no block barrier: the
            // barrier cost a quarter of the pass; mode 2, A/B: the lanes' own pairs only)
            if (mode == 2 ? ooo : __any(ooo)) continue;
            // per harmonic the cells of the predecessor and of the pair's two photons, each formed once (the second
            // photon's range starts at the first one's cell); cells fit 32 bits (nu_plan checks |G| + n < 2^31): one
            // v_cvt_i32_f64 each, and 32-bit bounds
            const double up = dp0 * s1, u0 = d0 * s1, u1 = d1 * s1;
#pragma unroll
            for (int j = 0; j < kNuCellK; ++j) {
                if (j >= nk) break;
                const double kd = (double)(k0 + j);
                const int gm = (int)a.gmin[j], gl = (int)(a.gmin[j] + a.span[j] - 1);
                int64_t* st = start + a.off[j];
                const int gA = i0 == 0 ? gm - 1 : (int)rint(kd * up);
                const int gB = (int)rint(kd * u0);
                if (v0) {  // photon i0 starts the cells (gA, gB]
                    const int lo = gA + 1 > gm ? gA + 1 : gm, hi = gB < gl ? gB : gl;
                    for (int G = lo; G <= hi; ++G) st[G - gm] = i0;
                    if (i0 == n - 1) st[a.span[j]] = n;
                }
                if (v1) {  // photon i0 + 1 the cells (gB, gC]
                    const int gC = (int)rint(kd * u1);
                    const int lo = gB + 1 > gm ? gB + 1 : gm, hi = gC < gl ? gC : gl;
                    for (int G = lo; G <= hi; ++G) st[G - gm] = i0 + 1;
                    if (i0 + 1 == n - 1) st[a.span[j]] = n;
                }
            }
        }
    }
    if (__any(b) && lane == 0) atomicOr(bad, 1);
    if (mode == 1 && blockIdx.x == 0 && threadIdx.x == 0) atomicOr(bad, 1);  // the probe's tables are not written
}

// L lanes per wrapped cell g sum, over its unwrapped cells G = g (mod n) and their photons in time order (lane s
// takes the cell's photons s, s + L, ...), the moments c_r T_p(2e) of rows r < nrow: b_p,r[g] = sum c_{i,r} T_p(2e_i) with
// c = e^{2 pi i k (fc dt + c2_r dt^2)}, e = k dt s1 - G, in registers; an xor butterfly over the L lanes (a fixed
// order: deterministic) completes the sums and lane s writes the moments p = s (mod L) to W[p * nrow + r][g].
// fp64 VALU throughout: per photon, row and harmonic one premultiplier phase and cis, then 3 operations per moment.
// L > 1 spreads a cell's photons over several lanes when cells are dense (many photons per cell, few cells).
// One launch serves up to kNuGatherSet harmonics (NuGatherSet: block ranges, cells, lanes per cell and W plane of
// each): the harmonics of a search share the launch's waves, so its last round of blocks is not one harmonic's tail
// (config 3 ran two launches of 1.7 and 3.4 rounds of resident waves).
constexpr int kNuGatherRows = 2;
constexpr int kNuGatherSet = 8;
struct NuGatherSet {
    int nk;
    int k[kNuGatherSet], lanes_log2[kNuGatherSet];
    int64_t blk0[kNuGatherSet + 1];                       // first block of each harmonic, then the total
    int64_t gmin[kNuGatherSet], gmax[kNuGatherSet], gbase[kNuGatherSet], gcount[kNuGatherSet];
    int64_t soff[kNuGatherSet], woff[kNuGatherSet];       // the harmonic's start table and W planes
};
template <int R, bool TWOD, int PP>  // PP >= P moments accumulated unconditionally (no per-moment selects)
__global__ __launch_bounds__(256) void k_nu_gather(const double* __restrict__ tt, double t0,
                                                   const int64_t* __restrict__ startb, int64_t nfft, double s1,
                                                   double fch, double fcl, const double* __restrict__ c2row, int nrow,
                                                   int P, const NuGatherSet S, const int* __restrict__ bad,
                                                   const double2* __restrict__ tab, double2* __restrict__ Wb) {
    // photons out of order (the cell starts found it): the start tables are not filled (nothing zeroes them), so no
    // lane may read them; the search's results are discarded and the default path runs
    if (*bad) return;
    __shared__ double2 stab[2048];  // the cis table (nu_cis2), read per photon: LDS, not L2 latency
    for (int e = threadIdx.x; e < 2048; e += 256) stab[e] = tab[e];
    __syncthreads();
    int j = 0;  // this block's harmonic (block-uniform)
    while (j + 1 < S.nk && (int64_t)blockIdx.x >= S.blk0[j + 1]) ++j;
    const int ll = S.lanes_log2[j], L = 1 << ll;
    const int64_t tid = ((int64_t)blockIdx.x - S.blk0[j]) * 256 + threadIdx.x;
    const int64_t idx = tid >> ll;
    const int sub = (int)(tid & (L - 1));
    if (idx >= S.gcount[j]) return;  // whole L-groups leave together (L divides 64); no barrier below
    const int64_t gmin = S.gmin[j], gmax = S.gmax[j];
    const int64_t* __restrict__ start = startb + S.soff[j];
    double2* __restrict__ W = Wb + S.woff[j];
    const int64_t g = (S.gbase[j] + idx) & (nfft - 1);  // the FFT's occupied rows only (nu_occupied)
    double ar[R][PP], ai[R][PP];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int p = 0; p < PP; ++p) ar[r][p] = ai[r][p] = 0.0;
    double c2[R];
#pragma unroll
    for (int r = 0; r < R; ++r) c2[r] = (TWOD && r < nrow) ? c2row[r] : 0.0;
    const double kd = (double)S.k[j];
    // the photon times are prefetched raw and unconditionally (indices clamped into the cell, whose stand-ins are
    // never weighted): a load whose value entered a select or a subtraction at its issue would be waited for there;
    // the next cell's photon range is loaded during the current cell
    int64_t G = gmin + (((g - gmin) % nfft) + nfft) % nfft;
    int64_t ns0 = 0, ns1 = 0;
    if (G <= gmax) {
        ns0 = start[G - gmin];
        ns1 = start[G - gmin + 1];
    }
    for (; G <= gmax; G += nfft) {
        const int64_t i0 = ns0, i1 = ns1;
        if (G + nfft <= gmax) {
            ns0 = start[G + nfft - gmin];
            ns1 = start[G + nfft - gmin + 1];
        }
        if (i1 <= i0) continue;  // an empty cell (no clamped load below i0)
        const double Gd = (double)G;
        // two photons per iteration (independent chains for the VALU; each one's terms still added in photon
        // order), their times prefetched two iterations ahead (HBM latency is several iterations of one wave)
        const int64_t il = i1 - 1;
        double dn[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) dn[q] = tt[i0 + sub + q * L < il ? i0 + sub + q * L : il];
        for (int64_t i = i0 + sub; i < i1; i += 2 * L) {
            const bool hb = i + L < i1;
            const double da = dn[0] - t0, db = (hb ? dn[1] : dn[0]) - t0;  // (no second photon: a stand-in, weight 0)
            dn[0] = dn[2];
            dn[1] = dn[3];
            dn[2] = tt[i + 4 * L < il ? i + 4 * L : il];
            dn[3] = tt[i + 5 * L < il ? i + 5 * L : il];
            const double ea = kd * (da * s1) - Gd, eb = kd * (db * s1) - Gd;
            const double p1a = nu_frac_prod(fch, fcl, da), p1b = nu_frac_prod(fch, fcl, db);
            double d2a = 0.0, d2ea = 0.0, d2b = 0.0, d2eb = 0.0;
            if (TWOD) {
                d2a = da * da;
                d2ea = fma(da, da, -d2a);
                d2b = db * db;
                d2eb = fma(db, db, -d2b);
            }
#pragma unroll
            for (int r = 0; r < R; ++r) {
                if (r < nrow) {
                    double phia = p1a, phib = p1b;
                    if (TWOD) {
                        phia += nu_frac_c2(c2[r], d2a, d2ea);
                        phib += nu_frac_c2(c2[r], d2b, d2eb);
                    }
                    phia -= rint(phia);
                    phib -= rint(phib);
                    const double2 ca = nu_cis2(stab, nu_frac_k(kd, phia));
                    double2 cb = nu_cis2(stab, nu_frac_k(kd, phib));
                    if (!hb) cb = make_double2(0.0, 0.0);
                    // Chebyshev moments T_p(2e): T_p+1 = 4e T_p - T_p-1 (nu_bes)
                    const double ua = 4.0 * ea, ub = 4.0 * eb;
                    double ta0 = 1.0, ta1 = 2.0 * ea, tb0 = 1.0, tb1 = 2.0 * eb;
#pragma unroll
                    for (int p = 0; p < PP; ++p) {
                        ar[r][p] = fma(ca.x, ta0, ar[r][p]);
                        ai[r][p] = fma(ca.y, ta0, ai[r][p]);
                        ar[r][p] = fma(cb.x, tb0, ar[r][p]);
                        ai[r][p] = fma(cb.y, tb0, ai[r][p]);
                        const double ta2 = fma(ua, ta1, -ta0), tb2 = fma(ub, tb1, -tb0);
                        ta0 = ta1;
                        ta1 = ta2;
                        tb0 = tb1;
                        tb1 = tb2;
                    }
                }
            }
        }
    }
    for (int o = L / 2; o > 0; o >>= 1)  // block-uniform L
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int p = 0; p < PP; ++p)
                if (p < P) {  // uniform
                    ar[r][p] += __shfl_xor(ar[r][p], o);
                    ai[r][p] += __shfl_xor(ai[r][p], o);
                }
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int p = 0; p < PP; ++p)
            if (r < nrow && p < P && (p & (L - 1)) == sub)
                W[((int64_t)p * nrow + r) * nfft + g] = make_double2(ar[r][p], ai[r][p]);
}

// slots -> W[beta][g] (beta = p * nrow + row, complex), for the wrapped cells g of one block
__global__ __launch_bounds__(256) void k_nu_merge(const double* __restrict__ U, int64_t SL,
                                                  const int64_t* __restrict__ ctab, int64_t nchunk, int64_t gmin,
                                                  int64_t gmax, int64_t nfft, int64_t gbase, int64_t gcount,
                                                  double2* __restrict__ W, const int* __restrict__ bad) {
    if (*bad) return;  // the spread did not run (k_nu_spread): its slots and cell table are not written
    __shared__ int64_t rs[kNuMergeG][kNuMaxWrap];
    __shared__ int rc[kNuMergeG][kNuMaxWrap];
    __shared__ int nr[kNuMergeG];
    extern __shared__ double nu_acc[];  // [kNuMergeG][SL]
    const int64_t i0 = (int64_t)blockIdx.x * kNuMergeG;  // cells gbase + i (mod n), i < gcount: the occupied rows
    const int tid = threadIdx.x;
    if (tid < kNuMergeG) {
        const int64_t g = (gbase + i0 + tid) & (nfft - 1);
        int cnt = 0;
        if (i0 + tid < gcount) {
            int64_t Gu = gmin + (((g - gmin) % nfft) + nfft) % nfft;  // smallest unwrapped cell >= gmin, = g mod n
            for (; Gu <= gmax && cnt < kNuMaxWrap; Gu += nfft) {
                int64_t lo = 0, hi = nchunk;  // first chunk whose last cell is >= Gu
                while (lo < hi) {
                    const int64_t mid = (lo + hi) >> 1;
                    if (ctab[2 * mid + 1] < Gu)
                        lo = mid + 1;
                    else
                        hi = mid;
                }
                int len = 0;
                while (lo + len < nchunk && ctab[2 * (lo + len)] <= Gu) ++len;
                if (len > 0) {
                    rs[tid][cnt] = Gu - gmin + lo;
                    rc[tid][cnt] = len;
                    ++cnt;
                }
            }
        }
        nr[tid] = cnt;
    }
    __syncthreads();
    for (int64_t idx = tid; idx < kNuMergeG * SL; idx += 256) {
        const int t = (int)(idx / SL);
        const int64_t e = idx - t * SL;
        double v = 0.0;
        for (int r = 0; r < nr[t]; ++r)
            for (int k = 0; k < rc[t][r]; ++k) v += U[(rs[t][r] + k) * SL + e];
        nu_acc[idx] = v;
    }
    __syncthreads();
    const int64_t B = SL / 2;
    for (int64_t idx = tid; idx < kNuMergeG * B; idx += 256) {
        const int t = (int)(idx % kNuMergeG);
        const int64_t beta = idx / kNuMergeG;
        if (i0 + t < gcount) {
            const int64_t g = (gbase + i0 + t) & (nfft - 1);
            W[beta * nfft + g] = make_double2(nu_acc[t * SL + 2 * beta], nu_acc[t * SL + 2 * beta + 1]);
        }
    }
}

// Power and error bound of one trial from its harmonic sums: CS[k * nbt + t] for k < m, except that with lastv the
// last harmonic's sum is the register value `last` (the fused row pass, k_nu_rows_combine8). The same operations
// in the same order either way, so the fused and separate finalize give identical powers and flags.
__device__ __forceinline__ void nu_power(const double2* __restrict__ CS, int64_t nbt, int64_t t, int m, int stat,
                                         double nph, double E, bool lastv, double2 last, double* pout,
                                         double* eout) {
    const double w = 2.0 / nph;
    auto zk = [&](int k, double* amag) {
        const double2 a = (lastv && k == m - 1) ? last : CS[(int64_t)k * nbt + t];
        const double z = a.x * a.x + a.y * a.y;
        *amag = sqrt(z);
        return z;
    };
    double p, err;
    if (stat == CRIMP_STAT_Z2) {
        double zsum = 0.0, eb = 0.0, am;
        for (int k = 0; k < m; ++k) {
            zsum += zk(k, &am);
            eb += 2.0 * am * E + E * E;
        }
        p = zsum * w;
        err = eb * w;
    } else {
        double cum = 0.0, best = -INFINITY, ebest = 0.0, eacc = 0.0, am;
        for (int k = 0; k < m; ++k) {
            const double z = zk(k, &am);
            cum += z * w;
            eacc += (2.0 * am * E + E * E) * w;
            const double v = cum - 4.0 * (double)k;
            if (v > best) {
                best = v;
                ebest = eacc;
            }
        }
        p = best;
        err = ebest;
        cum = 0.0;
        eacc = 0.0;
        for (int k = 0; k < m; ++k) {
            const double z = zk(k, &am);
            cum += z * w;
            eacc += (2.0 * am * E + E * E) * w;
            if (cum - 4.0 * (double)k + eacc >= best - ebest) err = fmax(err, eacc);
        }
    }
    *pout = p;
    *eout = err;
}
// E = N (x^P invfact + kNuRho) at trial offset jc (nu_trunc)
__device__ __forceinline__ double nu_err_bound(int64_t jc, int64_t nfft, int P, double invfact, double nph) {
    const double x = 3.14159265358979323846 * fabs((double)jc) / (double)nfft;
    double xp = 1.0;
    for (int p = 0; p < P; ++p) xp *= x;
    return nph * (xp * invfact + kNuRho);
}

// ---- FFT: DFTs of radix 2..16 in registers (X_k = sum_j x_j w_R^{+jk}, natural order) ----
__device__ __forceinline__ void nu_dft2(double2* v) {
    const double2 a = v[0], b = v[1];
    v[0] = nu_add(a, b);
    v[1] = nu_sub(a, b);
}
__device__ __forceinline__ void nu_dft4(double2& a0, double2& a1, double2& a2, double2& a3) {
    const double2 t0 = nu_add(a0, a2), t1 = nu_sub(a0, a2), t2 = nu_add(a1, a3), t3 = nu_muli(nu_sub(a1, a3));
    a0 = nu_add(t0, t2);
    a2 = nu_sub(t0, t2);
    a1 = nu_add(t1, t3);
    a3 = nu_sub(t1, t3);
}
__device__ __forceinline__ void nu_dft4v(double2* v) { nu_dft4(v[0], v[1], v[2], v[3]); }
__device__ __forceinline__ void nu_dft8(double2* v) {
    double2 e[4] = {v[0], v[2], v[4], v[6]}, o[4] = {v[1], v[3], v[5], v[7]};
    nu_dft4v(e);
    nu_dft4v(o);
    const double s = 0.70710678118654752440084436210485;
    const double2 w[4] = {make_double2(1.0, 0.0), make_double2(s, s), make_double2(0.0, 1.0), make_double2(-s, s)};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const double2 t = k == 0 ? o[0] : k == 2 ? nu_muli(o[2]) : nu_cmul(o[k], w[k]);
        v[k] = nu_add(e[k], t);
        v[k + 4] = nu_sub(e[k], t);
    }
}
__device__ __forceinline__ void nu_dft16(double2* v) {
    double2 e[8], o[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        e[k] = v[2 * k];
        o[k] = v[2 * k + 1];
    }
    nu_dft8(e);
    nu_dft8(o);
    const double c1 = 0.92387953251128675612818318939679, s1 = 0.38268343236508977172845998403040,
                 r2 = 0.70710678118654752440084436210485;
    const double2 w[8] = {make_double2(1.0, 0.0), make_double2(c1, s1), make_double2(r2, r2), make_double2(s1, c1),
                          make_double2(0.0, 1.0), make_double2(-s1, c1), make_double2(-r2, r2), make_double2(-c1, s1)};
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const double2 t = k == 0 ? o[0] : k == 4 ? nu_muli(o[4]) : nu_cmul(o[k], w[k]);
        v[k] = nu_add(e[k], t);
        v[k + 8] = nu_sub(e[k], t);
    }
}
template <int R>
__device__ __forceinline__ void nu_dft(double2* v) {
    if (R == 2) nu_dft2(v);
    else if (R == 4) nu_dft4v(v);
    else if (R == 8) nu_dft8(v);
    else nu_dft16(v);
}

// Twiddles of the in-LDS transforms (length <= 2^lt, lt = min(log2 n, 12)): w^m = e^{2 pi i m / 2^lt} as
// hi[m >> 6] * lo[m & 63], two 64-entry tables in LDS filled by fp64 sincospi at the kernel's start.
struct NuTile {
    double2 hi[64], lo[64];
};
__device__ __forceinline__ void nu_tile_init(NuTile* tw, int lt) {
    const int t = threadIdx.x;
    if (t < 128) {
        const int m = t < 64 ? t : (t - 64) << 6;
        double sv, cv;
        sincospi(ldexp((double)m, 1 - lt), &sv, &cv);  // 2 m / 2^lt
        if (t < 64)
            tw->lo[t] = make_double2(cv, sv);
        else
            tw->hi[t - 64] = make_double2(cv, sv);
    }
}
__device__ __forceinline__ double2 nu_tw_tile(const NuTile* tw, int m) { return nu_cmul(tw->hi[m >> 6], tw->lo[m & 63]); }

// v[r] *= w^r for r = 1 .. R-1: w^r as the product of w, w^2, w^4, w^8 over the bits of r (few live registers,
// product depth <= 3 after the squarings, instead of a chain of R - 2 products)
template <int R>
__device__ __forceinline__ void nu_twiddle(double2 w, double2* v) {
    double2 b[4];
    b[0] = w;
#pragma unroll
    for (int i = 1; i < 4; ++i)
        if ((1 << i) < R) b[i] = nu_cmul(b[i - 1], b[i - 1]);
#pragma unroll
    for (int r = 1; r < R; ++r) {
        double2 wr = make_double2(1.0, 0.0);
        bool first = true;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if (r & (1 << i)) {
                wr = first ? b[i] : nu_cmul(wr, b[i]);
                first = false;
            }
        v[r] = nu_cmul(v[r], wr);
    }
}

// One Stockham autosort stage of radix R over 2^lc transforms of length 2^ll held in LDS at s[a*sa + cc*sc]:
// butterfly (j, cc) reads x[j + r L/R], twiddles by w_{Ns R}^{(j mod Ns) r}, and writes
// y[(j / Ns) Ns R + (j mod Ns) + r Ns]. 16 / R butterflies per thread (a tile holds <= 16 elements per thread).
template <int R>
__device__ __forceinline__ void nu_stage(double2* s, int ll, int lc, int sa, int sc, int lns, const NuTile* tw,
                                         int lt) {
    constexpr int NB = 16 / R;
    constexpr int LR = R == 2 ? 1 : R == 4 ? 2 : R == 8 ? 3 : 4;
    const int L = 1 << ll, Ns = 1 << lns;
    const int nbt = (L >> LR) << lc;
    double2 v[NB][R];
#pragma unroll
    for (int k = 0; k < NB; ++k) {
        const int b = threadIdx.x + 256 * k;
        if (b < nbt) {
            const int cc = b & ((1 << lc) - 1), j = b >> lc;
#pragma unroll
            for (int r = 0; r < R; ++r) v[k][r] = s[(j + (r << (ll - LR))) * sa + cc * sc];
            if (lns > 0) {
                // w_{Ns R}^{(j mod Ns)} = w_{2^lt}^{(j mod Ns) 2^lt / (Ns R)}
                nu_twiddle<R>(nu_tw_tile(tw, (j & (Ns - 1)) << (lt - lns - LR)), v[k]);
            }
            nu_dft<R>(v[k]);
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < NB; ++k) {
        const int b = threadIdx.x + 256 * k;
        if (b < nbt) {
            const int cc = b & ((1 << lc) - 1), j = b >> lc;
            const int base = ((j >> lns) << (lns + LR)) + (j & (Ns - 1));
#pragma unroll
            for (int r = 0; r < R; ++r) s[(base + r * Ns) * sa + cc * sc] = v[k][r];
        }
    }
    __syncthreads();
}

// 2^lc transforms of length 2^ll in LDS (Stockham: natural order in, natural order out)
__device__ __forceinline__ void nu_fft_lds(double2* s, int ll, int lc, int sa, int sc, const NuTile* tw, int lt) {
    int lns = 0;
    while (lns < ll) {
        const int rem = ll - lns;
        if (rem >= 4) {
            nu_stage<16>(s, ll, lc, sa, sc, lns, tw, lt);
            lns += 4;
        } else if (rem == 3) {
            nu_stage<8>(s, ll, lc, sa, sc, lns, tw, lt);
            lns += 3;
        } else if (rem == 2) {
            nu_stage<4>(s, ll, lc, sa, sc, lns, tw, lt);
            lns += 2;
        } else {
            nu_stage<2>(s, ll, lc, sa, sc, lns, tw, lt);
            lns += 1;
        }
    }
}

// pass 1 of the four-step FFT: view each batch as [n1][n2]; DFT along a of 2^lc consecutive columns b, times
// w_n^{b k1}, stored at y[k1 n2 + b]
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void k_nu_fft_cols(const double2* __restrict__ X, double2* __restrict__ Y,
                                                     int lnfft, int ln1, int lc, NuTw T, int alo, int acnt) {
    extern __shared__ double2 nu_s[];
    __shared__ NuTile tw;
    const int lt = lnfft < 12 ? lnfft : 12;
    nu_tile_init(&tw, lt);
    const int ln2 = lnfft - ln1, c = 1 << lc, n1 = 1 << ln1;
    const int64_t nfft = int64_t(1) << lnfft;
    const int64_t b0 = (int64_t)blockIdx.x << lc;
    const double2* x = X + (int64_t)blockIdx.y * nfft;
    double2* y = Y + (int64_t)blockIdx.y * nfft;
    for (int e = threadIdx.x; e < (n1 << lc); e += 256) {  // rows a outside [alo, alo + acnt) (mod n1) hold no cell
        const int a = e >> lc, cc = e & (c - 1);
        nu_s[e] = ((a - alo) & (n1 - 1)) < acnt ? x[((int64_t)a << ln2) + b0 + cc] : make_double2(0.0, 0.0);
    }
    __syncthreads();
    nu_fft_lds(nu_s, ln1, lc, c, 1, &tw, lt);
    // times the inter-pass twiddles w_n^{b k1} (n1 c = 4096: 16 outputs per thread)
#pragma unroll
    for (int q = 0; q < kNuTile / 256; ++q) {
        const int e = threadIdx.x + 256 * q;
        if (e < (n1 << lc)) {
            const int k1 = e >> lc, cc = e & (c - 1);
            const int64_t b = b0 + cc;
            y[((int64_t)k1 << ln2) + b] = nu_cmul(nu_s[e], nu_tw(T, b * k1));
        }
    }
}

// k_nu_fft_cols for n1 = 256 (two radix-16 stages over 16 columns): stage 1 on the columns as loaded into registers
// (thread (j, cc): rows j + 16 r of column cc), one LDS exchange, stage 2's outputs (rows k1 = j + 16 r) twiddled and
// stored from registers: one LDS write and read instead of six. Persistent blocks walk the (batch, column block)
// groups with the next group's rows and twiddle bases loaded during the current one (the kernel is latency-bound at
// the two waves per SIMD its 64 KB of LDS allow). The inter-pass twiddle w_n^{b k1} = w_n^{b j} (w_n^{16 b})^r: two
// table values and products over the bits of r (a few ulp, as the tile twiddles).
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void k_nu_cols256(
    const double2* __restrict__ X, double2* __restrict__ Y, int lnfft, NuTw T, int alo, int acnt, int64_t ngroups) {
    extern __shared__ double2 nu_s[];  // [256 rows][16 columns]
    __shared__ NuTile tw;
    nu_tile_init(&tw, 12);
    const int ln2 = lnfft - 8;
    const int64_t nfft = int64_t(1) << lnfft;
    const int cc = threadIdx.x & 15, j = threadIdx.x >> 4;
    const int64_t cpb = int64_t(1) << (ln2 - 4);  // column blocks per batch
    // the prefetch keeps the twiddle bases as their two table factors each (loaded before the rows) and multiplies
    // them at use: a product at the fetch would wait for every load issued so far, the rows' included
    double2 nv[16], tf[4];
    auto fetch = [&](int64_t grp) {  // rows outside [alo, alo + acnt) (mod 256) hold no cell
        const int64_t b = ((grp % cpb) << 4) + cc;
        const double2* x = X + (grp / cpb) * nfft + b;
        const int64_t lm = (int64_t(1) << T.lbits) - 1, tb = (b * (int64_t)j) & T.mask, ts = (b << 4) & T.mask;
        tf[0] = T.hi[tb >> T.lbits];
        tf[1] = T.lo[tb & lm];
        tf[2] = T.hi[ts >> T.lbits];
        tf[3] = T.lo[ts & lm];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int a = j + 16 * r;
            nv[r] = ((a - alo) & 255) < acnt ? x[(int64_t)a << ln2] : make_double2(0.0, 0.0);
        }
    };
    int64_t grp = blockIdx.x;
    if (grp < ngroups) fetch(grp);
    __syncthreads();  // tw
    for (; grp < ngroups; grp += gridDim.x) {
        double2 v[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = nv[r];
        const double2 wb = nu_cmul(tf[0], tf[1]), ws = nu_cmul(tf[2], tf[3]);  // nu_tw's product
        const int64_t b = ((grp % cpb) << 4) + cc;
        double2* y = Y + (grp / cpb) * nfft + b;
        if (grp + gridDim.x < ngroups) fetch(grp + gridDim.x);
        nu_dft16(v);  // stage 1 (Ns = 1)
#pragma unroll
        for (int r = 0; r < 16; ++r) nu_s[((j << 4) + r) * 16 + cc] = v[r];
        __syncthreads();
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = nu_s[(j + 16 * r) * 16 + cc];
        __syncthreads();  // the next group's stage-1 writes reuse the tile
        nu_twiddle<16>(nu_tw_tile(&tw, j << 4), v);  // w_256^{j r}
        nu_dft16(v);                                 // stage 2 (Ns = 16): output rows k1 = j + 16 r
        v[0] = nu_cmul(v[0], wb);
        nu_twiddle<16>(ws, v);  // v[r] *= (w_n^{16 b})^r
#pragma unroll
        for (int r = 1; r < 16; ++r) v[r] = nu_cmul(v[r], wb);
#pragma unroll
        for (int r = 0; r < 16; ++r) y[(int64_t)(j + 16 * r) << ln2] = v[r];
    }
}

// k_nu_fft_cols for n1 = 512 (n = 512 n2; CRIMP_NUFFT_ROW2048=1): groups of 8 columns (NC = 1: 128 VGPRs, two blocks
// per CU; 16 columns at 248 VGPRs and one block measured 10 % slower), 512 threads (column cc = t & 7, j = t >> 3),
// three radix-8 Stockham stages over rows j + 64 q (8 elements per thread and column: rows as loaded, stage 3's outputs
// k1 = j + 64 q stored from registers), two exchanges through a [512 rows][8 columns] tile (conflict-free without a
// swizzle: 8 consecutive lanes hold 8 consecutive columns). Persistent blocks, the next group's occupied rows loaded
// during the current one; rows by buffer loads and stores (one offset register); the inter-pass twiddle
// w_n^{b k1} = w_n^{b j} (w_n^{64 b})^q as in k_nu_cols256.
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4))) void k_nu_cols512(
    const double2* __restrict__ X, double2* __restrict__ Y, int lnfft, NuTw T, int alo, int acnt, int64_t ngroups) {
    constexpr int NC = 1, C = 8;
    extern __shared__ double2 nu_s[];  // [512 rows][C columns]
    __shared__ NuTile tw;
    nu_tile_init(&tw, 9);
    const int ln2 = lnfft - 9;
    const int64_t nfft = int64_t(1) << lnfft;
    const int cc = threadIdx.x & 7, j = threadIdx.x >> 3;
    const int64_t cpb = int64_t(1) << (ln2 - 3);  // column groups per batch
    double2 nv[NC][8], tf[NC][4];
    const int voff = ((j << ln2) + cc) * 16;  // row offsets 64 q n2 16 B and column offsets 8 c 16 B: scalar
    auto fetch = [&](int64_t grp) {  // rows outside [alo, alo + acnt) (mod 512) hold no cell
        const int64_t b0 = (grp % cpb) * C;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(X + (grp / cpb) * nfft + b0), (short)0, (int)(16 << lnfft), 0x00020000);
        const int64_t lm = (int64_t(1) << T.lbits) - 1;
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            const int64_t b = b0 + cc + 8 * c, tb = (b * (int64_t)j) & T.mask, ts = (b << 6) & T.mask;
            tf[c][0] = T.hi[tb >> T.lbits];
            tf[c][1] = T.lo[tb & lm];
            tf[c][2] = T.hi[ts >> T.lbits];
            tf[c][3] = T.lo[ts & lm];
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const bool occ = ((j + 64 * q - alo) & 511) < acnt;
#pragma unroll
            for (int c = 0; c < NC; ++c)
                nv[c][q] = occ ? __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(
                                                                 rs, voff, ((64 * q << ln2) + 8 * c) * 16, 0))
                               : make_double2(0.0, 0.0);
        }
    };
    int64_t grp = blockIdx.x;
    if (grp < ngroups) fetch(grp);
    const int m2 = (j & 7) << 3;  // stage-2 twiddle w_64^{(j & 7) q} in units of w_512; stage 3: w_512^{j q}
    const int z2 = ((j >> 3) << 6) + (j & 7);
    __syncthreads();  // tw
    typedef unsigned int nu_u4 __attribute__((ext_vector_type(4)));
    for (; grp < ngroups; grp += gridDim.x) {
        double2 v[NC][8], wb[NC], ws[NC];
#pragma unroll
        for (int c = 0; c < NC; ++c) {
#pragma unroll
            for (int q = 0; q < 8; ++q) v[c][q] = nv[c][q];
            wb[c] = nu_cmul(tf[c][0], tf[c][1]);
            ws[c] = nu_cmul(tf[c][2], tf[c][3]);
        }
        const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(Y + (grp / cpb) * nfft + (grp % cpb) * C), (short)0, (int)(16 << lnfft), 0x00020000);
        if (grp + gridDim.x < ngroups) fetch(grp + gridDim.x);
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            nu_dft8(v[c]);  // stage 1 (Ns = 1): row 8 j + q
#pragma unroll
            for (int q = 0; q < 8; ++q) nu_s[((j << 3) + q) * C + cc + 8 * c] = v[c][q];
        }
        __syncthreads();
#pragma unroll
        for (int c = 0; c < NC; ++c) {
#pragma unroll
            for (int q = 0; q < 8; ++q) v[c][q] = nu_s[(j + 64 * q) * C + cc + 8 * c];
        }
        __syncthreads();  // the stage-2 writes reuse the tile
        const double2 t2 = nu_tw_tile(&tw, m2);
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            nu_twiddle<8>(t2, v[c]);
            nu_dft8(v[c]);  // stage 2 (Ns = 8): row z2 + 8 q
#pragma unroll
            for (int q = 0; q < 8; ++q) nu_s[(z2 + 8 * q) * C + cc + 8 * c] = v[c][q];
        }
        __syncthreads();
#pragma unroll
        for (int c = 0; c < NC; ++c) {
#pragma unroll
            for (int q = 0; q < 8; ++q) v[c][q] = nu_s[(j + 64 * q) * C + cc + 8 * c];
        }
        __syncthreads();  // the next group's stage-1 writes reuse the tile
        const double2 t3 = nu_tw_tile(&tw, j);
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            nu_twiddle<8>(t3, v[c]);
            nu_dft8(v[c]);  // stage 3 (Ns = 64): output row k1 = j + 64 q
            v[c][0] = nu_cmul(v[c][0], wb[c]);
            nu_twiddle<8>(ws[c], v[c]);  // v[q] *= (w_n^{64 b})^q
#pragma unroll
            for (int q = 1; q < 8; ++q) v[c][q] = nu_cmul(v[c][q], wb[c]);
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) {
#pragma unroll
            for (int c = 0; c < NC; ++c)
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(nu_u4, v[c][q]), ry, voff,
                                                       ((64 * q << ln2) + 8 * c) * 16, 0);
        }
    }
}

// pass 2 (or the only pass): DFT of 2^lr contiguous rows of length 2^ll each, in place
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void k_nu_fft_rows(double2* __restrict__ X, int ll, int lr, int lnfft) {
    extern __shared__ double2 nu_s[];
    __shared__ NuTile tw;
    const int lt = lnfft < 12 ? lnfft : 12;
    nu_tile_init(&tw, lt);
    const int L = 1 << ll;
    double2* x = X + ((int64_t)blockIdx.x << (ll + lr));
    for (int e = threadIdx.x; e < (L << lr); e += 256) nu_s[e] = x[e];
    __syncthreads();
    nu_fft_lds(nu_s, ll, lr, 1, L, &tw, lt);
    for (int e = threadIdx.x; e < (L << lr); e += 256) x[e] = nu_s[e];
}

// Pass 2 of the FFT fused with the combine: block (k1, r) transforms row k1 (length 2^ll = n2) of every moment p of
// trial-grid row r, from p = P-1 down to 0, and keeps the Horner sum A = B_p + (z / (p+1)) A of its 2^ll positions in
// registers (z = 2 pi i jc / n), so the moments' transforms are read once and never written back; the trials' (C_k,
// S_k) go to CS as k_nu_combine writes them. X[beta][pos], beta = p * nrow + r, pos = k1 n2 + k2 holds J = k1 + n1 k2.
constexpr int kNuFusedPer = kNuTile / 256;  // positions per thread
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1))) void k_nu_fft_rows_combine(const double2* __restrict__ X, int ll, int lnfft, int P,
                                                             int nrow, int64_t nf, int64_t jhi, int64_t h,
                                                             int64_t tbase, int64_t nbt, const double* __restrict__ bc,
                                                             double2* __restrict__ CS) {
    extern __shared__ double2 nu_s[];
    __shared__ NuTile tw;
    const int lt = lnfft < 12 ? lnfft : 12;
    nu_tile_init(&tw, lt);
    const int64_t nfft = int64_t(1) << lnfft;
    const int L = 1 << ll, ln1 = lnfft - ll;
    const int64_t k1 = blockIdx.x;
    const int r = blockIdx.y;
    double2 acc[kNuFusedPer], nx[kNuFusedPer];
    NuBes bs[kNuFusedPer];
    const double2* xr = X + (int64_t)r * nfft + (k1 << ll);  // moment p's row at xr + p nrow nfft
    const int64_t pstride = (int64_t)nrow * nfft;
#pragma unroll
    for (int q = 0; q < kNuFusedPer; ++q) {
        acc[q] = make_double2(0.0, 0.0);
        const int e = threadIdx.x + 256 * q;
        const int64_t J = k1 + ((int64_t)e << ln1);
        bs[q] = nu_bes_start(bc, P, nu_zh(J <= jhi ? J : J - nfft, lnfft));
        nx[q] = e < L ? xr[(int64_t)(P - 1) * pstride + e] : make_double2(0.0, 0.0);
    }
    for (int p = P - 1; p >= 0; --p) {
        // this moment's row into the tile, the next one's loads issued before the transform
        const int64_t pn = (int64_t)(p > 0 ? p - 1 : 0) * pstride;
#pragma unroll
        for (int q = 0; q < kNuFusedPer; ++q) {
            const int e = threadIdx.x + 256 * q;
            if (e < L) {
                nu_s[e] = nx[q];
                nx[q] = xr[pn + e];
            }
        }
        __syncthreads();
        nu_fft_lds(nu_s, ll, 0, 1, L, &tw, lt);
#pragma unroll
        for (int q = 0; q < kNuFusedPer; ++q) {
            const int b = threadIdx.x + 256 * q;
            if (b < L) {
                const double2 v = nu_s[b];
                const int64_t J = k1 + ((int64_t)b << ln1);
                const int64_t jc = J <= jhi ? J : J - nfft;  // positions between the two ends hold no trial
                // k_nu_combine's arithmetic exactly: eps_p i^p J_p(z), z/2 = (pi/2) jc / n (nu_bes_w)
                acc[q] = nu_bes_acc(acc[q], nu_bes_w(bs[q], p, nu_zh(jc, lnfft)), v, p);
            }
        }
        __syncthreads();  // the next moment's store overwrites the tile
    }
#pragma unroll
    for (int q = 0; q < kNuFusedPer; ++q) {
        const int b = threadIdx.x + 256 * q;
        if (b >= L) continue;
        const int64_t J = k1 + ((int64_t)b << ln1);
        int64_t jc;
        if (J <= jhi)
            jc = J;
        else if (J >= nfft - h)
            jc = J - nfft;
        else
            continue;
        const int64_t t = tbase + r * nf + jc;  // (row0 + r) nf + jbase + jc - tb0
        if (t >= 0 && t < nbt) CS[t] = acc[q];
    }
}

// k_nu_fft_rows_combine for n2 = 4096 (the four-step FFT's rows; three radix-16 stages): the same arithmetic as
// nu_fft_lds (the same stages, twiddles and butterflies, so bit-identical powers) with stage 1 on the row as loaded
// into registers (thread t holds elements t + 256 r) and stage 3's outputs -- positions t + 256 r -- kept in registers
// for the Horner sum: the tile is written and read twice per moment instead of four times. Two 64 KB tiles (stage 1
// -> A, stage 2 -> B) leave two barriers per moment; element i of a tile is stored at i ^ ((i >> 4) & 15), which
// spreads stage 1's stride-16 writes over all banks. The next moment's row loads are issued before the transform.
__device__ __forceinline__ int nu_sw(int i) { return i ^ ((i >> 4) & 15); }
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1))) void k_nu_rows4096_combine(
    const double2* __restrict__ X, int lnfft, int P, int nrow, int64_t nf, int64_t jhi, int64_t h, int64_t tbase,
    int64_t nbt, const double* __restrict__ bc, double2* __restrict__ CS) {
    extern __shared__ double2 nu_s[];  // [2][4096]
    __shared__ NuTile tw;
    nu_tile_init(&tw, 12);
    double2* A = nu_s;
    double2* B = nu_s + 4096;
    const int64_t nfft = int64_t(1) << lnfft;
    const int ln1 = lnfft - 12;
    const int64_t k1 = blockIdx.x;
    const int r = blockIdx.y;
    const int t = threadIdx.x;
    const double2* xr = X + (int64_t)r * nfft + (k1 << 12);
    const int64_t pstride = (int64_t)nrow * nfft;
    double2 acc[16], nx[16], v[16];
    NuBes bs[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        acc[q] = make_double2(0.0, 0.0);
        const int64_t J = k1 + ((int64_t)(t + 256 * q) << ln1);
        bs[q] = nu_bes_start(bc, P, nu_zh(J <= jhi ? J : J - nfft, lnfft));
        nx[q] = xr[(int64_t)(P - 1) * pstride + t + 256 * q];
    }
    // twiddle indices of this thread's butterflies (units of w_4096): stage 2 w_256^{t & 15}, stage 3 w_4096^t
    const int m2 = (t & 15) << 4, m3 = t;
    const int z0 = ((t >> 4) << 8) + (t & 15);  // stage 2's output base
    __syncthreads();                            // tw
    for (int p = P - 1; p >= 0; --p) {
        const int64_t pn = (int64_t)(p > 0 ? p - 1 : 0) * pstride;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            v[q] = nx[q];
            nx[q] = xr[pn + t + 256 * q];
        }
        nu_dft16(v);  // stage 1 (Ns = 1: no twiddles)
#pragma unroll
        for (int q = 0; q < 16; ++q) A[nu_sw(16 * t + q)] = v[q];
        __syncthreads();
#pragma unroll
        for (int q = 0; q < 16; ++q) v[q] = A[nu_sw(t + 256 * q)];
        nu_twiddle<16>(nu_tw_tile(&tw, m2), v);
        nu_dft16(v);  // stage 2 (Ns = 16)
#pragma unroll
        for (int q = 0; q < 16; ++q) B[nu_sw(z0 + 16 * q)] = v[q];
        __syncthreads();
#pragma unroll
        for (int q = 0; q < 16; ++q) v[q] = B[nu_sw(t + 256 * q)];
        nu_twiddle<16>(nu_tw_tile(&tw, m3), v);
        nu_dft16(v);  // stage 3 (Ns = 256): output position t + 256 q
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int64_t J = k1 + ((int64_t)(t + 256 * q) << ln1);
            const int64_t jc = J <= jhi ? J : J - nfft;
            acc[q] = nu_bes_acc(acc[q], nu_bes_w(bs[q], p, nu_zh(jc, lnfft)), v[q], p);
        }
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const int64_t J = k1 + ((int64_t)(t + 256 * q) << ln1);
        int64_t jc;
        if (J <= jhi)
            jc = J;
        else if (J >= nfft - h)
            jc = J - nfft;
        else
            continue;
        const int64_t tt = tbase + r * nf + jc;
        if (tt >= 0 && tt < nbt) CS[tt] = acc[q];
    }
}

// k_nu_rows4096_combine with 512 threads and four radix-8 stages (8 elements per thread): two waves per SIMD from
// one block per CU (the radix-16 form holds 16 elements per thread and runs one). Stage 1 on the loaded row, stage 4's
// outputs (positions t + 512 r) in registers for the moment sum, stages 2-3 through two padded 72 KB tiles whose
// roles alternate between moments (three barriers per moment). The transform's arithmetic differs from the radix-16
// form's in rounding only. Measured (profiles/r06/ab_p2_probes.log, config 3): without its loads the pass takes 0.90
// of its time, without its LDS exchanges 0.85, without the transform's arithmetic 0.81, without both 0.69 -- the
// loads, exchanges and arithmetic of one block per CU overlap little; 30 % fewer VALU instructions (below) or a second
// moment's loads in flight moved it by 1-2 %, rows of 2048 with two blocks per CU by 9 % (pass 1 then needs 512-row
// columns), an L2 touch of the rows two moments ahead cost 12 % (profiles/r06/ab_p2_l2prefetch_rejected.log).
// Moment chunks: the launch transforms moments plo .. P-1 (X holds their planes only, beta = (p - plo) nrow + r) and,
// with accum, adds its partial sum to the CS an earlier chunk (moments above P) wrote -- the sum over moments is
// linear, and each chunk starts the Bessel recurrence at its own top (nu_bes_start(P)).
// The last harmonic's launch may finalize (NuFinal.on): its sums stay in registers and each trial's power and
// certificate are formed there from the earlier harmonics' CS (nu_power), the fix-up list appended, and the block's
// best trial (np.argmax semantics) written to best_part for k_best_final -- no CS write, no finalize launch, no
// reduction pass over the powers.
struct NuFinal {
    int on, m, stat, Pc;           // Pc: the plan's moments (the certificate), P of the launch may be a chunk's top
    double nph, invfact, rel;
    int64_t tb0;                   // out index of the batch's trial 0
    double* out;
    int* nflag;
    int64_t* flagged;
    BestCand* best_part;           // per-block best (nullable)
    int64_t best_base;
    const double2* CS0;            // harmonic 0's sums of the batch (stride nbt)
};
// The row pass's epilogue: each position's sum to CS (F.on == 0), or (fused finalize, k_nu_finalize's arithmetic
// with the last harmonic from registers) each trial's power, the fix-up list and the block's best trial. Position
// q of thread t is t + TPB q of the row.
template <int TPB, int NP>
__device__ __forceinline__ void nu_rows_epilogue(const double2 (&acc)[NP], int64_t k1, int ln1, int64_t nfft,
                                                 int64_t jhi, int64_t h, int64_t tbase, int r, int64_t nf, int64_t nbt,
                                                 double2* __restrict__ CS, const NuFinal& F, double2* lds,
                                                 int pos0 = -1) {
    const int t = threadIdx.x;
    const int b0 = pos0 < 0 ? t : pos0;  // the thread's first row position (then + TPB q)
    if (!F.on) {
#pragma unroll
        for (int q = 0; q < NP; ++q) {
            const int64_t J = k1 + ((int64_t)(b0 + TPB * q) << ln1);
            int64_t jc;
            if (J <= jhi)
                jc = J;
            else if (J >= nfft - h)
                jc = J - nfft;
            else
                continue;
            const int64_t tt = tbase + r * nf + jc;
            if (tt >= 0 && tt < nbt) CS[tt] = acc[q];
        }
        return;
    }
    BestCand bc_ = {-INFINITY, INT64_MAX};
#pragma unroll
    for (int q = 0; q < NP; ++q) {
        const int64_t J = k1 + ((int64_t)(b0 + TPB * q) << ln1);
        int64_t jc;
        if (J <= jhi)
            jc = J;
        else if (J >= nfft - h)
            jc = J - nfft;
        else
            continue;
        const int64_t tt = tbase + r * nf + jc;
        if (tt < 0 || tt >= nbt) continue;
        double p, err;
        nu_power(F.CS0, nbt, tt, F.m, F.stat, F.nph, nu_err_bound(jc, nfft, F.Pc, F.invfact, F.nph), true, acc[q], &p,
                 &err);
        F.out[F.tb0 + tt] = p;
        if (!(err <= F.rel * fabs(p))) F.flagged[atomicAdd(F.nflag, 1)] = F.tb0 + tt;
        if (best_better(p, F.tb0 + tt, bc_.v, bc_.i)) bc_ = {p, F.tb0 + tt};
    }
    if (!F.best_part) return;
    for (int o = 32; o > 0; o >>= 1) {
        const double v = __shfl_xor(bc_.v, o);
        const int64_t i = __shfl_xor(bc_.i, o);
        if (best_better(v, i, bc_.v, bc_.i)) bc_ = {v, i};
    }
    __syncthreads();  // the tiles are free: the wave candidates go to LDS
    BestCand* red = reinterpret_cast<BestCand*>(lds);
    if ((t & 63) == 0) red[t >> 6] = bc_;
    __syncthreads();
    if (t == 0) {
        for (int w = 1; w < TPB / 64; ++w)
            if (best_better(red[w].v, red[w].i, bc_.v, bc_.i)) bc_ = red[w];
        F.best_part[F.best_base + (int64_t)blockIdx.y * gridDim.x + blockIdx.x] = bc_;
    }
}

// The moment sum is carried in a rotating frame: S_p = sum_{p' >= p} eps_p' i^p' J_p'(z) v_p' as T_p = i^-p S_p,
// T_p = i T_p+1 + w_p v_p -- the product by i an exact swap and negation folded into the two fmas, no per-moment
// select of i^p -- and the Bessel recurrence as 2 J (exact), so w_p = 2 J_p is the state itself (p > 0). Every rounding
// is that of nu_bes_w / nu_bes_acc, so the sums are those of the direct form bit for bit, in ~30 % fewer VALU
// instructions. Two moments per loop iteration: the register arrays alternate between the moment in use and the next
// one's loads, the tiles between their roles (no copies). Rows by buffer loads (one offset register, the element
// offsets in a scalar register); tile element i at i + i / 8, so that every stage's element offsets are compile-time
// constants and its accesses a base plus immediates: 221 VGPRs, no spills (the xor swizzle's per-lane store addresses
// took 256 and spilled). Stride-8 stores stay conflict-free; some reads of a 16-lane group meet 2-way.
struct NuRot {
    double j1, j2, iz2;  // 2 J_p+1, 2 J_p+2 (the next moment's), 2 / z
};
// dynamic LDS of k_nu_rows_combine8<LN2>: two padded tiles
constexpr size_t nu_rows_lds(int ln2) { return 2 * ((size_t(1) << ln2) + (size_t(1) << (ln2 - 3))) * sizeof(double2); }
// LN2 = 12: rows of 4096, 512 threads, four radix-8 stages (Ns = 1, 8, 64, 512). LN2 = 11: rows of 2048 (n = 2^20:
// columns of 512, k_nu_cols512), 256 threads, one radix-4 stage (butterflies t and t + 1024 on v[0, 2, 4, 6] and
// v[1, 3, 5, 7]) then three radix-8 (Ns = 4, 32, 256): half the LDS and threads, two blocks per CU.
template <int LN2>
__global__ __launch_bounds__(1 << (LN2 - 3)) __attribute__((amdgpu_waves_per_eu(2))) void k_nu_rows_combine8(
    const double2* X, int lnfft, int P, int plo, int accum, int nrow, int64_t nf, int64_t jhi, int64_t h,
    int64_t tbase, int64_t nbt, const double* __restrict__ bc, double2* __restrict__ CS, const NuFinal F) {
    constexpr int N = 1 << LN2, TPB = N / 8, NT = N + N / 8;
    constexpr int Ns2 = LN2 == 12 ? 8 : 4, Ns3 = 8 * Ns2;
    static_assert(LN2 == 11 || LN2 == 12, "rows of 2048 or 4096");
    extern __shared__ double2 nu_s[];  // [2][NT]
    __shared__ NuTile tw;
    nu_tile_init(&tw, LN2);
    const int64_t nfft = int64_t(1) << lnfft;
    const int ln1 = lnfft - LN2;
    const int64_t k1 = blockIdx.x;
    const int r = blockIdx.y;
    const int t = threadIdx.x;
    const double2* xr = X + (int64_t)r * nfft + (k1 << LN2);
    const int64_t pstride = (int64_t)nrow * nfft;
    auto load_row = [&](int pm, double2 (&dst)[8]) {  // moment pm's row: elements t + TPB q
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc((void*)(xr + (int64_t)pm * pstride), (short)0, N * 16, 0x00020000);
#pragma unroll
        for (int q = 0; q < 8; ++q)
            dst[q] = __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(rs, t * 16, TPB * 16 * q, 0));
    };
    double2 acc[8], xa[8], xb[8];
    NuRot bs[8];
    // the frame at the top moment: T_P = i^-P S_P (S_P: an earlier chunk's sum at this position's trial, else 0)
    const int rP = P & 3;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        double2 a0 = make_double2(0.0, 0.0);
        const int64_t J = k1 + ((int64_t)(t + TPB * q) << ln1);
        const int64_t jc = J <= jhi ? J : J - nfft;
        if (accum) {
            const int64_t tt = tbase + r * nf + jc;
            if ((J <= jhi || J >= nfft - h) && tt >= 0 && tt < nbt) a0 = CS[tt];
        }
        acc[q] = rP == 0 ? a0 : rP == 1 ? make_double2(a0.y, -a0.x) : rP == 2 ? make_double2(-a0.x, -a0.y)
                                                                        : make_double2(-a0.y, a0.x);
        const NuBes b0 = nu_bes_start(bc, P, nu_zh(jc, lnfft));
        bs[q] = {2.0 * b0.j1, 2.0 * b0.j2, b0.iz2};
    }
    load_row(P - 1 - plo, xa);
    // stage twiddles in units of w_N (stage 4: w_N^{t q})
    const int m2 = (t & (Ns2 - 1)) * (N / (8 * Ns2)), m3 = (t & (Ns3 - 1)) * (N / (8 * Ns3)), m4 = t;
    const int z2 = (t / Ns2) * 8 * Ns2 + (t & (Ns2 - 1)), z3 = (t / Ns3) * 8 * Ns3 + (t & (Ns3 - 1));  // outputs
    // padded bases: element e = base + offset lands at e + e / 8 = (base + base / 8) + (offset + offset / 8 (+1 where
    // the stage-2 offset 4 q carries into the base's bit 3 at LN2 = 11)) -- compile-time offsets
    const int w1 = LN2 == 12 ? 9 * t : 4 * t + (t >> 1), w2 = z2 + (z2 >> 3), w3 = z3 + (z3 >> 3), rd = t + (t >> 3);
    __syncthreads();  // tw
    // one moment: v (its row) through the four stages, moment p - 1's loads into nv, then the sum
    auto moment = [&](auto LAST, int p, double2 (&v)[8], double2 (&nv)[8], double2* A, double2* B) {
        constexpr bool last = decltype(LAST)::value;  // p == 0: w_0 = J_0 (1 where z = 0)
        if (p > plo) load_row(p - 1 - plo, nv);
        if constexpr (LN2 == 12) {
            nu_dft8(v);  // stage 1 (Ns = 1): element 8 t + q
#pragma unroll
            for (int q = 0; q < 8; ++q) A[w1 + q] = v[q];
        } else {
            nu_dft4(v[0], v[2], v[4], v[6]);  // stage 1 (R 4, Ns = 1): elements 4 t + q and 4 t + 1024 + q
            nu_dft4(v[1], v[3], v[5], v[7]);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                A[w1 + q] = v[2 * q];
                A[w1 + N / 2 + N / 16 + q] = v[2 * q + 1];
            }
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = A[rd + TPB * 9 / 8 * q];
        nu_twiddle<8>(nu_tw_tile(&tw, m2), v);
        nu_dft8(v);  // stage 2: element z2 + Ns2 q
#pragma unroll
        for (int q = 0; q < 8; ++q) B[w2 + Ns2 * q + (Ns2 == 8 ? q : q >> 1)] = v[q];
        __syncthreads();
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = B[rd + TPB * 9 / 8 * q];
        nu_twiddle<8>(nu_tw_tile(&tw, m3), v);
        nu_dft8(v);  // stage 3: element z3 + Ns3 q
#pragma unroll
        for (int q = 0; q < 8; ++q) A[w3 + Ns3 * 9 / 8 * q] = v[q];
        __syncthreads();
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = A[rd + TPB * 9 / 8 * q];
        nu_twiddle<8>(nu_tw_tile(&tw, m4), v);
        nu_dft8(v);  // stage 4: output position t + TPB q
        const double pp1 = (double)(p + 1);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const double j = fma(pp1 * bs[q].iz2, bs[q].j1, -bs[q].j2);  // 2 J_p
            bs[q].j2 = bs[q].j1;
            bs[q].j1 = j;
            double w = j;
            // w_0 = J_0, and 1 at z = 0: trial offset jc = J = 0, position 0 of row 0
            if constexpr (last) w = (q == 0 && k1 == 0 && t == 0) ? 1.0 : 0.5 * j;
            acc[q] = make_double2(fma(w, v[q].x, -acc[q].y), fma(w, v[q].y, acc[q].x));  // i T + w v
        }
    };
    // moments P-1 .. max(plo, 1) two per iteration (the first alone when their count is odd), then moment 0
    const int pend = plo > 0 ? plo : 1;
    int p = P - 1;
    double2* TA = nu_s;
    double2* TB = nu_s + NT;
    if (p >= pend && ((p - pend + 1) & 1)) {
        moment(std::false_type(), p, xa, xb, TA, TB);
        --p;
#pragma unroll
        for (int q = 0; q < 8; ++q) xa[q] = xb[q];
        double2* tt = TA;
        TA = TB;
        TB = tt;
    }
    for (; p >= pend; p -= 2) {
        moment(std::false_type(), p, xa, xb, TA, TB);
        moment(std::false_type(), p - 1, xb, xa, TB, TA);
    }
    if (plo == 0) moment(std::true_type(), 0, xa, xb, TA, TB);
    // back to S = i^plo T
    const int rl = plo & 3;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const double2 a = acc[q];
        acc[q] = rl == 0 ? a : rl == 1 ? make_double2(-a.y, a.x) : rl == 2 ? make_double2(-a.x, -a.y)
                                                                : make_double2(a.y, -a.x);
    }
    nu_rows_epilogue<TPB, 8>(acc, k1, ln1, nfft, jhi, h, tbase, r, nf, nbt, CS, F, nu_s);
}

// The 4096-element row pass with one cross-wave exchange per moment. Radix-8 decimation in frequency over the input
// digits n = 512 n3 + 64 n2 + 8 n1 + n0 (outputs k0 + 8 k1 + 64 k2 + 512 k3): stage 1 (over n3, the row as loaded:
// thread t = m = 64 n2 + 8 n1 + n0) then w_4096^(m k0); one exchange through a 64 KB tile to thread (wave k0, lane
// m' = 8 n1 + n0), whose wave reads the tile's 8 KB region k0 only; stage 2 (over n2) then w_512^(m' k1); an exchange
// inside the wave (lane 8 k1 + n0) through its own region of the tile, which no other wave reads; stage 3 (over n1)
// then w_64^(n0 k2); a second exchange inside the wave (lane 8 k1 + k2); stage 4 (over n0): outputs k3 at positions
// k0 + 8 k1 + 64 k2 + 512 k3. Two tiles alternate between moments, so one barrier per moment (the cross-wave exchange)
// suffices: a tile is written again two moments later, after every wave has passed the next moment's barrier and with
// it left the tile. Every exchange conflict-free (linear or lane-xor layouts); the wave-level exchanges wait only for
// their own stores. Moment sum as k_nu_rows_combine8 (rotating frame, doubled Bessel state, two moments per iteration).
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2))) void k_nu_rows_iw(
    const double2* X, int lnfft, int P, int plo, int accum, int nrow, int64_t nf, int64_t jhi, int64_t h,
    int64_t tbase, int64_t nbt, const double* __restrict__ bc, double2* __restrict__ CS, const NuFinal F) {
    constexpr int N = 4096, TPB = 512;
    extern __shared__ double2 nu_s[];  // [2][4096]
    __shared__ NuTile tw;
    nu_tile_init(&tw, 12);
    const int64_t nfft = int64_t(1) << lnfft;
    const int ln1 = lnfft - 12;
    const int64_t k1b = blockIdx.x;
    const int r = blockIdx.y;
    const int t = threadIdx.x, w = t >> 6, L = t & 63, hi3 = L >> 3, lo3 = L & 7;
    const int pos0 = w + 8 * hi3 + 64 * lo3;  // output positions pos0 + 512 q
    const double2* xr = X + (int64_t)r * nfft + (k1b << 12);
    const int64_t pstride = (int64_t)nrow * nfft;
    auto load_row = [&](int pm, double2 (&dst)[8]) {  // moment pm's row: elements t + 512 q
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc((void*)(xr + (int64_t)pm * pstride), (short)0, N * 16, 0x00020000);
#pragma unroll
        for (int q = 0; q < 8; ++q)
            dst[q] = __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(rs, t * 16, TPB * 16 * q, 0));
    };
    double2 acc[8], xa[8], xb[8];
    NuRot bs[8];
    const int rP = P & 3;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        double2 a0 = make_double2(0.0, 0.0);
        const int64_t J = k1b + ((int64_t)(pos0 + TPB * q) << ln1);
        const int64_t jc = J <= jhi ? J : J - nfft;
        if (accum) {
            const int64_t tt = tbase + r * nf + jc;
            if ((J <= jhi || J >= nfft - h) && tt >= 0 && tt < nbt) a0 = CS[tt];
        }
        acc[q] = rP == 0 ? a0 : rP == 1 ? make_double2(a0.y, -a0.x) : rP == 2 ? make_double2(-a0.x, -a0.y)
                                                                        : make_double2(-a0.y, a0.x);
        const NuBes b0 = nu_bes_start(bc, P, nu_zh(jc, lnfft));
        bs[q] = {2.0 * b0.j1, 2.0 * b0.j2, b0.iz2};
    }
    load_row(P - 1 - plo, xa);
    // tile offsets: cross-wave store (q 512 + n2 64 + m'), its read (k0 512 + n2 64 + m'), wave-level exchange 1 store
    // (64 n1 + 8 k1 + n0) / read (64 n1 + 8 k1 + n0, n1 = q), exchange 2 store (64 k2 + 8 k1 + (n0 ^ k2)) / read
    const int cw = 64 * w + L, cr = 512 * w + L, e1w = 512 * w + 64 * hi3 + lo3, e2w = 512 * w + 8 * hi3,
              e2r = 512 * w + 64 * lo3 + 8 * hi3;
    __syncthreads();  // tw
    auto moment = [&](auto LAST, int p, double2 (&v)[8], double2 (&nv)[8], double2* A) {
        constexpr bool last = decltype(LAST)::value;
        if (p > plo) load_row(p - 1 - plo, nv);
        nu_dft8(v);  // stage 1 (over n3): k0 = q
        nu_twiddle<8>(nu_tw_tile(&tw, t), v);
#pragma unroll
        for (int q = 0; q < 8; ++q) A[cw + 512 * q] = v[q];
        __syncthreads();
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = A[cr + 64 * q];
        nu_dft8(v);  // stage 2 (over n2): k1 = q
        nu_twiddle<8>(nu_tw_tile(&tw, 8 * L), v);
#pragma unroll
        for (int q = 0; q < 8; ++q) A[e1w + 8 * q] = v[q];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the wave's own stores, before its lanes read them
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = A[cr + 64 * q];
        nu_dft8(v);  // stage 3 (over n1): k2 = q
        nu_twiddle<8>(nu_tw_tile(&tw, 64 * lo3), v);
#pragma unroll
        for (int q = 0; q < 8; ++q) A[e2w + 64 * q + (lo3 ^ q)] = v[q];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = A[e2r + (q ^ lo3)];
        nu_dft8(v);  // stage 4 (over n0): k3 = q, position pos0 + 512 q
        const double pp1 = (double)(p + 1);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const double j = fma(pp1 * bs[q].iz2, bs[q].j1, -bs[q].j2);  // 2 J_p
            bs[q].j2 = bs[q].j1;
            bs[q].j1 = j;
            double wgt = j;
            // w_0 = J_0, and 1 at z = 0: position 0 of row 0 (pos0 = 0: thread 0)
            if constexpr (last) wgt = (q == 0 && k1b == 0 && pos0 == 0) ? 1.0 : 0.5 * j;
            acc[q] = make_double2(fma(wgt, v[q].x, -acc[q].y), fma(wgt, v[q].y, acc[q].x));
        }
    };
    const int pend = plo > 0 ? plo : 1;
    int p = P - 1;
    double2* TA = nu_s;
    double2* TB = nu_s + N;
    if (p >= pend && ((p - pend + 1) & 1)) {
        moment(std::false_type(), p, xa, xb, TA);
        --p;
#pragma unroll
        for (int q = 0; q < 8; ++q) xa[q] = xb[q];
        double2* tt = TA;
        TA = TB;
        TB = tt;
    }
    for (; p >= pend; p -= 2) {
        moment(std::false_type(), p, xa, xb, TA);
        moment(std::false_type(), p - 1, xb, xa, TB);
    }
    if (plo == 0) moment(std::true_type(), 0, xa, xb, TA);
    const int rl = plo & 3;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const double2 a = acc[q];
        acc[q] = rl == 0 ? a : rl == 1 ? make_double2(-a.y, a.x) : rl == 2 ? make_double2(-a.x, -a.y)
                                                                : make_double2(a.y, -a.x);
    }
    nu_rows_epilogue<TPB, 8>(acc, k1b, ln1, nfft, jhi, h, tbase, r, nf, nbt, CS, F, nu_s, pos0);
}

// (C_k, S_k) of the trials of one harmonic: position pos = k1 n2 + k2 of the FFT output holds J = k1 + n1 k2
// (ln1 = 0: natural order); J = jc mod n. The moments' transforms weighted by eps_p i^p J_p(pi jc / n) (nu_bes).
__global__ __launch_bounds__(256) void k_nu_combine(const double2* __restrict__ Z, int lnfft, int ln1, int P, int nrow,
                                                    int64_t nf, int64_t nseg, int64_t h, int64_t jbase, int64_t row0,
                                                    int64_t tb0, int64_t nbt, const double* __restrict__ bc,
                                                    double2* __restrict__ CS) {
    const int64_t nfft = int64_t(1) << lnfft;
    const int64_t pos = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int row = blockIdx.y;
    if (pos >= nfft) return;
    const int ln2 = lnfft - ln1;
    const int64_t J = (pos >> ln2) + ((pos & ((int64_t(1) << ln2) - 1)) << ln1);
    int64_t jc;
    if (J <= nseg - 1 - h)
        jc = J;
    else if (J >= nfft - h)
        jc = J - nfft;
    else
        return;
    const int64_t t = (row0 + row) * nf + jbase + jc - tb0;
    if (t < 0 || t >= nbt) return;
    const double zh = nu_zh(jc, lnfft);
    double2 A = make_double2(0.0, 0.0);
    NuBes bs = nu_bes_start(bc, P, zh);
    for (int p = P - 1; p >= 0; --p) {  // sum_p eps_p i^p J_p(z) B_p (nu_bes_w)
        const double2 b = Z[((int64_t)p * nrow + row) * nfft + pos];
        A = nu_bes_acc(A, nu_bes_w(bs, p, zh), b, p);
    }
    CS[t] = A;
}

// Z^2 / H of trials tb0 .. tb0+nbt-1 (flat, relative to the call's first) from CS[k][t], in the reference's formula
// order, with the certificate: |A_k error| <= E = N (2.4 (x/2)^P / P! + kNuRho), x = pi |jc| / n (invfact =
// 2.4 / (2^P P!), nu_trunc), so Z2_k = (2/N)|A_k|^2
// errs by <= (2/N)(2 |A_k| E + E^2); Z^2 sums them, H = max_k g_k takes the largest bound among the g_k that the
// errors could lift to the maximum (as k_search_finalize_exact). A trial whose bound exceeds rel |power| goes to the
// fp64 fix-up list.
__global__ __launch_bounds__(256) void k_nu_finalize(const double2* __restrict__ CS, int64_t nbt, int m, int stat,
                                                     double nph, int64_t nf, int64_t jbase, int64_t nfft, int P,
                                                     double invfact, double rel, int64_t tb0, int64_t first,
                                                     double* __restrict__ out, int* __restrict__ nflag,
                                                     int64_t* __restrict__ flagged) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nbt) return;
    const int64_t flat = tb0 + t + first;
    const int64_t jc = flat % nf - jbase;
    double p, err;
    nu_power(CS, nbt, t, m, stat, nph, nu_err_bound(jc, nfft, P, invfact, nph), false, make_double2(0.0, 0.0), &p,
             &err);
    out[tb0 + t] = p;
    if (!(err <= rel * fabs(p))) flagged[atomicAdd(nflag, 1)] = tb0 + t;
}

// ---- host ----
static int g_last_search_path = 0;  // crimp_last_search_path(): 0 fp64 direct, 1 exact, 2 nufft
static int64_t g_last_nufft_n = 0;   // crimp_last_nufft_plan(): the last NUFFT's largest FFT length, its moments,
static int g_last_nufft_p = 0;       // and its spread form (1 cell gather, 0 MFMA slots)
static int g_last_nufft_gather = 0;
// Kernel classes of a NUFFT search (timed spans and work counts): cell starts, spread (cell gather or MFMA slots),
// merge, FFT pass 1 (columns), FFT pass 2 (rows, with the Horner sum when fused), the separate Horner sum, finalize.
enum { kNuClsCellStart, kNuClsSpread, kNuClsMerge, kNuClsPass1, kNuClsPass2, kNuClsCombine, kNuClsFinalize, kNuCls };
// crimp_last_nufft_work(): the last NUFFT's algorithmic work -- [0] spread fp64 flops, then HBM bytes per class 1..6
// ([1] the spread's bytes; class 0, the cell starts, is not counted)
static double g_nu_work[kNuCls] = {0, 0, 0, 0, 0, 0, 0};

// truncation bound of P Chebyshev moments per unit photon weight at x = pi |jc| / n: 2.4 (x/2)^P / P! (nu_bes);
// invfact = 2.4 / (2^P P!), so that k_nu_finalize's x^P invfact is the bound
static double nu_trunc(double x, int P, double* invfact) {
    double f = 1.0, xp = 1.0;
    for (int p = 1; p <= P; ++p) {
        f *= 2.0 * (double)p;
        xp *= x;
    }
    *invfact = 2.4 / f;
    return 2.4 * xp / f;
}

static int ilog2(int64_t v) {
    int l = 0;
    while ((int64_t(1) << l) < v) ++l;
    return l;
}

// per-call twiddle (w_n^t) and cis tables, fp64 from long double
// Twiddle (w_n, two-level) and cis tables for n = 2^lnfft, built once per device and n (long double on the host) and
// kept for the process: a search reuses them without an upload.
static int nu_tables(Scratch& sc, hipStream_t s, int lnfft, NuTw* T, const double2** cis, const double** bc,
                     const double2** cis2) {
    (void)sc;
    static std::mutex mu;
    static std::map<std::pair<int, int>, double2*> cache;
    const int lbits = std::min(lnfft, 11);
    const int64_t nlo = int64_t(1) << lbits, nhi = int64_t(1) << (lnfft - lbits);
    int dev = 0;
    HIPCHK(hipGetDevice(&dev));
    double2* d = nullptr;
    {
        std::lock_guard<std::mutex> lk(mu);
        auto it = cache.find({dev, lnfft});
        if (it != cache.end()) {
            d = it->second;
        } else {
            std::vector<double2> h((size_t)(nlo + nhi + 1024 + kNuBesP * kNuBesM / 2 + 2048));
            const long double tp = 6.283185307179586476925286766559L;
            const long double nf = (long double)(int64_t(1) << lnfft);
            for (int64_t i = 0; i < nlo; ++i) {
                const long double a = tp * (long double)i / nf;
                h[(size_t)i] = make_double2((double)cosl(a), (double)sinl(a));
            }
            for (int64_t i = 0; i < nhi; ++i) {
                const long double a = tp * (long double)(i << lbits) / nf;
                h[(size_t)(nlo + i)] = make_double2((double)cosl(a), (double)sinl(a));
            }
            for (int i = 0; i < 1024; ++i) {
                const long double a = tp * (long double)i / 1024.0L;
                h[(size_t)(nlo + nhi + i)] = make_double2((double)cosl(a), (double)sinl(a));
            }
            // nu_bes_series coefficients 1 / (m! (m+p)!), [p][m]
            double* bco = reinterpret_cast<double*>(h.data() + nlo + nhi + 1024);
            for (int p = 0; p < kNuBesP; ++p)
                for (int m = 0; m < kNuBesM; ++m) {
                    long double f = 1.0L;
                    for (int q = 2; q <= m; ++q) f *= (long double)q;
                    for (int q = 2; q <= m + p; ++q) f *= (long double)q;
                    bco[p * kNuBesM + m] = (double)(1.0L / f);
                }
            for (int i = 0; i < 2048; ++i) {  // nu_cis2
                const long double a = tp * (long double)i / 2048.0L;
                h[(size_t)(nlo + nhi + 1024 + kNuBesP * kNuBesM / 2 + i)] = make_double2((double)cosl(a), (double)sinl(a));
            }
            HIPCHK(hipMalloc(&d, h.size() * sizeof(double2)));
            HIPCHK(hipMemcpyAsync(d, h.data(), h.size() * sizeof(double2), hipMemcpyHostToDevice, s));
            HIPCHK(hipStreamSynchronize(s));  // h is pageable and local
            cache[{dev, lnfft}] = d;
        }
    }
    T->lo = d;
    T->hi = d + nlo;
    T->lbits = lbits;
    T->mask = (int64_t(1) << lnfft) - 1;
    *cis = d + nlo + nhi;
    *bc = reinterpret_cast<const double*>(d + nlo + nhi + 1024);
    *cis2 = d + nlo + nhi + 1024 + kNuBesP * kNuBesM / 2;
    return CRIMP_OK;
}

// The FFT input's occupied rows a in [alo, alo + acnt) (mod n1) of the four-step view [n1][n2]: the wrapped cells
// of harmonic k's unwrapped range [gmin, gmax], widened to whole rows; a single-pass FFT (n1 = 1) or a range that
// wraps the grid takes all rows. Only those rows are spread into and read by pass 1; the others are zero.
static void nu_occupied(int64_t gmin, int64_t gmax, int lnfft, int ln1, int* alo, int* acnt) {
    const int64_t nfft = int64_t(1) << lnfft, n1 = int64_t(1) << ln1;
    const int ln2 = lnfft - ln1;
    *alo = 0;
    *acnt = (int)n1;
    if (ln1 == 0 || gmax - gmin + 1 >= nfft) return;
    const int64_t glo = gmin & (nfft - 1), ghi = glo + (gmax - gmin);  // unwrapped end
    const int64_t a0 = glo >> ln2, a1 = ghi >> ln2;
    if (a1 - a0 + 1 >= n1) return;
    *alo = (int)a0;
    *acnt = (int)(a1 - a0 + 1);
}

template <bool TWOD>
static void nu_launch_spread(int G, dim3 grid, hipStream_t s, const double* tt, double t0, int64_t n, int64_t nchunk,
                             double s1,
                             double fch, double fcl, const double* c2, int nrow, int k0, int P, const NuPass* ps,
                             const double2* tab, double* U, int64_t* ctab, const int* bad) {
#define CRIMP_NS(GG) \
    k_nu_spread<GG, TWOD><<<grid, 256, 0, s>>>(tt, t0, n, nchunk, s1, fch, fcl, c2, nrow, k0, P, ps, tab, U, ctab, bad)
    if (G == 10) CRIMP_NS(10); else if (G == 8) CRIMP_NS(8); else if (G == 6) CRIMP_NS(6); else if (G == 4) CRIMP_NS(4);
    else CRIMP_NS(2);
#undef CRIMP_NS
}

// Budget of the NUFFT path's device buffers (CRIMP_NUFFT_BUDGET_MB, default 6144): slots, FFT ping-pong, sums.
template <int R, bool TWOD>
static void launch_gather_r(int64_t blocks, const double* tt, double t0, const int64_t* start, int64_t nfft, double s1,
                            double fch, double fcl, const double* c2, int nrow, int P, const NuGatherSet& S,
                            const int* bad, const double2* tab, double2* W, hipStream_t s) {
    const dim3 grid((unsigned)blocks);
#define NU_GATHER(PPP) \
    k_nu_gather<R, TWOD, PPP><<<grid, 256, 0, s>>>(tt, t0, start, nfft, s1, fch, fcl, c2, nrow, P, S, bad, tab, W)
    if (P <= 14) {  // Z^2_m (m >= 2) at config-3-like grids (kNuEpsZm)
        NU_GATHER(14);
    } else if (P <= 15) {
        NU_GATHER(15);
    } else if (P <= 16) {
        NU_GATHER(16);
    } else if (P <= 20) {
        NU_GATHER(20);
    } else {
        NU_GATHER(kNuGatherMaxP);
    }
#undef NU_GATHER
}
static void launch_gather(bool twod, int64_t blocks, const double* tt, double t0, const int64_t* start, int64_t nfft,
                          double s1, double fch, double fcl, const double* c2, int nrow, int P, const NuGatherSet& S,
                          const int* bad, const double2* tab, double2* W, hipStream_t s) {
    if (twod)
        launch_gather_r<kNuGatherRows, true>(blocks, tt, t0, start, nfft, s1, fch, fcl, c2, nrow, P, S, bad, tab, W, s);
    else
        launch_gather_r<1, false>(blocks, tt, t0, start, nfft, s1, fch, fcl, c2, nrow, P, S, bad, tab, W, s);
}

static int64_t nu_cus() {  // compute units of the current device (persistent grids)
    int dev = 0, ncu = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        ncu <= 0)
        ncu = 256;
    return ncu;
}

// Moments per pass-1 / pass-2 chunk of the radix-8 row path (CRIMP_NUFFT_PCHUNK, an A/B hook read per call; unset, 0
// or above P: one chunk, the whole moment set). Chunks meant the chunk's pass-1 output to be read back from the
// Infinity Cache; measured slower at every size (config 3 pass 1 + pass 2: 0.265 ms whole, 0.352 at 8 moments, 0.527
// at 4, 0.874 at 2; profiles/r06/ab_pchunk.log), so the default is one chunk.
static int nu_pchunk() {
    const char* e = getenv("CRIMP_NUFFT_PCHUNK");
    const int c = e ? atoi(e) : 0;
    return c > 0 ? c : (1 << 20);
}

// CRIMP_NUFFT_FINAL=separate: the k_nu_finalize launch after every row batch instead of the fused finalize (A/B and
// identity test hook, read per call)
static bool nu_final_separate() {
    const char* e = getenv("CRIMP_NUFFT_FINAL");
    return e && !strcmp(e, "separate");
}

static int64_t nufft_budget() {
    static int64_t b = -1;
    if (b < 0) {
        const char* e = getenv("CRIMP_NUFFT_BUDGET_MB");
        const long long mb = e ? atoll(e) : 6144;
        b = (int64_t)(mb > 0 ? mb : 6144) << 20;
    }
    return b;
}

// One group of rows that share their trial segment: rows [r0, r1), trials j0 .. j0+nseg-1 of each, planned on that
// segment alone (a rank's slice of a row is its own progression, so a sharded search costs its share).
struct NuPlan {
    int64_t r0 = 0, r1 = 0, j0 = 0, nseg = 0, h = 0;  // jc = j - (j0 + h) in [-h, nseg - 1 - h]
    int lnfft = 0, P = 0;
    double invfact = 1.0, s1 = 0.0, fch = 0.0, fcl = 0.0;
    std::vector<int64_t> gmin, gmax;                     // unwrapped cells of dt[0], dt[n-1] per harmonic
};

// n and P: among the powers of two n >= nseg (up to 2^24) whose edge truncation (nu_trunc) <= kNuEps within P <= pmax
// moments, the one with the least FFT work n P; false when none exists or the photons wrap the grid more than
// kNuMaxWrap times
static bool nu_plan(NuPlan* pl, double delta, double f0, double dt0, double dtn, int nharm, int64_t nchunk, int pmax,
                    double eps) {
    // an ascending progression only: with delta < 0 the cells of the later photons come first (s1 < 0) and every
    // table below would be sized negative (a descending grid takes the exact rule)
    if (!(delta > 0.0) || !std::isfinite(delta) || !std::isfinite(f0)) return false;
    const int64_t h = pl->nseg / 2;
    pl->h = h;
    int lnfft = 0, P = 0;
    double invfact = 1.0;
    for (int l = std::max(ilog2(pl->nseg), 6); l <= 24; ++l) {
        const double x = M_PI * (double)std::max<int64_t>(h, pl->nseg - 1 - h) / (double)(int64_t(1) << l);
        int p = 1;
        while (p <= pmax && nu_trunc(x, p, &invfact) > eps) ++p;
        if (p > pmax) continue;
        if (lnfft == 0 || ((int64_t)p << l) < ((int64_t)P << lnfft)) {
            lnfft = l;
            P = p;
        }
        if (p <= 4) break;  // larger n only adds work
    }
    if (lnfft == 0) return false;
    nu_trunc(0.0, P, &invfact);
    pl->lnfft = lnfft;
    pl->P = P;
    pl->invfact = invfact;
    const int64_t nfft = int64_t(1) << lnfft;
    pl->s1 = (double)nfft * delta;
    // fc = f_0 + (j0 + h) delta in double-double (the whole grid's progression model, whatever the segment)
    const double c = (double)(pl->j0 + h);
    const double hp = c * delta, hpe = std::fma(c, delta, -hp);
    const double fch = f0 + hp, bb = fch - f0;  // TwoSum(f0, hp)
    pl->fch = fch;
    pl->fcl = ((f0 - (fch - bb)) + (hp - bb)) + hpe;
    // the kernel's arithmetic: rint(k * (dt * s1))
    const double u0 = dt0 * pl->s1, un = dtn * pl->s1;
    // The kernels convert cells with 32-bit rint (k_nu_spread, k_nu_cellstart, k_nu_gather): every cell of every
    // harmonic, one FFT length of margin included, must fit an int -- a t0 far from the photons (t0 = 0 with MJD
    // seconds) can push |G| past 2^31 although the span is small. The plan is declined then (the exact rule runs).
    const double glim = 2147483647.0 - (double)nfft;
    pl->gmin.assign((size_t)nharm, 0);
    pl->gmax.assign((size_t)nharm, 0);
    (void)nchunk;
    for (int k = 1; k <= nharm; ++k) {
        const double a = (double)k * u0, b = (double)k * un;
        if (!(std::fabs(a) < glim && std::fabs(b) < glim)) return false;  // NaN declines too
        pl->gmin[(size_t)(k - 1)] = (int64_t)std::rint(a);
        pl->gmax[(size_t)(k - 1)] = (int64_t)std::rint(b);
        // descending cells (a descending grid, delta < 0, or photons out of order at the ends) would size the
        // slot and start tables negative: declined
        if (pl->gmax[(size_t)(k - 1)] < pl->gmin[(size_t)(k - 1)]) return false;
        if ((pl->gmax[(size_t)(k - 1)] - pl->gmin[(size_t)(k - 1)]) / nfft + 1 > kNuMaxWrap) return false;
    }
    return true;
}

// Z^2 / H by NUFFT over trials [first, first + count) of the fd-outer grid (nf trials per row, arithmetic
// progression with step ap[0]). *applicable = false (nothing computed) for unsorted photons or an out-of-range plan:
// the caller takes the exact path.
// The spread form of a grid of nrows_grid rows: the cell gather for <= kNuGatherRows rows, the MFMA slots otherwise
// (CRIMP_NUFFT_SPREAD=gather|mfma forces one, a test hook). Decided from the whole grid, so that row shards compute
// exactly what the whole grid does.
static bool nu_gather_form(int64_t nrows_grid) {
    const char* spread_env = getenv("CRIMP_NUFFT_SPREAD");
    return spread_env && !strcmp(spread_env, "gather")  ? true
           : spread_env && !strcmp(spread_env, "mfma") ? false
                                                       : nrows_grid <= kNuGatherRows;
}

// hs: [delta, f0, dt[0], dt[n-1], unsorted flag (int bits)] as grid_is_progression read them back (the flag only for
// MFMA-slot plans: a cell-gather plan checks the order in its cell-start pass).
// t: photon times (seconds), t0 the search's reference time: the kernels form dt = t - t0 as k_search_prep does;
// dt (and dt^2) arrays are made only for a fix-up.
// A search's last plan, keyed by its buffers and shape (crimp_search reuses it on the next identical call; the device
// re-checks its scalars, k_ap_final). Up to 16 entries, the oldest dropped first.
struct NuSpecKey {
    const void* t;
    const void* f;
    int64_t n, nf, nfd, first, count;
    double t0;
    int nharm, stat, dev, gather;
    bool operator==(const NuSpecKey& o) const {
        return t == o.t && f == o.f && n == o.n && nf == o.nf && nfd == o.nfd && first == o.first &&
               count == o.count && t0 == o.t0 && nharm == o.nharm && stat == o.stat && dev == o.dev &&
               gather == o.gather;
    }
};
struct NuSpecEntry {
    NuSpecKey key;
    double hs[5];
};
static std::vector<NuSpecEntry> g_nu_spec;
static bool nu_spec_disabled() {  // CRIMP_NUFFT_PLAN_CACHE=0: every search reads its plan back (A/B hook)
    const char* e = getenv("CRIMP_NUFFT_PLAN_CACHE");
    return e && !strcmp(e, "0");
}
static NuSpecKey nu_spec_key(const double* t, int64_t n, double t0, const double* f, int64_t nf, int64_t nfd,
                             int nharm, int stat, int64_t first, int64_t count, bool gather) {
    NuSpecKey k{};
    k.stat = stat;
    k.t = t;
    k.f = f;
    k.n = n;
    k.nf = nf;
    k.nfd = nfd;
    k.first = first;
    k.count = count;
    k.t0 = t0;
    k.nharm = nharm;
    k.gather = gather ? 1 : 0;
    (void)hipGetDevice(&k.dev);
    return k;
}
static bool nu_spec_find(const NuSpecKey& k, double* hs) {
    if (nu_spec_disabled()) return false;
    for (const NuSpecEntry& e : g_nu_spec)
        if (e.key == k) {
            std::memcpy(hs, e.hs, sizeof(e.hs));
            return true;
        }
    return false;
}
static void nu_spec_drop(const NuSpecKey& k) {
    for (size_t i = 0; i < g_nu_spec.size(); ++i)
        if (g_nu_spec[i].key == k) {
            g_nu_spec.erase(g_nu_spec.begin() + (std::ptrdiff_t)i);
            return;
        }
}
static void nu_spec_store(const NuSpecKey& k, const double* hs) {
    if (nu_spec_disabled()) return;
    nu_spec_drop(k);
    if (g_nu_spec.size() >= 16) g_nu_spec.erase(g_nu_spec.begin());
    NuSpecEntry e;
    e.key = k;
    std::memcpy(e.hs, hs, sizeof(e.hs));
    g_nu_spec.push_back(e);
}

static int nufft_search(Scratch& sc, hipStream_t s, const double* t, double t0, int64_t n, const double* freq,
                        int64_t nf, int64_t nrows_grid, const double* c2, const double* hs, bool twod, int nharm,
                        int stat, int64_t first,
                        int64_t count, double* out, bool timed, int64_t* nfixed, bool no_fixup, bool* applicable,
                        double* best, bool* best_done, int* nflag, bool* mismatch) {
    *applicable = false;
    *best_done = false;
    *nfixed = 0;
    *mismatch = false;
    int bad = 0;
    memcpy(&bad, hs + 4, sizeof(int));
    if (bad) return CRIMP_OK;
    const double delta = hs[0], f0 = hs[1], dt0 = hs[2], dtn = hs[3];
    const int64_t nchunk = cdiv(n, kNuCW);
    // spread form: the cell gather (VALU, one lane per wrapped cell) for grids of <= kNuGatherRows rows, the MFMA
    // slots otherwise -- decided from the whole grid, so that row shards compute exactly what the whole grid does
    // (CRIMP_NUFFT_SPREAD=gather|mfma forces one, a test hook)
    const bool gather_grid = nu_gather_form(nrows_grid);
    // row groups: the first row's segment, the full rows between, the last row's segment
    const int64_t r_lo = first / nf, r_hi = (first + count - 1) / nf;
    std::vector<NuPlan> plans;
    for (int64_t r = r_lo; r <= r_hi;) {
        const int64_t a = std::max<int64_t>(first, r * nf) - r * nf, b = std::min<int64_t>(first + count, (r + 1) * nf) - r * nf;
        int64_t r1 = r + 1;
        if (a == 0 && b == nf)
            while (r1 <= r_hi && std::min<int64_t>(first + count, (r1 + 1) * nf) - r1 * nf == nf) ++r1;
        NuPlan pl;
        pl.r0 = r;
        pl.r1 = r1;
        pl.j0 = a;
        pl.nseg = b - a;
        if (pl.nseg < 64 || !nu_plan(&pl, delta, f0, dt0, dtn, nharm + 1, nchunk, gather_grid ? kNuGatherMaxP : kNuMaxP,
                                     stat == 0 && nharm >= 2 ? kNuEpsZm : kNuEps))
            return CRIMP_OK;
        plans.push_back(std::move(pl));
        r = r1;
    }
    *applicable = true;
    g_last_search_path = 2;
    g_last_nufft_n = 0;
    for (const NuPlan& pl : plans)
        if ((int64_t(1) << pl.lnfft) > g_last_nufft_n) {
            g_last_nufft_n = int64_t(1) << pl.lnfft;
            g_last_nufft_p = pl.P;
        }
    g_last_nufft_gather = gather_grid ? 1 : 0;
    for (double& w : g_nu_work) w = 0.0;
    // buffers sized for the largest group; harmonics per spread pass: the largest G in {8, 4, 2, 1} whose slots fit
    // the budget beside W, Y and the sums
    int64_t Bmax = 0, nfmax = 0, csmax = 0, nrow_all = 0;
    for (const NuPlan& pl : plans) {
        const int64_t nrow_max = std::min<int64_t>(kNuRows, pl.r1 - pl.r0);
        const int lrow = 12 - std::min(pl.lnfft, 12);
        Bmax = std::max<int64_t>(Bmax, (cdiv((int64_t)pl.P * nrow_max, int64_t(1) << lrow) << lrow) << pl.lnfft);
        csmax = std::max<int64_t>(csmax, (int64_t)nharm * nrow_max * pl.nseg);
        nfmax = std::max<int64_t>(nfmax, int64_t(1) << pl.lnfft);
        nrow_all = std::max<int64_t>(nrow_all, nrow_max);
    }
    // cell-gather grids gather up to kNuGatherSet harmonics per launch, each into its own W planes
    int gw = 1;
    if (gather_grid) {
        gw = std::min(nharm, kNuGatherSet);
        while (gw > 1 && (gw + 1) * Bmax * 16 + csmax * 16 > nufft_budget()) --gw;
    }
    const int64_t fixed_bytes = (gw + 1) * Bmax * 16 + csmax * 16;
    std::vector<std::pair<int, int>> passes;  // (k0, harmonics) of each spread pass, harmonics a power of two
    int64_t ubytes = 0;
    // harmonics per MFMA spread pass: the largest size in {10, 8, 6, 4, 2} (<= Gmax) the remaining harmonics fill,
    // allowing one past nharm (its cells are planned, nu_plan(nharm + 1)): H_20 runs as 10 + 10 (two photon passes;
    // 8 + 8 + 4 paid the per-photon phase and cis three times)
    for (int Gmax = 10;; Gmax = Gmax == 10 ? 8 : Gmax / 2) {  // Gmax >= 2
        const int G = Gmax;
        passes.clear();
        ubytes = 0;
        for (int k0 = 1; k0 <= nharm;) {
            const int rem = nharm - k0 + 1;
            int gl = 2;
            for (int cand : {10, 8, 6, 4, 2})
                if (cand <= G && cand <= rem + 1) {
                    gl = cand;
                    break;
                }
            for (const NuPlan& pl : plans) {
                const int64_t SLmax = 2 * (int64_t)pl.P * std::min<int64_t>(kNuRows, pl.r1 - pl.r0);
                int64_t sl = 0;
                for (int k = k0; k < k0 + gl; ++k)
                    sl += (pl.gmax[(size_t)(k - 1)] - pl.gmin[(size_t)(k - 1)] + 1 + nchunk) * SLmax;
                ubytes = std::max<int64_t>(ubytes, sl * 8);
            }
            passes.emplace_back(k0, gl);
            k0 += gl;
        }
        if (G == 2 || ubytes + fixed_bytes <= nufft_budget()) break;
    }
    auto use_gather = [&](const NuPlan&) { return gather_grid; };
    // pass 2 fused with the combine (default); CRIMP_NUFFT_FUSED=0 runs them as two kernels (A/B hook)
    const char* fused_env = getenv("CRIMP_NUFFT_FUSED");
    const bool fused_combine = !(fused_env && !strcmp(fused_env, "0"));
    // CRIMP_NUFFT_ROWS4096=0 runs 4096-element rows and 256-element columns through the generic kernels (A/B and
    // identity test hook)
    const char* r4_env = getenv("CRIMP_NUFFT_ROWS4096");
    const bool rows4096 = !(r4_env && !strcmp(r4_env, "0"));
    // pass 2 of 4096-element rows by the 512-thread radix-8 kernel (default: 0.178 vs 0.190 ms per config-3 search,
    // profiles/r05/ab_r8_ilp.log); CRIMP_NUFFT_R8=0 runs the radix-16 form
    const char* r8_env = getenv("CRIMP_NUFFT_R8");
    const bool rows_r8 = !(r8_env && !strcmp(r8_env, "0"));
    // CRIMP_NUFFT_ROW2048=1: n = 2^20 as 512 x 2048 (k_nu_cols512, k_nu_rows_combine8<11>), else 256 x 4096. The row
    // pass gains what the column pass loses (config 3: pass 2 0.160 vs 0.180 ms, pass 1 0.138 vs 0.115 ms per search,
    // profiles/r06/ab_rows2048_cols512.log), so 4096-element rows stay the default.
    const char* r2k_env = getenv("CRIMP_NUFFT_ROW2048");
    const bool row2048 = r2k_env && !strcmp(r2k_env, "1") && rows4096 && rows_r8 && fused_combine;
    auto row_log = [&](int lnfft) { return row2048 && lnfft == 20 ? 11 : std::min(lnfft, 12); };
    // 4096-element rows by k_nu_rows_iw (one cross-wave exchange per moment; 0.171 vs 0.180 ms per config-3 search,
    // profiles/r06/ab_p2_iw.log); CRIMP_NUFFT_P2_IW=0: k_nu_rows_combine8<12> (three block-wide exchanges)
    const char* iw_env = getenv("CRIMP_NUFFT_P2_IW");
    const bool p2_iw = !(iw_env && !strcmp(iw_env, "0"));
    {  // 128 KB of dynamic LDS for k_nu_rows4096_combine, set once per device
        static std::mutex mu;
        static uint64_t done = 0;
        int dev = 0;
        HIPCHK(hipGetDevice(&dev));
        std::lock_guard<std::mutex> lk(mu);
        if (dev >= 64 || !(done >> dev & 1)) {
            HIPCHK(hipFuncSetAttribute(reinterpret_cast<const void*>(k_nu_rows4096_combine),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 2 * kNuTile * (int)sizeof(double2)));
            HIPCHK(hipFuncSetAttribute(reinterpret_cast<const void*>(k_nu_rows_combine8<12>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)nu_rows_lds(12)));
            HIPCHK(hipFuncSetAttribute(reinterpret_cast<const void*>(k_nu_rows_iw),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 2 * kNuTile * (int)sizeof(double2)));
            HIPCHK(hipFuncSetAttribute(reinterpret_cast<const void*>(k_nu_rows_combine8<11>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)nu_rows_lds(11)));
            if (dev < 64) done |= uint64_t(1) << dev;
        }
    }
    const char* lanes_s = getenv("CRIMP_NUFFT_LANES");
    const int lanes_env = lanes_s ? atoi(lanes_s) : 0;
    ARGCHK(lanes_env == 0 || lanes_env == 1 || lanes_env == 2 || lanes_env == 4 || lanes_env == 8,
           "CRIMP_NUFFT_LANES must be 1, 2, 4 or 8");
    bool any_mfma = false;
    int64_t starts_max = 0;
    for (const NuPlan& pl : plans) {
        if (!use_gather(pl)) {
            any_mfma = true;
            continue;
        }
        int64_t tot = 0;
        for (int k = 1; k <= nharm; ++k) tot += pl.gmax[(size_t)(k - 1)] - pl.gmin[(size_t)(k - 1)] + 2;
        starts_max = std::max<int64_t>(starts_max, tot);
    }
    double* U = nullptr;
    double2 *W = nullptr, *Y = nullptr, *CS = nullptr;
    int64_t* ctab = nullptr;
    int64_t* cstart = nullptr;
    int64_t* flagged = nullptr;
    // nflag: [fix-up count, photons out of order (1; cell-gather plans) or a cached plan no longer valid (2), -, -,
    // best power, best index (as doubles)], zeroed or set by k_ap_final, read back in one transfer at the end
    if (any_mfma) {
        HIPCHK(sc.alloc(&U, (size_t)(ubytes / 8)));
        HIPCHK(sc.alloc(&ctab, (size_t)(2 * kNuPassMax * nchunk)));
    }
    if (starts_max > 0) HIPCHK(sc.alloc(&cstart, (size_t)starts_max));
    HIPCHK(sc.alloc(&W, (size_t)(Bmax * gw)));
    HIPCHK(sc.alloc(&Y, (size_t)Bmax));
    HIPCHK(sc.alloc(&CS, (size_t)csmax));
    HIPCHK(sc.alloc(&flagged, (size_t)count));
    // per-block best trials of the fused finalize (k_nu_rows_combine8 blocks of every row batch)
    BestCand* best_part = nullptr;
    int64_t best_count = 0, separate_batches = 0;
    if (best) {
        int64_t nb = 0;
        for (const NuPlan& pl : plans) nb += (pl.r1 - pl.r0) * (int64_t(1) << (pl.lnfft - row_log(pl.lnfft)));
        HIPCHK(sc.alloc(&best_part, (size_t)std::max<int64_t>(nb, 1)));
    }
    // every MFMA (group, row batch, pass)'s slot table, uploaded once before the launches
    std::vector<NuPass> hps;
    for (const NuPlan& pl : plans) {
        if (use_gather(pl)) continue;
        for (int64_t rb = pl.r0; rb < pl.r1; rb += kNuRows) {
            const int64_t SL = 2 * (int64_t)pl.P * std::min<int64_t>(kNuRows, pl.r1 - rb);
            for (const auto& pass : passes) {
                NuPass ps{};
                int64_t off = 0;
                for (int kk = 0; kk < pass.second; ++kk) {
                    const int k = pass.first + kk;
                    ps.gmin[kk] = pl.gmin[(size_t)(k - 1)];
                    ps.ubase[kk] = off;
                    off += (pl.gmax[(size_t)(k - 1)] - pl.gmin[(size_t)(k - 1)] + 1 + nchunk) * SL;
                }
                hps.push_back(ps);
            }
        }
    }
    NuPass* dps = nullptr;
    if (!hps.empty()) {
        HIPCHK(sc.alloc(&dps, hps.size()));
        HIPCHK(hipMemcpyAsync(dps, hps.data(), hps.size() * sizeof(NuPass), hipMemcpyHostToDevice, s));
    }
    size_t ipass = 0;
    const size_t lds_fft = (size_t)kNuTile * sizeof(double2);
    // timed spans (CRIMP_FLAG_TIME_KERNELS): the whole pipeline, then each kernel class's sum and launch count
    std::vector<hipEvent_t> ev;
    std::vector<int> evcls;  // class of the span ending at each mark (kNuCls*)
    auto mark = [&]() -> hipError_t {
        if (!timed) return hipSuccess;
        hipEvent_t e = nullptr;
        hipError_t r = hipEventCreate(&e);
        if (r != hipSuccess) return r;
        ev.push_back(e);
        return hipEventRecord(e, s);
    };
    auto span = [&](int cls) -> hipError_t {
        if (!timed) return hipSuccess;
        evcls.push_back(cls);
        return mark();
    };
    int cur_lnfft = -1;
    NuTw T{};
    const double2* cis = nullptr;
    const double2* cis2 = nullptr;
    const double* bc = nullptr;
    for (const NuPlan& pl : plans) {
        if (pl.lnfft != cur_lnfft) {  // tables for this group's n (a group's first launch follows their upload)
            const int rc = nu_tables(sc, s, pl.lnfft, &T, &cis, &bc, &cis2);
            if (rc) return rc;
            cur_lnfft = pl.lnfft;
        }
        if (ev.empty()) HIPCHK(mark());
        const int lnfft = pl.lnfft, P = pl.P;
        const int64_t nfft = int64_t(1) << lnfft;
        // FFT shape: one row pass for n <= kNuTile (2^lrow transforms per block), else columns (n1 = n / 4096 <= 4096)
        // then rows of 4096
        const int ln2 = row_log(lnfft), ln1 = lnfft - ln2;
        const int lcol = 12 - ln1;  // columns per block in pass 1 (n1 * c = 4096)
        const int lrow = 12 - ln2;  // rows per block in pass 2
        const int64_t jbase = pl.j0 + pl.h;
        // W (moments of harmonic k, rows [rb, rb + nrow)) -> FFT -> (C_k, S_k) of the batch's trials
        auto occupied = [&](int k, int* alo, int* acnt) {
            nu_occupied(pl.gmin[(size_t)(k - 1)], pl.gmax[(size_t)(k - 1)], lnfft, ln1, alo, acnt);
        };
        // fused finalize: the last harmonic's row pass forms the powers (NuFinal), for the 4096-row radix-8 path
        const bool fuse_final = fused_combine && ln2 >= 11 && rows4096 && rows_r8 && !nu_final_separate();
        bool final_done = false;  // set by fft_combine when it finalized the batch
        auto fft_combine = [&](int k, int64_t rb, int nrow, int64_t tb0, int64_t nbt, double2* W) -> int {
            const int64_t Bp = (int64_t)P * nrow;
            const double plane = 16.0 * (double)Bp * (double)nfft;  // one complex FFT buffer of the batch
            if (fused_combine && ln2 >= 11 && rows4096 && rows_r8) {
                // moment chunks of <= nu_pchunk() (default: all P moments in one): pass 1 and pass 2 of a chunk in turn
                int alo = 0, acnt = 0;
                if (ln1 > 0) occupied(k, &alo, &acnt);
                const int pc = std::max(1, std::min(nu_pchunk(), P));
                for (int phi = P; phi > 0; phi -= pc) {
                    const int plo = std::max(0, phi - pc);
                    const int64_t Bc = (int64_t)(phi - plo) * nrow;
                    const double cplane = 16.0 * (double)Bc * (double)nfft;
                    const double2* Win = W + (int64_t)plo * nrow * nfft;
                    const double2* Zo = Win;
                    if (ln1 > 0) {
                        g_nu_work[kNuClsPass1] += cplane * ((double)acnt / (double)(int64_t(1) << ln1)) + cplane;
                        if (ln1 == 8) {
                            const int64_t ngroups = Bc << (ln2 - 4);
                            k_nu_cols256<<<(unsigned)std::min<int64_t>(ngroups, 2 * nu_cus()), 256, lds_fft, s>>>(
                                Win, Y, lnfft, T, alo, acnt, ngroups);
                        } else if (ln1 == 9) {
                            const int64_t ngroups = Bc << (ln2 - 3);
                            k_nu_cols512<<<(unsigned)std::min<int64_t>(ngroups, 2 * nu_cus()), 512, lds_fft, s>>>(
                                Win, Y, lnfft, T, alo, acnt, ngroups);
                        } else {
                            k_nu_fft_cols<<<dim3((unsigned)(int64_t(1) << (ln2 - lcol)), (unsigned)Bc), 256, lds_fft,
                                            s>>>(Win, Y, lnfft, ln1, lcol, T, alo, acnt);
                        }
                        HIPCHK(hipGetLastError());
                        Zo = Y;
                        HIPCHK(span(kNuClsPass1));
                    }
                    NuFinal F{};
                    if (fuse_final && k == nharm && plo == 0) {
                        F.on = 1;
                        F.m = nharm;
                        F.stat = stat;
                        F.Pc = P;
                        F.nph = (double)n;
                        F.invfact = pl.invfact;
                        F.rel = fixup_rel();
                        F.tb0 = tb0;
                        F.out = out;
                        F.nflag = nflag;
                        F.flagged = flagged;
                        F.best_part = best ? best_part : nullptr;
                        F.best_base = best_count;
                        F.CS0 = CS;
                        best_count += (int64_t(1) << ln1) * nrow;
                        final_done = true;
                    }
                    // bytes: the chunk's planes; CS read by a later chunk and written, or (fused finalize) the
                    // earlier harmonics' sums read and the powers written
                    g_nu_work[kNuClsPass2] += cplane + (F.on ? (16.0 * (nharm - 1) + 8.0) * (double)nbt
                                                             : 16.0 * (double)nbt * (phi < P ? 2.0 : 1.0));
                    const dim3 g2((unsigned)(int64_t(1) << ln1), (unsigned)nrow);
                    if (ln2 == 12 && p2_iw)
                        k_nu_rows_iw<<<g2, 512, 2 * lds_fft, s>>>(
                            Zo, lnfft, phi, plo, phi < P ? 1 : 0, nrow, nf, pl.nseg - 1 - pl.h, pl.h,
                            rb * nf + jbase - (tb0 + first), nbt, bc, CS + (int64_t)(k - 1) * nbt, F);
                    else if (ln2 == 11)
                        k_nu_rows_combine8<11><<<g2, 256, nu_rows_lds(11), s>>>(
                            Zo, lnfft, phi, plo, phi < P ? 1 : 0, nrow, nf, pl.nseg - 1 - pl.h, pl.h,
                            rb * nf + jbase - (tb0 + first), nbt, bc, CS + (int64_t)(k - 1) * nbt, F);
                    else
                        k_nu_rows_combine8<12><<<g2, 512, nu_rows_lds(12), s>>>(
                            Zo, lnfft, phi, plo, phi < P ? 1 : 0, nrow, nf, pl.nseg - 1 - pl.h, pl.h,
                            rb * nf + jbase - (tb0 + first), nbt, bc, CS + (int64_t)(k - 1) * nbt, F);
                    HIPCHK(hipGetLastError());
                    HIPCHK(span(kNuClsPass2));
                }
                return CRIMP_OK;
            }
            double2* Zo = W;
            if (ln1 > 0) {
                int alo = 0, acnt = 0;
                occupied(k, &alo, &acnt);
                g_nu_work[kNuClsPass1] += plane * ((double)acnt / (double)(int64_t(1) << ln1)) + plane;  // occupied rows in, all out
                if (ln1 == 8 && rows4096) {
                    const int64_t ngroups = Bp << (ln2 - 4);
                    k_nu_cols256<<<(unsigned)std::min<int64_t>(ngroups, 2 * nu_cus()), 256, lds_fft, s>>>(
                        W, Y, lnfft, T, alo, acnt, ngroups);
                    HIPCHK(hipGetLastError());
                } else {
                    k_nu_fft_cols<<<dim3((unsigned)(int64_t(1) << (ln2 - lcol)), (unsigned)Bp), 256, lds_fft, s>>>(
                        W, Y, lnfft, ln1, lcol, T, alo, acnt);
                    HIPCHK(hipGetLastError());
                }
                Zo = Y;
                HIPCHK(span(kNuClsPass1));
            }
            if (fused_combine && ln2 == 12 && rows4096) {  // the specialised form for 4096-element rows
                g_nu_work[kNuClsPass2] += plane + 16.0 * (double)nbt;
                k_nu_rows4096_combine<<<dim3((unsigned)(int64_t(1) << ln1), (unsigned)nrow), 256, 2 * lds_fft, s>>>(
                    Zo, lnfft, P, nrow, nf, pl.nseg - 1 - pl.h, pl.h, rb * nf + jbase - (tb0 + first), nbt, bc,
                    CS + (int64_t)(k - 1) * nbt);
                HIPCHK(hipGetLastError());
                HIPCHK(span(kNuClsPass2));
                return CRIMP_OK;
            }
            if (fused_combine) {  // pass 2 and the moments' Horner sum in one kernel
                g_nu_work[kNuClsPass2] += plane + 16.0 * (double)nbt;
                k_nu_fft_rows_combine<<<dim3((unsigned)(int64_t(1) << ln1), (unsigned)nrow), 256, lds_fft, s>>>(
                    Zo, ln2, lnfft, P, nrow, nf, pl.nseg - 1 - pl.h, pl.h, rb * nf + jbase - (tb0 + first), nbt, bc,
                    CS + (int64_t)(k - 1) * nbt);
                HIPCHK(hipGetLastError());
                HIPCHK(span(kNuClsPass2));
                return CRIMP_OK;
            }
            g_nu_work[kNuClsPass2] += 2.0 * plane;
            g_nu_work[kNuClsCombine] += plane + 16.0 * (double)nbt;
            k_nu_fft_rows<<<(unsigned)cdiv(Bp << ln1, int64_t(1) << lrow), 256, lds_fft, s>>>(Zo, ln2, lrow, lnfft);
            HIPCHK(hipGetLastError());
            HIPCHK(span(kNuClsPass2));
            k_nu_combine<<<dim3((unsigned)cdiv(nfft, 256), (unsigned)nrow), 256, 0, s>>>(
                Zo, lnfft, ln1, P, nrow, nf, pl.nseg, pl.h, jbase, rb, tb0 + first, nbt, bc,
                CS + (int64_t)(k - 1) * nbt);
            HIPCHK(hipGetLastError());
            HIPCHK(span(kNuClsCombine));
            return CRIMP_OK;
        };
        auto finalize = [&](int64_t tb0, int64_t nbt) -> int {
            g_nu_work[kNuClsFinalize] += 16.0 * (double)nharm * (double)nbt + 8.0 * (double)nbt;
            k_nu_finalize<<<(unsigned)cdiv(nbt, 256), 256, 0, s>>>(CS, nbt, nharm, stat, (double)n, nf, jbase, nfft, P,
                                                                   pl.invfact, fixup_rel(), tb0, first, out, nflag,
                                                                   flagged);
            HIPCHK(hipGetLastError());
            HIPCHK(span(kNuClsFinalize));
            return CRIMP_OK;
        };
        if (use_gather(pl)) {
            std::vector<int64_t> soff((size_t)nharm);
            int64_t off = 0;
            // no zeroing of the start tables: on time-sorted photons every entry is written (each cell's first
            // photon writes it), and on unsorted ones the gathers read none of them (k_nu_gather exits on *bad)
            for (int k0 = 1; k0 <= nharm; k0 += kNuCellK) {
                NuCellArgs ca{};
                const int nk = std::min(kNuCellK, nharm - k0 + 1);
                for (int j = 0; j < nk; ++j) {
                    const int k = k0 + j;
                    ca.gmin[j] = pl.gmin[(size_t)(k - 1)];
                    ca.span[j] = pl.gmax[(size_t)(k - 1)] - pl.gmin[(size_t)(k - 1)] + 1;
                    ca.off[j] = off;
                    soff[(size_t)(k - 1)] = off;
                    off += ca.span[j] + 1;
                }
                const unsigned cb = (unsigned)std::min<int64_t>(cdiv(cdiv(n, 2), 256 * kNuCellU), 2048);
                // CRIMP_NUFFT_CS_MODE (A/B probe of the pass's cost): 1 = loads and order check only (the search is
                // discarded), 2 = no block barrier; 0 = the pass
                const char* csm = getenv("CRIMP_NUFFT_CS_MODE");
                const int cs_mode = csm ? atoi(csm) : 0;
                if ((reinterpret_cast<uintptr_t>(t) & 15u) == 0)
                    k_nu_cellstart<true><<<cb, 256, 0, s>>>(t, t0, n, pl.s1, k0, nk, ca, cstart, nflag + 1, cs_mode);
                else
                    k_nu_cellstart<false><<<cb, 256, 0, s>>>(t, t0, n, pl.s1, k0, nk, ca, cstart, nflag + 1, cs_mode);
                HIPCHK(hipGetLastError());
            }
            HIPCHK(span(kNuClsCellStart));
            for (int64_t rb = pl.r0; rb < pl.r1; rb += kNuGatherRows) {
                const int nrow = (int)std::min<int64_t>(kNuGatherRows, pl.r1 - rb);
                const int64_t tb0 = std::max<int64_t>(first, rb * nf) - first;
                const int64_t nbt = std::min<int64_t>(first + count, (rb + nrow) * nf) - first - tb0;
                for (int k0 = 1; k0 <= nharm; k0 += gw) {
                    NuGatherSet S{};
                    S.nk = std::min(gw, nharm - k0 + 1);
                    int64_t blocks = 0, set_cells = 0;  // the set's occupied cells (threads at one lane per cell)
                    for (int jj = 0; jj < S.nk; ++jj) {
                        int alo = 0, acnt = 0;
                        occupied(k0 + jj, &alo, &acnt);
                        set_cells += (int64_t)acnt << ln2;
                    }
                    for (int jj = 0; jj < S.nk; ++jj) {
                        const int k = k0 + jj;
                        int alo = 0, acnt = 0;
                        occupied(k, &alo, &acnt);
                        const int64_t gbase = (int64_t)alo << ln2, gcount = (int64_t)acnt << ln2;
                        // lanes per cell: doubled (up to 4) while the launch's threads stay <= 2^20 -- counted over
                        // every harmonic of the set at the doubled lanes -- and each lane keeps >= 8 photons (config
                        // 3, both harmonics in one launch: 0.099 ms at 2 lanes, 0.108 at 4, 0.143 at 8,
                        // profiles/r06/ab_gather_lanes.log)
                        const int64_t kspan = pl.gmax[(size_t)(k - 1)] - pl.gmin[(size_t)(k - 1)] + 1;
                        const int64_t ppc = n / std::max<int64_t>(1, std::min<int64_t>(kspan, nfft));
                        int L = 1;
                        while (L < 4 && set_cells * 2 * L <= (int64_t(1) << 20) && ppc >= 4 * 2 * L) L *= 2;
                        if (lanes_env > 0) L = lanes_env;  // test hook: CRIMP_NUFFT_LANES=1|2|4|8
                        S.k[jj] = k;
                        S.lanes_log2[jj] = L == 8 ? 3 : L == 4 ? 2 : L == 2 ? 1 : 0;
                        S.blk0[jj] = blocks;
                        blocks += cdiv(gcount * L, 256);
                        S.gmin[jj] = pl.gmin[(size_t)(k - 1)];
                        S.gmax[jj] = pl.gmax[(size_t)(k - 1)];
                        S.gbase[jj] = gbase;
                        S.gcount[jj] = gcount;
                        S.soff[jj] = soff[(size_t)(k - 1)];
                        S.woff[jj] = (int64_t)jj * Bmax;
                        // per photon and row: premultiplier phase + cis ~ 40 flops, then 2 FMA + 1 multiply per moment
                        g_nu_work[0] += (40.0 + 5.0 * P) * (double)n * nrow;
                        g_nu_work[kNuClsSpread] += 8.0 * (double)n + 16.0 * (double)P * nrow * (double)gcount;
                    }
                    S.blk0[S.nk] = blocks;
                    launch_gather(twod, blocks, t, t0, cstart, nfft, pl.s1, pl.fch, pl.fcl, twod ? c2 + rb : nullptr,
                                  nrow, P, S, nflag + 1, cis2, W, s);
                    HIPCHK(hipGetLastError());
                    HIPCHK(span(kNuClsSpread));
                    for (int jj = 0; jj < S.nk; ++jj) {
                        int rc = fft_combine(k0 + jj, rb, nrow, tb0, nbt, W + (int64_t)jj * Bmax);
                        if (rc) return rc;
                    }
                }
                if (final_done) {
                    final_done = false;
                    continue;
                }
                ++separate_batches;
                int rc = finalize(tb0, nbt);
                if (rc) return rc;
            }
            continue;
        }
        for (int64_t rb = pl.r0; rb < pl.r1; rb += kNuRows) {
            const int nrow = (int)std::min<int64_t>(kNuRows, pl.r1 - rb);
            const int64_t tb0 = std::max<int64_t>(first, rb * nf) - first;
            const int64_t tb1 = std::min<int64_t>(first + count, (rb + nrow) * nf) - first;
            const int64_t nbt = tb1 - tb0;
            const int64_t SL = 2 * (int64_t)P * nrow;
            for (const auto& pass : passes) {
                const int k0 = pass.first, gl = pass.second;
                const NuPass& ps = hps[ipass];
                const NuPass* dp = dps + ipass++;
                dim3 grid((unsigned)cdiv(nchunk, kNuWaves));
                // issued: one 16x16x4 f64 MFMA (2048 flops) per 4 photons and harmonic; slots written
                g_nu_work[0] += 512.0 * (double)n * gl;
                g_nu_work[kNuClsSpread] += 8.0 * (double)n;
                for (int kk = 0; kk < gl; ++kk)
                    g_nu_work[kNuClsSpread] += 8.0 * (double)SL *
                                    (double)(pl.gmax[(size_t)(k0 + kk - 1)] - ps.gmin[kk] + 1 + nchunk);
                if (twod)
                    nu_launch_spread<true>(gl, grid, s, t, t0, n, nchunk, pl.s1, pl.fch, pl.fcl, c2 + rb, nrow, k0, P, dp, cis,
                                           U, ctab, nflag + 1);
                else
                    nu_launch_spread<false>(gl, grid, s, t, t0, n, nchunk, pl.s1, pl.fch, pl.fcl, c2 + rb, nrow, k0, P, dp,
                                            cis, U, ctab, nflag + 1);
                HIPCHK(hipGetLastError());
                HIPCHK(span(kNuClsSpread));
                for (int kk = 0; kk < gl && k0 + kk <= nharm; ++kk) {
                    const int k = k0 + kk;
                    int alo = 0, acnt = 0;
                    occupied(k, &alo, &acnt);
                    const int64_t gbase = (int64_t)alo << ln2, gcount = (int64_t)acnt << ln2;
                    g_nu_work[kNuClsMerge] += 8.0 * (double)SL * (double)(pl.gmax[(size_t)(k - 1)] - ps.gmin[kk] + 1 + nchunk) +
                                    16.0 * (double)P * nrow * (double)gcount;
                    k_nu_merge<<<(unsigned)cdiv(gcount, kNuMergeG), 256, (size_t)kNuMergeG * SL * sizeof(double), s>>>(
                        U + ps.ubase[kk], SL, ctab + 2 * kk * nchunk, nchunk, ps.gmin[kk], pl.gmax[(size_t)(k - 1)],
                        nfft, gbase, gcount, W, nflag + 1);
                    HIPCHK(hipGetLastError());
                    HIPCHK(span(kNuClsMerge));
                    int rc = fft_combine(k, rb, nrow, tb0, nbt, W);
                    if (rc) return rc;
                }
            }
            if (final_done) {
                final_done = false;
                continue;
            }
            ++separate_batches;
            int rc = finalize(tb0, nbt);
            if (rc) return rc;
        }
    }
    if (timed) {
        HIPCHK(hipEventSynchronize(ev.back()));
        float tot = 0.0f;
        double cls[kNuCls] = {0, 0, 0, 0, 0, 0, 0}, cnt[kNuCls] = {0, 0, 0, 0, 0, 0, 0};
        HIPCHK(hipEventElapsedTime(&tot, ev.front(), ev.back()));
        for (size_t i = 1; i < ev.size(); ++i) {
            float ms = 0.0f;
            HIPCHK(hipEventElapsedTime(&ms, ev[i - 1], ev[i]));
            cls[evcls[i - 1]] += ms;
            cnt[evcls[i - 1]] += 1.0;  // launches: one per span except the cell starts (one span per nharm launches)
        }
        cnt[kNuClsCellStart] *= (nharm + kNuCellK - 1) / kNuCellK;
        for (hipEvent_t e : ev) (void)hipEventDestroy(e);
        if (g_kernel_times.empty()) g_last_kernel_ms = tot;
        g_kernel_times.push_back(tot);  // then the classes' ms, then their launch counts
        for (double v : cls) g_kernel_times.push_back(v);
        for (double v : cnt) g_kernel_times.push_back(v);
    }
    // the best trial of the powers (crimp_search_best) rides on the same read-back; valid unless a fix-up follows
    if (best) {
        if (separate_batches == 0 && best_count > 0) {  // every batch finalized in its row pass: reduce their blocks
            k_best_final<<<1, 256, 0, s>>>(best_part, (int)best_count, reinterpret_cast<double*>(nflag + 4));
            HIPCHK(hipGetLastError());
        } else {
            const int rc = launch_best(sc, s, out, count, reinterpret_cast<double*>(nflag + 4));
            if (rc) return rc;
        }
    }
    int fl[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    HIPCHK(d2h(s, fl, nflag, (best ? 8 : 2) * sizeof(int)));
    if (fl[1]) {  // photons out of order (found by the cell starts), or a cached plan that no longer holds (2):
        *applicable = false;  // nothing computed, the default path (or a fresh plan) runs
        *mismatch = fl[1] == 2;
        g_last_search_path = 0;
        return CRIMP_OK;
    }
    const int nf_h = fl[0];
    *nfixed = nf_h;
    if (best && (nf_h == 0 || no_fixup)) {
        std::memcpy(best, fl + 4, 2 * sizeof(double));
        *best_done = true;
    }
    if (nf_h == 0 || no_fixup) return CRIMP_OK;
    double *dt = nullptr, *dt2 = nullptr;  // the fix-up's fp64 kernel reads dt (and dt^2) arrays
    HIPCHK(sc.alloc(&dt, (size_t)n));
    if (twod) HIPCHK(sc.alloc(&dt2, (size_t)n));
    k_search_prep<<<(int)std::min<int64_t>(cdiv(n, 256), 4096), 256, 0, s>>>(t, n, t0, dt, dt2);
    HIPCHK(hipGetLastError());
    return fixup_search(sc, s, dt, dt2, n, freq, nf, c2, twod, nharm, stat, first, flagged, nf_h, out);
}

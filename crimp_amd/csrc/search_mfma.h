// search_mfma.h -- factorised periodicity search on the fp32 matrix cores (MI355X / gfx950).
//
// For a trial grid that is an arithmetic progression f_j = f_0 + j*delta (within 16 ulp), a tile
// of 1024 consecutive trials j = c0 + a + 32*b (a, b in 0..31) factorises:
//     exp(2*pi*i*k*f_j*dt) = U_a * V_b,  U_a = exp(2*pi*i*k*(f_{c0+a}*dt + c2*dt^2)),
//                                         V_b = exp(2*pi*i*k*(32*b*delta)*dt),
// so the harmonic sums over photons are a complex matrix product
//     C_ab + i S_ab = sum_i U_ai V_bi,
// computed as two real 32x32x2 f32 MFMAs per photon and harmonic (K=2 = the (re, im) pair):
//     Re = [Ur, -Ui] . [Vr; Vi],   Im = [Ui, Ur] . [Vr; Vi].
// U and V cost 64 sin/cos per photon per wave instead of 1024 for the direct kernel; the phases
// are fp64 and reduced to a centred fractional cycle before the fp32 sin/cos, the MFMA chain
// accumulates kMfmaChunk photons in fp32 (exact fp32 fma chain) before folding into fp64.
// One wave owns one tile and one photon range (split); results go to the same part[] layout as
// the direct kernel, so k_search_finalize forms Z^2 / H.
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kMfmaChunk = 32;
constexpr int kTile = 1024;

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
    const bool hi = lane >= 32;
    int64_t ca = c0 + a;
    ca = ca < nf ? ca : nf - 1;
    const double fa = freq[ca];
    const double gb = (double)(32 * a) * delta;
    const double c2 = TWOD ? c2row[frow] : 0.0;
    const double kf = (double)k0;
    const int64_t split = blockIdx.y;
    const int64_t i0 = split * chunk;
    const int64_t i1 = i0 + chunk < n ? i0 + chunk : n;

    double Cr[G][16], Ci[G][16];
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
        for (int r = 0; r < 16; ++r) Cr[g][r] = Ci[g][r] = 0.0;

    for (int64_t ib = i0; ib < i1; ib += kMfmaChunk) {
        f32x16 re[G], im[G];
#pragma unroll
        for (int g = 0; g < G; ++g) {
#pragma unroll
            for (int r = 0; r < 16; ++r) re[g][r] = im[g][r] = 0.0f;
        }
        const int64_t ie = ib + kMfmaChunk < i1 ? ib + kMfmaChunk : i1;
        for (int64_t i = ib; i < ie; ++i) {
            const double d = dt[i];
            const double phu1 = TWOD ? fma(fa, d, c2 * dt2[i]) : fa * d;
            const double phv1 = gb * d;
            float su1, cu1, sv1, cv1;
            sincos_rev_poly((float)(phu1 - rint(phu1)), su1, cu1);
            sincos_rev_poly((float)(phv1 - rint(phv1)), sv1, cv1);
            float su, cu, sv, cv;
            if (FIRST) {
                su = su1; cu = cu1; sv = sv1; cv = cv1;
            } else {
                const double phu = phu1 * kf, phv = phv1 * kf;
                sincos_rev_poly((float)(phu - rint(phu)), su, cu);
                sincos_rev_poly((float)(phv - rint(phv)), sv, cv);
            }
#pragma unroll
            for (int g = 0; g < G; ++g) {
                const float bop = hi ? sv : cv;
                const float are = hi ? -su : cu;
                const float aim = hi ? cu : su;
                re[g] = __builtin_amdgcn_mfma_f32_32x32x2f32(are, bop, re[g], 0, 0, 0);
                im[g] = __builtin_amdgcn_mfma_f32_32x32x2f32(aim, bop, im[g], 0, 0, 0);
                if (g + 1 < G) {  // next harmonic by angle addition with the fundamental
                    const float cun = __builtin_fmaf(cu, cu1, -su * su1);
                    su = __builtin_fmaf(su, cu1, cu * su1);
                    cu = cun;
                    const float cvn = __builtin_fmaf(cv, cv1, -sv * sv1);
                    sv = __builtin_fmaf(sv, cv1, cv * sv1);
                    cv = cvn;
                }
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
        const int ra = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
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

static int g_num_cus = 0;
static int num_cus() {
    if (g_num_cus == 0) {
        int dev = 0;
        hipDeviceProp_t p;
        if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&p, dev) == hipSuccess)
            g_num_cus = p.multiProcessorCount;
        if (g_num_cus <= 0) g_num_cus = 256;
    }
    return g_num_cus;
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

    const int64_t tpr = cdiv(nf, kTile);
    const int64_t last = first + count - 1;
    const int64_t tf = (first / nf) * tpr + (first % nf) / kTile;
    const int64_t tl = (last / nf) * tpr + (last % nf) / kTile;
    const int64_t nt = tl - tf + 1;
    // photon splits: fill the resident wave slots (2 waves/SIMD at this kernel's VGPR budget) in
    // as few rounds as possible
    const int64_t slots = (int64_t)num_cus() * 4 * 2;
    int64_t best_s = 1;
    double best_cost = 1e300;
    for (int64_t sp = 1; sp <= 16; ++sp) {
        if (sp > 1 && cdiv(n, sp) < 256) break;
        const double cost = (double)cdiv(nt * sp, slots) / (double)sp;
        if (cost < best_cost - 1e-12) {
            best_cost = cost;
            best_s = sp;
        }
    }
    int64_t chunk = cdiv(cdiv(n, best_s), kMfmaChunk) * kMfmaChunk;
    const int64_t splits = cdiv(n, chunk);
    const int ncomp = 2 * nharm;
    double* part = nullptr;
    e = sc.alloc(&part, (size_t)(splits * ncomp * count));
    if (e != hipSuccess) return set_err(CRIMP_ERR_HIP, std::string("mfma_search alloc: ") + hipGetErrorString(e));
    dim3 grid((unsigned)cdiv(nt, 4), (unsigned)splits);
    for (int k0 = 1; k0 <= nharm;) {
        // groups {1,2}, {3}, {4,5}, {6,7}, {8,9}, ...: never reach k = 0 (mod 4) by angle addition
        // from the fundamental (see direct_group in crimp_hip.hip)
        const int G = ((nharm - k0 + 1) >= 2 && (k0 & 3) != 3) ? 2 : 1;
        if (twod)
            launch_mfma<true>(G, k0 == 1, grid, s, dt, dt2, n, chunk, freq, nf, c2, delta, tf, nt, tpr, first, count, k0,
                              ncomp, part);
        else
            launch_mfma<false>(G, k0 == 1, grid, s, dt, dt2, n, chunk, freq, nf, c2, delta, tf, nt, tpr, first, count,
                               k0, ncomp, part);
        e = hipGetLastError();
        if (e != hipSuccess) return set_err(CRIMP_ERR_HIP, std::string("k_search_mfma: ") + hipGetErrorString(e));
        k0 += G;
    }
    k_search_finalize<<<(unsigned)cdiv(count, 256), 256, 0, s>>>(part, count, (int)splits, nharm, stat, (double)n,
                                                               out);
    e = hipGetLastError();
    if (e != hipSuccess) return set_err(CRIMP_ERR_HIP, std::string("finalize: ") + hipGetErrorString(e));
    return 1;
}

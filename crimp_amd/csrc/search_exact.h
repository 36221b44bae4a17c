// search_exact.h -- the default periodicity-search kernel: factorised harmonic sums on the i8 matrix cores
// with EXACT integer accumulation (MI355X / gfx950).
//
// Trial grid: an arithmetic progression f_j = f_0 + j*delta (fd-outer rows for the 2-D grid). A tile of
// 1024 trials j = c0 + 32a + b (a, b in 0..31) factorises (periodsearch.py:67, :93-98, :120):
//     exp(2 pi i k (f_j dt + c2 dt^2)) = U_a * V_b,   U_a = exp(2 pi i k (f_{c0+32a} dt + c2 dt^2)),
//                                                   V_b = exp(2 pi i k (b delta) dt),
// so C_k + i S_k of the tile is the complex matrix product sum_photons U_a V_b.
//
// Numerics (why this is the default): the phase is fp64 (as the reference's argument), reduced to table
// units t = phase * kExTab turns; cos/sin come from a 4096-entry LDS table of fp64 values plus a short
// fp32 rotation by the residual angle (|theta| <= pi/4096), and are emitted directly as 2^30 fixed-point
// integers (error <= ~1.3 units = 1.2e-9). Each integer is split into four balanced base-256 digits
// (d3 2^24 + d2 2^16 + d1 2^8 + d0, d_i in [-128, 127], |d3| <= 64) packed in one dword by two
// integer ops: digits(y) = (y + 0x808080) ^ 0x808080. A product U.V = sum_{i,j} d_i e_j 2^{8(i+j)} is
// accumulated per digit LEVEL L = i+j on v_mfma_i32_32x32x32_i8 in int32 (exact), levels 3..6
// kept (the dropped levels 0..2 contribute < 5e-14 per photon): the A operand holds U's digits in natural
// order, the B operand V's digits byte-reversed, so one dword pair dots to level 3, and A >> 8, >> 16,
// >> 24 give levels 4, 5, 6 against the same B. The level sums are folded into int64 running sums in units
// of 2^-36 (acc3 + acc4 << 8 + acc5 << 16 + acc6 << 24, exact) every kExFold chunks -- kept per lane in global
// scratch between folds, so that the photon loop has the registers for both accumulators and operands --, and each block adds
// its int64 totals to the global per-trial totals with 64-bit integer atomics: integer sums are exact and
// order-independent, so the result does not depend on photon splits, trial blocking or sharding, and the
// only errors are the 2^30 roundings of U and V (per-term ~1e-9, against ~1e-7 for fp32 sin/cos).
//
// Layout: one 512-thread block (8 waves, one 1024-trial tile per wave) per group of 8 consecutive tiles
// and photon split. Per chunk of 32 photons the block stages dt in LDS, all 512 threads compute the
// tile-independent V digits once for the 8 tiles (32 photons x 32 b, stored [photon][b] as
// {rev Vr, rev -Vi, rev Vi, rev Vr}), and every wave computes its own U digits in registers; lane
// (a, h) holds photons 4q+2h, 4q+2h+1 of quad q ({Ur, Ui} of each: 16 bytes = the K slice of one
// i8 MFMA), so one quad costs 8 MFMAs (4 levels x Re/Im). V and dt are double/triple buffered so
// that the producers of chunk c+1 run beside the MFMAs of chunk c with one barrier per chunk.
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));

constexpr int kExTab = 4096;    // sin/cos table entries per turn
constexpr int kExChunk = 64;    // photons per LDS chunk (one barrier per chunk)
constexpr int kExWaves = 8;     // waves (tiles) per block
constexpr int kExBlock = 64 * kExWaves;
// int32 headroom per photon and level (balanced digits, |top digit| <= 64): level 3 <= 2 x 49152, level 4
// <= 2 x 32768, level 5 <= 2 x 16384, level 6 <= 2 x 4096. Every kExCarry chunks (16384 photons: level 3
// reaches 1.61e9 < 2^31) the level sums are carried upward exactly (acc_L = 256 q + r, r in [0, 255]:
// acc_L <- r, acc_{L+1} += q), which leaves level 6 growing by <= 2^27 per period; every kExFold chunks
// (131072 photons, 8 periods: level 6 < 2^30 + carries) they are folded into the int64 running sums.
constexpr int kExCarry = 16384 / kExChunk;
constexpr int kExFold = 131072 / kExChunk;
constexpr int kExFoldVals = 32;             // int64 running sums per lane (16 result rows x Re, Im)
constexpr double kExUnit = 1.4551915228366852e-11;  // 2^-36: value of one unit of the int64 totals

struct ExEntry {
    int32_t sk, ck;  // rint(sin, cos(2 pi k / T) * 2^30) + 0x808080 - 0x4B400000: the fp32 rounding bias of ex_end and
                     // the digit bias of ex_digits folded in
    float s1, c1;    // sin, cos(2 pi k / T) * 2^30 * (2 pi / T): the residual rotation's first-order coefficients
};

// t in table units (turns * kExTab) -> the digit dwords of (cos, sin) * 2^30 (ex_digits of the rounded integers),
// in two halves so that the table read of one photon can be issued ahead of the arithmetic of another.
// x = 2 pi (k + y) / T, |y| <= 1/2: sin x = s_k + c_k sin(th) + s_k (cos(th) - 1) with th = 2 pi y / T, and to
// 2^30 units  sin x * 2^30 = S_k + y (C1 - u S1),  cos x * 2^30 = C_k - y (S1 + u C1),  u = (pi / T) y,
// (C1, S1 = (c_k, s_k) 2^30 2 pi / T); the dropped th^3/6 term is <= 0.08 units at the cell edge.
struct ExArg {
    uint32_t idx;  // table index
    float y;       // residual in table steps, |y| <= 1/2
};
__device__ __forceinline__ ExArg ex_begin(double t) {
    const double M = 6755399441055744.0;  // 1.5 * 2^52: low mantissa bits of t + M = rint(t) (|t| < 2^51)
    const double tm = t + M;
    const double kf = tm - M;
    return ExArg{(uint32_t)__double2loint(tm) & (kExTab - 1), (float)(t - kf)};  // t - kf is exact
}
// -> digit dwords of cos (dc) and sin (ds)
__device__ __forceinline__ void ex_end(const ExEntry& e, float y, uint32_t& dc, uint32_t& ds) {
    const float u = y * (3.14159265358979323846f / (float)kExTab);
    const float ts = __builtin_fmaf(-u, e.s1, e.c1);
    const float tc = __builtin_fmaf(u, e.c1, e.s1);
    // |value| < 2^22: the low mantissa bits of fma(y, t, 1.5 * 2^23) are rint(y t) + 0x400000
    ds = ((uint32_t)e.sk + __float_as_uint(__builtin_fmaf(y, ts, 12582912.0f))) ^ 0x00808080u;
    dc = ((uint32_t)e.ck + __float_as_uint(__builtin_fmaf(-y, tc, 12582912.0f))) ^ 0x00808080u;
}
__device__ __forceinline__ void ex_sincos_digits(const ExEntry* __restrict__ tab, double t, uint32_t& dc,
                                                 uint32_t& ds) {
    const ExArg g = ex_begin(t);
    ex_end(tab[g.idx], g.y, dc, ds);
}
__device__ __forceinline__ ExEntry ex_entry(int i) {
    double s, c;
    sincospi((double)i * (2.0 / kExTab), &s, &c);
    const double w = 1073741824.0 * (6.283185307179586476925 / kExTab);
    ExEntry e;
    e.s1 = (float)(s * w);
    e.c1 = (float)(c * w);
    e.sk = (int32_t)((uint32_t)(int32_t)rint(s * 1073741824.0) + 0x00808080u - 0x4B400000u);
    e.ck = (int32_t)((uint32_t)(int32_t)rint(c * 1073741824.0) + 0x00808080u - 0x4B400000u);
    return e;
}

// digit dword of -y from the digit dword of y: -y's balanced digits are the negated digits (with carries),
// recomputed from the integer: y = (d ^ 0x808080) - 0x808080
__device__ __forceinline__ uint32_t ex_neg_digits(uint32_t d) {
    const uint32_t y = (d ^ 0x00808080u) - 0x00808080u;
    return (0x00808080u - y) ^ 0x00808080u;
}


__device__ __forceinline__ int64_t ex_level_sum(int a3, int a4, int a5, int a6) {
    return (int64_t)a3 + ((int64_t)a4 << 8) + ((int64_t)a5 << 16) + ((int64_t)a6 << 24);
}

template <bool TWOD>
__global__ __launch_bounds__(kExBlock, 2) void k_search_exact(
    const double* __restrict__ dt, const double* __restrict__ dt2, int64_t n, int64_t chunk,
    const double* __restrict__ freq, int64_t nf, const double* __restrict__ c2row, const double* __restrict__ apinfo,
    int64_t tile_first, int64_t ntiles, int64_t tiles_per_row, int64_t first, int64_t count, int kh,
    unsigned long long* __restrict__ tot, long long* __restrict__ fold) {
    __shared__ ExEntry tab[kExTab];                        // 64 KB
    __shared__ uint4 vre[2][kExChunk / 2][32];             // B fragments (Re) per photon pair and column b
    __shared__ uint4 vim[2][kExChunk / 2][32];             // B fragments (Im)
    __shared__ double sdt[3][kExChunk];
    __shared__ double sdt2[TWOD ? 3 : 1][kExChunk];
    const int tid = threadIdx.x;
    const int lane = tid & 63, wv = tid >> 6;
    for (int i = tid; i < kExTab; i += kExBlock) tab[i] = ex_entry(i);
    const double kT = (double)kh * (double)kExTab;
    const int64_t T = (int64_t)blockIdx.x * kExWaves + wv;  // this wave's tile; waves past the end only produce V
    const bool active = T < ntiles;                          // wave-uniform
    const int64_t gt = tile_first + (active ? T : 0);
    const int64_t frow = gt / tiles_per_row;
    const int64_t c0 = (gt - frow * tiles_per_row) * 1024;
    const int ar = lane & 31, h = lane >> 5;
    const int64_t ca = c0 + 32 * ar;
    const double fa = freq[ca < nf ? ca : nf - 1] * kT;
    const double c2 = TWOD ? c2row[frow] * kT : 0.0;
    const int pb = tid & 31;                                  // producer: V_b for b = pb, photons (tid >> 5) + 16 s
    const double gbv = (double)pb * apinfo[0] * kT;
    const int64_t split = blockIdx.y;
    const int64_t i0 = split * chunk;
    const int64_t i1 = i0 + chunk < n ? i0 + chunk : n;
    const int nch = (int)((i1 - i0 + kExChunk - 1) / kExChunk);

    auto load_dt = [&](int c, int slot) {
        if (tid < kExChunk) {
            const int64_t i = i0 + (int64_t)c * kExChunk + tid;
            const bool ok = c < nch && i < i1;
            sdt[slot][tid] = ok ? dt[i] : 0.0;
            if (TWOD) sdt2[TWOD ? slot : 0][tid] = ok ? dt2[i] : 0.0;
        }
    };
    // V digits of chunk c as B fragments; photons past the split get V = 0, so that their products vanish
    // one store address per thread: item s writes photon pp + 16 s, i.e. pair (pp >> 1) + 8 s (an immediate
    // offset), half pp & 1 of the pair's uint4
    const int pp = tid >> 5;
    uint2* const wre = reinterpret_cast<uint2*>(&vre[0][pp >> 1][pb]) + (pp & 1);
    uint2* const wim = reinterpret_cast<uint2*>(&vim[0][pp >> 1][pb]) + (pp & 1);
    constexpr int kPairU2 = 32 * 2;                    // uint2 per photon pair row of 32 columns
    constexpr int kBufU2 = (kExChunk / 2) * kPairU2;   // uint2 per buffer
    auto produce_items = [&](int slot, int vb, int nlive, bool masked) {
#pragma unroll
        for (int s = 0; s < kExChunk * 32 / kExBlock; ++s) {
            const int p = pp + (kExBlock / 32) * s;
            uint32_t dc, dsn;
            ex_sincos_digits(tab, gbv * sdt[slot][p], dc, dsn);
            uint32_t rc = __builtin_bswap32(dc), rs = __builtin_bswap32(dsn),
                     rn = __builtin_bswap32(ex_neg_digits(dsn));
            if (masked && p >= nlive) rc = rs = rn = 0u;
            wre[vb * kBufU2 + s * 8 * kPairU2] = make_uint2(rc, rn);
            wim[vb * kBufU2 + s * 8 * kPairU2] = make_uint2(rs, rc);
        }
    };
    auto produce = [&](int c, int slot, int vb) {
        const int64_t rest = i1 - (i0 + (int64_t)c * kExChunk);
        if (rest >= kExChunk)
            produce_items(slot, vb, kExChunk, false);  // every chunk but a split's last: no masks
        else
            produce_items(slot, vb, (int)rest, true);
    };
    auto uphase = [&](int ds, int p) -> double {
        return TWOD ? fma(fa, sdt[ds][p], c2 * sdt2[TWOD ? ds : 0][p]) : fa * sdt[ds][p];
    };

    i32x16 acc[4][2];
#pragma unroll
    for (int L = 0; L < 4; ++L)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[L][0][r] = acc[L][1][r] = 0;
    // the block's running int64 sums between folds: per lane in global scratch (coalesced, written and read
    // by the same lane), so that they take no registers inside the photon loop
    long long* const fs =
        fold + (((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * kExWaves + wv) * (kExFoldVals * 64) + lane;
    const int comp = 2 * (kh - 1);

    load_dt(0, 0);
    load_dt(1, 1);
    __syncthreads();  // table + first two dt chunks
    produce(0, 0, 0);
    __syncthreads();
    for (int c = 0; c < nch; ++c) {
        const int ds = c % 3, vb = c & 1;
        load_dt(c + 2, (c + 2) % 3);
        if (c + 1 < nch) produce(c + 1, (c + 1) % 3, vb ^ 1);
        if (active) {
#pragma unroll 2
            for (int q = 0; q < kExChunk / 4; ++q) {
                const int p0 = 4 * q + 2 * h;
                uint32_t a0, a1, a2, a3;
                ex_sincos_digits(tab, uphase(ds, p0), a0, a1);
                ex_sincos_digits(tab, uphase(ds, p0 + 1), a2, a3);
                const uint4 br = vre[vb][2 * q + h][ar], bi = vim[vb][2 * q + h][ar];
                const i32x4 bre = {(int)br.x, (int)br.y, (int)br.z, (int)br.w};
                const i32x4 bim = {(int)bi.x, (int)bi.y, (int)bi.z, (int)bi.w};
                i32x4 A[4];
#pragma unroll
                for (int L = 0; L < 4; ++L) {
                    const int sh = 8 * L;
                    A[L] = i32x4{(int)(a0 >> sh), (int)(a1 >> sh), (int)(a2 >> sh), (int)(a3 >> sh)};
                }
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int L = 0; L < 4; ++L) {
                    acc[L][0] = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[L], bre, acc[L][0], 0, 0, 0);
                    acc[L][1] = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[L], bim, acc[L][1], 0, 0, 0);
                }
                mfma_operand_guard();
            }
            const bool fold_now = (c + 1) % kExFold == 0 || c + 1 == nch;
            if (!fold_now && (c + 1) % kExCarry == 0) {
                mfma_drain();
#pragma unroll
                for (int r = 0; r < 16; ++r)
#pragma unroll
                    for (int x = 0; x < 2; ++x)
#pragma unroll
                        for (int L = 0; L < 3; ++L) {
                            const int q = acc[L][x][r] >> 8;  // floor division by 256
                            acc[L][x][r] &= 255;
                            acc[L + 1][x][r] += q;
                        }
            }
            if (fold_now) {
                mfma_drain();
                const bool first_fold = c + 1 <= kExFold, last = c + 1 == nch;
                // opaque copies of the lane's scratch pointer and trial index: the 32 addresses derived from them
                // must be formed here, not hoisted out of the photon loop (they would hold 64 registers there)
                long long* f = fs;
                int64_t cl = c0 + ar - first + frow * nf;
                asm volatile("" : "+v"(f), "+v"(cl));
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    long long re = ex_level_sum(acc[0][0][r], acc[1][0][r], acc[2][0][r], acc[3][0][r]);
                    long long im = ex_level_sum(acc[0][1][r], acc[1][1][r], acc[2][1][r], acc[3][1][r]);
                    if (!first_fold) {
                        re += f[r * 64];
                        im += f[(16 + r) * 64];
                    }
                    if (!last) {
                        f[r * 64] = re;
                        f[(16 + r) * 64] = im;
                    } else {
                        // D[row a][col b] of the 32x32 tile: col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 h;
                        // trial c0 + 32 a + b, output slot o = frow * nf + trial - first
                        const int ra = (r & 3) + 8 * (r >> 2) + 4 * h;
                        const int64_t o = cl + 32 * ra;
                        if (c0 + 32 * ra + ar < nf && o >= 0 && o < count) {
                            atomicAdd(&tot[(int64_t)comp * count + o], (unsigned long long)re);
                            atomicAdd(&tot[(int64_t)(comp + 1) * count + o], (unsigned long long)im);
                        }
                    }
                }
#pragma unroll
                for (int L = 0; L < 4; ++L)
#pragma unroll
                    for (int r = 0; r < 16; ++r) acc[L][0][r] = acc[L][1][r] = 0;
            }
        }
        __syncthreads();
    }
}

// Statistic from the exact totals (periodsearch.py:67-69 and :120-123 in the reference's formula order), and
// the fix-up list: trials whose power is too small for the kernel's error bound to guarantee 1e-6 relative.
// Error model: per term of U.V (2^30 roundings of both factors, fp32 residual rotation) |e| <= 3e-9, rms <= 1e-9,
// independent across photons and harmonics, so C_k and S_k carry errors of standard deviation
// sc = sqrt(N) 1e-9 and Z2_k = (2/N)(C^2 + S^2) one of (4/N) sc sqrt(C^2 + S^2) (+ (2/N) 2 sc^2 bias). A sum of
// harmonics i <= k (Z2, and H's cumulative g_k = sum_{i<=k} Z2_i - 4(k-1)) has standard deviation
// (4/N) sc sqrt(sum_{i<=k} (C_i^2 + S_i^2)); the bound is kappa = 10 of them plus the bias. H = max_k g_k moves
// by at most the bound of any g_k that can reach the maximum (g_k + err_k >= H - err_k*), so only those count.
__global__ __launch_bounds__(256) void k_search_finalize_exact(const long long* __restrict__ tot, int64_t count, int m,
                                                               int stat, double n, double sc, double rel, int64_t tbase,
                                                               double* __restrict__ out, int* __restrict__ nflag,
                                                               int64_t* __restrict__ flagged) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= count) return;
    const double w = 2.0 / n, kappa = 10.0;
    const double lin = kappa * 2.0 * w * sc, quad = w * 2.0 * (kappa * sc) * (kappa * sc);
    auto zk = [&](int k) {
        const double c = (double)tot[(int64_t)(2 * k) * count + t] * kExUnit;
        const double s = (double)tot[(int64_t)(2 * k + 1) * count + t] * kExUnit;
        return c * c + s * s;
    };
    double p, err;
    if (stat == CRIMP_STAT_Z2) {
        double zsum = 0.0;
        for (int k = 0; k < m; ++k) zsum += zk(k);
        p = zsum * w;
        err = lin * sqrt(zsum) + m * quad;
    } else {
        double cum = 0.0, raw = 0.0, best = -INFINITY, ebest = 0.0;
        for (int k = 0; k < m; ++k) {
            const double z = zk(k);
            cum += z * w;
            raw += z;
            const double v = cum - 4.0 * (double)k;
            if (v > best) {
                best = v;
                ebest = lin * sqrt(raw) + (k + 1) * quad;
            }
        }
        p = best;
        err = ebest;
        cum = 0.0;
        raw = 0.0;
        for (int k = 0; k < m; ++k) {  // every g_k that the errors could lift to the maximum
            const double z = zk(k);
            cum += z * w;
            raw += z;
            const double ek = lin * sqrt(raw) + (k + 1) * quad;
            if (cum - 4.0 * (double)k + ek >= best - ebest) err = fmax(err, ek);
        }
    }
    out[t] = p;
    if (!(err <= rel * fabs(p))) flagged[atomicAdd(nflag, 1)] = tbase + t;
}

// arithmetic-progression check on the device: |f_j - (f_0 + j delta)| <= 16 ulp(max|f|), delta from the ends.
// info[0] = delta, info[1] = max deviation (as bits: non-negative doubles order as integers), info[2] = max |f|.
__global__ __launch_bounds__(256) void k_ap_check(const double* __restrict__ f, int64_t nf,
                                                  unsigned long long* __restrict__ info) {
    const double d = (f[nf - 1] - f[0]) / (double)(nf - 1);
    double dev = 0.0, fm = 0.0;
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < nf; j += (int64_t)gridDim.x * blockDim.x) {
        dev = fmax(dev, fabs(f[j] - (f[0] + (double)j * d)));
        fm = fmax(fm, fabs(f[j]));
    }
    for (int o = 32; o > 0; o >>= 1) {
        dev = fmax(dev, __shfl_xor(dev, o));
        fm = fmax(fm, __shfl_xor(fm, o));
    }
    if ((threadIdx.x & 63) == 0) {
        atomicMax(&info[1], (unsigned long long)__double_as_longlong(dev));
        atomicMax(&info[2], (unsigned long long)__double_as_longlong(fm));
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) info[0] = (unsigned long long)__double_as_longlong(d);
}

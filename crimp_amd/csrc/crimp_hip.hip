// crimp_hip.hip -- MI355X (gfx950) kernels + C-ABI for CRIMP's photon hot path.
//
// Entry points are declared (with the reference routine each replaces) in
// include/crimp_hip.h. Layout of this file:
//   1. runtime helpers (errors, stream-ordered scratch, staging of host buffers)
//   2. fp32 sin/cos in revolutions (polynomial and hardware v_sin/v_cos)
//   3. calcphase            -- HBM-bound fp64 phase folding
//   4. periodicity search   -- exact i8-MFMA kernel (search_exact.h, default), NUFFT (search_nufft.h,
//                              opt-in), fp64 kernel, finalize
//   5. ToA likelihood scan  -- fp64 point evaluator, fp32 brute grid, binning
//   6. C-ABI
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <chrono>
#include <functional>
#include <vector>

#include "../../include/crimp_hip.h"

#define CRIMP_VERSION 2

// ============================================================== 1. runtime helpers
static thread_local std::string g_err;
static std::mutex g_mutex;

// CRIMP_FLAG_TIME_KERNELS: hipEvents around the timed spans of the last call (ms): the harmonic-sum kernels of a
// search, the calcphase kernel, the brute-grid and the fit kernels of crimp_toa_fit
static double g_last_kernel_ms = -1.0;
static std::vector<double> g_kernel_times;
// trials of the last crimp_search recomputed by the fp64 fix-up (exact path)
static int64_t g_last_fixups = 0;
static int64_t g_last_grid_norms = 0;  // brute-grid norms evaluated per phShift by the last crimp_toa_fit
static int64_t g_last_grid_fast = 0;   // the last crimp_toa_fit's brute-grid mode (kGridNoMin | kGridProd8 bits)
struct KernelTimer {
    hipEvent_t a = nullptr, b = nullptr;
    hipStream_t s;
    bool on;
    KernelTimer(hipStream_t st, bool enable) : s(st), on(enable) {
        if (on && (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess)) on = false;
    }
    void start() {
        if (on) (void)hipEventRecord(a, s);
    }
    void stop() {
        if (!on) return;
        (void)hipEventRecord(b, s);
        float ms = -1.0f;
        if (hipEventSynchronize(b) == hipSuccess && hipEventElapsedTime(&ms, a, b) == hipSuccess) {
            if (g_kernel_times.empty()) g_last_kernel_ms = ms;
            g_kernel_times.push_back(ms);
        }
    }
    ~KernelTimer() {
        if (a) (void)hipEventDestroy(a);
        if (b) (void)hipEventDestroy(b);
    }
};

static int set_err(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define HIPCHK(expr)                                                                               \
    do {                                                                                           \
        hipError_t e_ = (expr);                                                                    \
        if (e_ != hipSuccess)                                                                      \
            return set_err(CRIMP_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));     \
    } while (0)

#define ARGCHK(cond, msg)                                                                          \
    do {                                                                                           \
        if (!(cond)) return set_err(CRIMP_ERR_ARG, msg);                                           \
    } while (0)

// CRIMP_DEBUG=1: poison every scratch allocation with 0xFF (NaN) bytes before use.
static int debug_level() {
    static int lvl = -1;
    if (lvl < 0) {
        const char* e = getenv("CRIMP_DEBUG");
        lvl = e ? atoi(e) : 0;
    }
    return lvl;
}

// Device scratch: a small caching allocator (hipMalloc'd blocks reused across calls). Every
// entry point synchronises its stream before returning and calls are serialised by g_mutex, so
// a block handed back at the end of a call is idle when the next call takes it. The idle blocks
// of a device are freed when hipMalloc fails (then the allocation is retried once) or when the
// cached bytes would pass CRIMP_SCRATCH_CAP_MB (default 8192), and by crimp_release_scratch().
struct Block {
    void* p;
    size_t bytes;
    int dev;
    bool busy;
};
static std::vector<Block> g_blocks;

static size_t scratch_cap_bytes() {
    static size_t cap = 0;
    if (cap == 0) {
        const char* e = getenv("CRIMP_SCRATCH_CAP_MB");
        const long long mb = e ? atoll(e) : 8192;
        cap = (size_t)(mb > 0 ? mb : 8192) << 20;
    }
    return cap;
}

// frees the idle blocks of device `dev` (all devices for dev < 0)
static void release_idle_blocks(int dev) {
    std::vector<Block> keep;
    for (const Block& b : g_blocks) {
        if (!b.busy && (dev < 0 || b.dev == dev)) {
            (void)hipFree(b.p);
        } else {
            keep.push_back(b);
        }
    }
    g_blocks.swap(keep);
}

struct Scratch {
    hipStream_t s;
    int dev = 0;
    std::vector<void*> held;
    explicit Scratch(hipStream_t st) : s(st) { (void)hipGetDevice(&dev); }
    ~Scratch() {
        // an error return may leave kernels of this call queued on the stream: drain it before the blocks
        // they may still write become reusable (a no-op on the normal path, which returns drained)
        if (!held.empty()) (void)hipStreamSynchronize(s);
        for (void* p : held)
            for (Block& b : g_blocks)
                if (b.p == p) b.busy = false;
    }
    template <typename T>
    hipError_t alloc(T** out, size_t count) {
        const size_t bytes = (std::max<size_t>(count * sizeof(T), 16) + 255) & ~size_t(255);
        size_t pick = (size_t)-1, cached = 0;
        for (size_t i = 0; i < g_blocks.size(); ++i) {
            const Block& b = g_blocks[i];
            cached += b.bytes;
            if (!b.busy && b.dev == dev && b.bytes >= bytes && b.bytes <= 2 * bytes + (1u << 20) &&
                (pick == (size_t)-1 || b.bytes < g_blocks[pick].bytes))
                pick = i;
        }
        if (pick == (size_t)-1) {
            if (cached + bytes > scratch_cap_bytes()) release_idle_blocks(dev);
            void* p = nullptr;
            hipError_t e = hipMalloc(&p, bytes);
            if (e != hipSuccess) {
                (void)hipGetLastError();
                release_idle_blocks(dev);
                e = hipMalloc(&p, bytes);
                if (e != hipSuccess) return e;
            }
            g_blocks.push_back(Block{p, bytes, dev, false});
            pick = g_blocks.size() - 1;
        }
        g_blocks[pick].busy = true;
        held.push_back(g_blocks[pick].p);
        *out = static_cast<T*>(g_blocks[pick].p);
        if (debug_level() > 0) return hipMemset(g_blocks[pick].p, 0xFF, g_blocks[pick].bytes);
        return hipSuccess;
    }
};

// Host staging uses blocking copies: inputs are copied before any kernel of the call is queued,
// outputs after the stream has drained.
template <typename T>
static hipError_t stage_in(Scratch& sc, const T* src, size_t count, bool dev, const T** out) {
    if (dev || src == nullptr || count == 0) {
        *out = src;
        return hipSuccess;
    }
    T* d = nullptr;
    hipError_t e = sc.alloc(&d, count);
    if (e != hipSuccess) return e;
    *out = d;
    return hipMemcpy(d, src, count * sizeof(T), hipMemcpyHostToDevice);
}

template <typename T>
static hipError_t stage_out(Scratch& sc, T* dst, size_t count, bool dev, T** out) {
    if (dev || dst == nullptr) {
        *out = dst;
        return hipSuccess;
    }
    return sc.alloc(out, count);
}

template <typename T>
static hipError_t copy_back(hipStream_t s, T* host, const T* devp, size_t count, bool dev) {
    if (dev || host == nullptr || count == 0) return hipSuccess;
    hipError_t e = hipStreamSynchronize(s);
    if (e != hipSuccess) return e;
    return hipMemcpy(host, devp, count * sizeof(T), hipMemcpyDeviceToHost);
}

// blocking host <-> device copies of small host-side tables
static hipError_t h2d(void* d, const void* h, size_t bytes) { return hipMemcpy(d, h, bytes, hipMemcpyHostToDevice); }

// Page-locked staging of a call's small host->device uploads (crimp_toa_fit: template, lattice, candidate norms,
// certificate masks): copied into one hipHostMalloc'd buffer and queued with hipMemcpyAsync on the call's stream, so
// the host does not wait for each pageable copy (~290 us of setup before the first kernel, profiles/r04). Calls are
// serialised by g_mutex and drain their stream before returning, so the buffer is free again at the next call.
struct PinnedStage {
    char* p = nullptr;
    size_t cap = 0, used = 0;
};
static PinnedStage g_pin;
static void pin_begin(size_t bytes) {
    g_pin.used = 0;
    if (g_pin.cap >= bytes || bytes > (size_t(64) << 20)) return;  // (huge batches: the blocking copies past the cap)
    if (g_pin.p) (void)hipHostFree(g_pin.p);
    g_pin.p = nullptr;
    g_pin.cap = 0;
    const size_t cap = std::max<size_t>(bytes, size_t(1) << 20);
    if (hipHostMalloc(reinterpret_cast<void**>(&g_pin.p), cap, hipHostMallocDefault) != hipSuccess) {
        (void)hipGetLastError();
        g_pin.p = nullptr;  // no staging: h2d_async falls back to the blocking copy
        return;
    }
    g_pin.cap = cap;
}
static hipError_t h2d_async(hipStream_t s, void* d, const void* h, size_t bytes) {
    const size_t need = (bytes + 255) & ~size_t(255);
    if (!g_pin.p || g_pin.used + need > g_pin.cap) return h2d(d, h, bytes);
    char* q = g_pin.p + g_pin.used;
    g_pin.used += need;
    std::memcpy(q, h, bytes);
    return hipMemcpyAsync(d, q, bytes, hipMemcpyHostToDevice, s);
}
// Device -> host after the stream's queued work. Small reads (flags, counts, grid scalars: the routing readbacks
// of a search) go through a page-locked per-thread buffer with one async copy and one stream sync: a blocking
// pageable hipMemcpy of a few bytes after the sync cost ~30 us per readback (rocprofv3 sys-trace, profiles/r05).
static hipError_t d2h(hipStream_t s, void* h, const void* d, size_t bytes) {
    constexpr size_t kSmall = 4096;
    thread_local void* pin = nullptr;
    if (bytes <= kSmall) {
        if (!pin && hipHostMalloc(&pin, kSmall, hipHostMallocDefault) != hipSuccess) {
            (void)hipGetLastError();
            pin = nullptr;
        }
        if (pin) {
            hipError_t e = hipMemcpyAsync(pin, d, bytes, hipMemcpyDeviceToHost, s);
            if (e == hipSuccess) e = hipStreamSynchronize(s);
            if (e != hipSuccess) return e;
            std::memcpy(h, pin, bytes);
            return hipSuccess;
        }
    }
    hipError_t e = hipStreamSynchronize(s);
    if (e != hipSuccess) return e;
    return hipMemcpy(h, d, bytes, hipMemcpyDeviceToHost);
}

static inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// ============================================================== 2. sin/cos in revolutions
// r in [-0.5, 0.5] revolutions -> sin(2*pi*r), cos(2*pi*r).
// Polynomial form: quarter-turn reduction y = r - q/4 (exact), |y| <= 1/8, Taylor series of
// sin/cos(2*pi*y) to degree 9/10 (truncation < 2e-9), then an exact quadrant rotation.
__device__ __forceinline__ void sincos_rev_poly(float r, float& s, float& c) {
    const float q = __builtin_rintf(4.0f * r);
    const float y = __builtin_fmaf(-0.25f, q, r);
    const float y2 = y * y;
    const float S1 = 6.28318530717958647692f, S3 = -41.3417022403997f, S5 = 81.6052492760750f,
                S7 = -76.7058597530613f, S9 = 42.0587782776566f;
    const float C2 = -19.7392088021787f, C4 = 64.9393940226683f, C6 = -85.4568172844813f,
                C8 = 60.2446397079094f, C10 = -26.4262625987960f;
    float sp = __builtin_fmaf(y2, S9, S7);
    sp = __builtin_fmaf(y2, sp, S5);
    sp = __builtin_fmaf(y2, sp, S3);
    sp = __builtin_fmaf(y2, sp, S1);
    sp *= y;
    float cp = __builtin_fmaf(y2, C10, C8);
    cp = __builtin_fmaf(y2, cp, C6);
    cp = __builtin_fmaf(y2, cp, C4);
    cp = __builtin_fmaf(y2, cp, C2);
    cp = __builtin_fmaf(y2, cp, 1.0f);
    const int iq = ((int)q) & 3;
    const float s_a = (iq & 1) ? cp : sp;
    const float c_a = (iq & 1) ? sp : cp;
    s = (iq & 2) ? -s_a : s_a;
    c = ((iq + 1) & 2) ? -c_a : c_a;
}

// ============================================================== 3. calcphase
struct CPModel {
    double pepoch;
    double coef[13];  // (1/n!) * F_{n-1}, exactly as calcphase.py:84 forms it
    int32_t nterms;   // highest n with a non-zero coefficient
    int32_t parts;
    int32_t n_glitch;
    int32_t n_wave;
    double glitch[CRIMP_MAX_GLITCH][7];
    double wave_epoch, wave_om, f0;
    double wave_ab[CRIMP_MAX_WAVE][2];
};
static_assert(sizeof(CPModel) + 64 <= 4096, "CPModel is passed by value in the kernel arguments (4 KB limit)");

__device__ __forceinline__ double cp_one(const CPModel* __restrict__ M, double t) {
    double te = 0.0;
    if (M->parts & 1) {
        // calcphase.py:80-85: te = sum_{n=1}^{13} coef_n * dt**n, summed in increasing n.
        const double dt = (t - M->pepoch) * 86400.0;
        double dn = dt;
        const int nt = M->nterms;
        for (int k = 0; k < nt; ++k) {
            te += M->coef[k] * dn;
            dn *= dt;
        }
    }
    double gl = 0.0;
    if (M->parts & 2) {
        // calcphase.py:98-124
        for (int j = 0; j < M->n_glitch; ++j) {
            const double* g = M->glitch[j];
            if (t >= g[0]) {
                const double dts = (t - g[0]) * 86400.0;
                const double ex = (g[6] == 0.0) ? 0.0 : (g[6] * 86400.0) * (1.0 - exp(-(t - g[0]) / g[6]));
                gl += (((g[1] + g[2] * dts) + (0.5 * g[3]) * (dts * dts)) + ((1.0 / 6.0) * g[4]) * (dts * dts * dts)) +
                      g[5] * ex;
            }
        }
    }
    double wv = 0.0;
    if ((M->parts & 4) && M->n_wave > 0) {
        // calcphase.py:138-149
        for (int j = 1; j <= M->n_wave; ++j) {
            const double arg = (j * M->wave_om) * (t - M->wave_epoch);
            wv += (M->wave_ab[j - 1][0] * sin(arg)) + (M->wave_ab[j - 1][1] * cos(arg));
        }
        wv *= M->f0;
    }
    return te + gl + wv;
}

// Two photons per thread, 16-byte loads and stores (24 B of HBM traffic per photon; non-temporal loads and
// stores measured the same, profiles/r1_final/ab_cos6_nt.log). One pair per thread over a
// grid that covers the array (up to 2^28 pairs per sweep): 5.5-5.6 TB/s at 1e8 photons, against 4.6-5.1 TB/s
// for a 4096-block grid-stride loop with 1, 2 or 4 loads in flight per thread (profiles/r1_s4/calcphase_ab.log).
__global__ __launch_bounds__(256) void k_calcphase_vec(const double2* __restrict__ t, int64_t npair,
                                                       const CPModel Mv, double2* __restrict__ total,
                                                       double2* __restrict__ folded, double fscale) {
    const CPModel* M = &Mv;  // the model rides in the kernel arguments (no upload, no copy to the stack)
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < npair; i += (int64_t)gridDim.x * blockDim.x) {
        const double2 tv = t[i];
        double2 tot;
        tot.x = cp_one(M, tv.x);
        tot.y = cp_one(M, tv.y);
        total[i] = tot;
        if (folded) {
            double2 fo;
            fo.x = (tot.x - floor(tot.x)) * fscale;  // fscale 1 (cycles) or 2 pi (measureToAs.py:195, :200)
            fo.y = (tot.y - floor(tot.y)) * fscale;
            folded[i] = fo;
        }
    }
}

__global__ __launch_bounds__(256) void k_calcphase_scalar(const double* __restrict__ t, int64_t n,
                                                          const CPModel Mv, double* __restrict__ total,
                                                          double* __restrict__ folded, double fscale) {
    const CPModel* M = &Mv;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const double tot = cp_one(M, t[i]);
        total[i] = tot;
        if (folded) folded[i] = (tot - floor(tot)) * fscale;
    }
}

// ============================================================== 4. periodicity search
// Three paths compute the per-trial harmonic sums C_k, S_k (periodsearch.py:67-69, :93-99, :120-121):
//   k_search_exact (search_exact.h, the default for arithmetic-progression grids): i8 MFMA, exact integer sums;
//   the NUFFT (search_nufft.h, opt-in CRIMP_FLAG_NUFFT, progressions of time-sorted photons): fp64 moments on
//                   the f64 matrix cores, fp64 FFT, fp64 Horner sums;
//   k_search_f64   (any grid; the default when the grid is not a progression or has < 256 trials, and the
//                   fix-up of trials the exact and NUFFT paths cannot certify): fp64 throughout.
// dt[i] = t[i] - t0 (periodsearch.py: self.time - self.t0); dt2 = dt*dt for the 2-D grid.
__global__ __launch_bounds__(256) void k_search_prep(const double* __restrict__ t, int64_t n, double t0,
                                                     double* __restrict__ dt, double* __restrict__ dt2) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const double d = t[i] - t0;
        dt[i] = d;
        if (dt2) dt2[i] = d * d;
    }
}

// Direct kernels: one lane per trial, every photon of its split broadcast to the wave through the scalar
// path. Trial t of the launch is flat grid index first + (tidx ? tidx[t] : t). part layout: [split][2m][count]
// (C_k at 2(k-1), S_k at 2(k-1)+1).
constexpr int kSearchBlock = 256;
constexpr int kSearchFold = 32;

__device__ __forceinline__ int64_t trial_index(const int64_t* __restrict__ tidx, int64_t first, int64_t t) {
    return first + (tidx ? tidx[t] : t);
}

// fp64 kernel: the reference's arithmetic precision end to end. fp64 phase reduced to a centred fractional
// cycle r, fp64 sincospi(2r) for harmonic k0 of the group, harmonics k0+1 .. k0+G-1 by fp64 angle addition,
// fp64 sums. Every term differs from np.cos(2*k*pi*f*(t-t0)) (periodsearch.py:67) by the fp64 rounding of the
// phase argument only.
template <int G, bool TWOD>
__global__ __launch_bounds__(kSearchBlock) void k_search_f64(
    const double* __restrict__ dt, const double* __restrict__ dt2, int64_t n, int64_t chunk,
    const double* __restrict__ freq, int64_t nf, const double* __restrict__ c2row, int64_t first,
    const int64_t* __restrict__ tidx, int64_t count, int k0, int ncomp, double* __restrict__ part) {
    const int64_t t = (int64_t)blockIdx.x * kSearchBlock + threadIdx.x;
    const int64_t split = blockIdx.y;
    const int64_t g = trial_index(tidx, first, t < count ? t : count - 1);
    const int64_t row = TWOD ? g / nf : 0;
    const double f = freq[g - row * nf];
    const double c2 = TWOD ? c2row[row] : 0.0;
    const double kf = (double)k0;
    const int64_t i0 = split * chunk;
    const int64_t i1 = i0 + chunk < n ? i0 + chunk : n;
    double C[G], S[G];
#pragma unroll
    for (int k = 0; k < G; ++k) C[k] = S[k] = 0.0;
#pragma unroll 2
    for (int64_t i = i0; i < i1; ++i) {
        const double d = dt[i];
        const double ph = TWOD ? fma(f, d, c2 * dt2[i]) : f * d;
        double s1 = 0.0, c1 = 1.0, s, c;
        if (G > 1) sincospi(2.0 * (ph - rint(ph)), &s1, &c1);
        if (k0 == 1 && G > 1) {
            s = s1;
            c = c1;
        } else {
            const double pk = ph * kf;
            sincospi(2.0 * (pk - rint(pk)), &s, &c);
        }
        C[0] += c;
        S[0] += s;
#pragma unroll
        for (int k = 1; k < G; ++k) {
            const double cn = fma(c, c1, -s * s1);
            const double sn = fma(s, c1, c * s1);
            c = cn;
            s = sn;
            C[k] += c;
            S[k] += s;
        }
    }
    if (t < count) {
#pragma unroll
        for (int k = 0; k < G; ++k) {
            const int comp = 2 * (k0 - 1 + k);
            part[(split * ncomp + comp) * count + t] = C[k];
            part[(split * ncomp + comp + 1) * count + t] = S[k];
        }
    }
}

// Z^2 = sum_k (C_k^2 + S_k^2) * (2/n)            (periodsearch.py:67-69)
// H   = max_k (cumsum_k[(C^2+S^2)(2/n)] - 4(k-1)) (periodsearch.py:120-123)
// from fp64 per-split partial sums; out[map ? map[t] : t].
__global__ __launch_bounds__(256) void k_search_finalize(const double* __restrict__ part, int64_t count, int splits,
                                                         int m, int stat, double n, const int64_t* __restrict__ map,
                                                         double* __restrict__ out) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= count) return;
    const int ncomp = 2 * m;
    double zsum = 0.0, cum = 0.0, best = -INFINITY;
    const double w = 2.0 / n;
    for (int k = 0; k < m; ++k) {
        double c = 0.0, s = 0.0;
        for (int sp = 0; sp < splits; ++sp) {
            c += part[((int64_t)sp * ncomp + 2 * k) * count + t];
            s += part[((int64_t)sp * ncomp + 2 * k + 1) * count + t];
        }
        const double z = c * c + s * s;
        if (stat == CRIMP_STAT_Z2) {
            zsum += z;
        } else {
            cum += z * w;
            const double v = cum - 4.0 * (double)k;
            best = v > best ? v : best;
        }
    }
    out[map ? map[t] : t] = (stat == CRIMP_STAT_Z2) ? zsum * w : best;
}

#include "mfma_drain.h"
#include "f16_split.h"
#include "search_exact.h"

// ============================================================== 5. ToA likelihood scan
struct TplDev {
    int32_t model, K;
    double amp[CRIMP_MAX_COMP];   // amp_j * ampShift (fourier), amp_j*ampShift/(2 pi) * sinh(w) (cauchy),
                                  // amp_j*ampShift/(2 pi I0(1/w^2)) (vonmises)
    double loc[CRIMP_MAX_COMP];   // ph_j or cen_j
    double ch[CRIMP_MAX_COMP];    // cosh(wid_j) (cauchy)
    double kap[CRIMP_MAX_COMP];   // 1/wid_j^2 (vonmises)
};

constexpr int kPtsPerGroup = 4;
#ifndef CRIMP_PTS_BLOCK
#define CRIMP_PTS_BLOCK 512
#endif
constexpr int kPtsBlock = CRIMP_PTS_BLOCK;  // = kFitBlock: the device fit driver strides and reduces as k_toa_points

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
__device__ __forceinline__ double wave_min(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o));
    return v;
}

// Point coefficients of component j at phShift phi:
//   fourier   c0 = A cos(ph_j - j phi), c1 = -A sin(ph_j - j phi)
//   cauchy/vm c0 = cos(cen_j + phi),    c1 = sin(cen_j + phi)
__device__ __forceinline__ void tpl_coef(const TplDev* __restrict__ T, int j, double phi, double& c0, double& c1) {
    if (T->model == CRIMP_MODEL_FOURIER) {
        const double d = T->loc[j] - (double)(j + 1) * phi;
        c0 = T->amp[j] * cos(d);
        c1 = -T->amp[j] * sin(d);
    } else {
        const double d = T->loc[j] + phi;
        c0 = cos(d);
        c1 = sin(d);
    }
}

// sin/cos of a photon's phase: x in cycles (fourier) or radians (cauchy, von Mises)
__device__ __forceinline__ void photon_sincos(int model, double xv, double& s1, double& c1) {
    if (model == CRIMP_MODEL_FOURIER)
        sincospi(2.0 * xv, &s1, &c1);
    else
        sincos(xv, &s1, &c1);
}

// The same sin/cos from a 4096-entry fp64 table in LDS (k_toa_points and the fit kernels; CRIMP_FIT_TABLE=0 keeps
// the library sincospi / sincos): r = x in turns (x / 2 pi for radians), k = rint(4096 r), delta = 2 pi (r - k / 4096)
// (the subtraction is exact), |delta| <= pi / 4096, cos/sin(delta) by their Taylor series to delta^4 / delta^5
// (truncation < 3e-22), rotated by the table entry: ~2 ulp, against ~30 fp64 operations of the library call.
#ifndef CRIMP_FIT_GENERIC
#define CRIMP_FIT_GENERIC 0
#endif
#ifndef CRIMP_FIT_TABLE
#define CRIMP_FIT_TABLE 1
#endif
constexpr int kSinTab = 4096;
__device__ __forceinline__ void sintab_fill(double2* tab) {
    for (int i = threadIdx.x; i < kSinTab; i += blockDim.x) {
        double sv, cv;
        sincospi((double)i * (2.0 / kSinTab), &sv, &cv);
        tab[i] = make_double2(cv, sv);
    }
    __syncthreads();
}
__device__ __forceinline__ void photon_sincos_tab(int model, const double2* __restrict__ tab, double xv, double& s1,
                                                  double& c1) {
    const double r = (model == CRIMP_MODEL_FOURIER) ? xv : xv * 0.15915494309189533577;
    const double k = rint(r * (double)kSinTab);
    const double d = fma(-k, 1.0 / kSinTab, r) * 6.283185307179586476925;
    const double d2 = d * d;
    const double cd = fma(d2, fma(d2, 1.0 / 24.0, -0.5), 1.0);
    const double sd = d * fma(d2, fma(d2, 1.0 / 120.0, -1.0 / 6.0), 1.0);
    const double2 e = tab[(int)(int64_t)k & (kSinTab - 1)];
    s1 = fma(e.y, cd, e.x * sd);
    c1 = fma(e.x, cd, -(e.y * sd));
}

// 1/v for the likelihood sums: v_rcp_f64 and two Newton steps (5 fp64 operations instead of the ~10 of a correctly
// rounded division; measured equal to 1/v on 2^24 values, one step alone 11 ulps, v_rcp_f64 alone 2^-24.6:
// profiles/r06/mb_rcp.txt). The fit kernels and k_toa_points use the same, so the device-driven and the
// host-driven fits sum identical terms.
#ifndef CRIMP_FIT_EXACT_DIV
#define CRIMP_FIT_EXACT_DIV 0
#endif
__device__ __forceinline__ double lk_rcp(double v) {
#if CRIMP_FIT_EXACT_DIV
    return 1.0 / v;
#else
    double r = __builtin_amdgcn_rcp(v);
    r = fma(fma(-v, r, 1.0), r, r);
    return fma(fma(-v, r, 1.0), r, r);
#endif
}

// h = model - norm at one photon and its first two phShift derivatives h1, h2 (templatemodels.py:64-82,
// :166-185, :271-290), from the photon's (s1, c1) and one point's coefficient rows c0[], cs[].
__device__ __forceinline__ void tpl_terms(const TplDev* __restrict__ T, int model, int K, const double* c0,
                                          const double* cs, double s1, double c1, double& h, double& h1,
                                          double& h2) {
    h = 0.0;
    h1 = 0.0;
    h2 = 0.0;
    if (model == CRIMP_MODEL_FOURIER) {
        // cos, sin of harmonic j+1 by the Chebyshev recurrence c_{j+1} = 2 c_1 c_j - c_{j-1} (one fma each instead of
        // the four operations of an angle addition; error <= ~K^2 ulp)
        const double tc = c1 + c1;
        double cj = c1, sj = s1, cp = 1.0, sp = 0.0;
        for (int j = 0; j < K; ++j) {
            const double al = c0[j], be = cs[j];
            const double tj = fma(al, cj, be * sj);
            const double jj = (double)(j + 1);
            h += tj;
            h2 = fma(-(jj * jj), tj, h2);
            h1 = fma(jj, fma(al, sj, -(be * cj)), h1);
            const double cn = fma(tc, cj, -cp), sn = fma(tc, sj, -sp);
            cp = cj;
            sp = sj;
            cj = cn;
            sj = sn;
        }
    } else {
        for (int j = 0; j < K; ++j) {
            const double C = c0[j], S = cs[j];
            const double cu = c1 * C + s1 * S;  // cos(x - cen - phi)
            const double su = s1 * C - c1 * S;  // sin(x - cen - phi)
            if (model == CRIMP_MODEL_CAUCHY) {
                const double iD = 1.0 / (T->ch[j] - cu);
                const double v = T->amp[j] * iD;  // amp' = a*sinh(w)
                const double dvdu = -v * su * iD;
                const double d2 = -v * iD * (cu - 2.0 * su * su * iD);
                h += v;
                h1 -= dvdu;
                h2 += d2;
            } else {
                const double kp = T->kap[j];
                const double v = T->amp[j] * exp(kp * cu);
                h += v;
                h1 += kp * su * v;
                h2 += (-kp * cu + kp * kp * su * su) * v;
            }
        }
    }
}

// The Fourier branch of tpl_terms for a template size fixed at compile time (the device fit kernel): the same
// per-photon operation order, coefficient rows held in registers, the harmonic loop unrolled.
template <int KF>
__device__ __forceinline__ void tpl_terms_fourier(const double (&al)[KF], const double (&be)[KF], double s1, double c1,
                                                  double& h, double& h1, double& h2) {
    // harmonic 1 starts the sums (not 0 + term: three adds per photon fewer, the same values up to the sign of zero)
    const double tc = c1 + c1;
    double cj = c1, sj = s1, cp = 1.0, sp = 0.0;
#pragma unroll
    for (int j = 0; j < KF; ++j) {
        const double tj = fma(al[j], cj, be[j] * sj);
        const double jj = (double)(j + 1);
        if (j == 0) {
            h = tj;
            h2 = -tj;
            h1 = fma(al[0], sj, -(be[0] * cj));
        } else {
            h += tj;
            h2 = fma(-(jj * jj), tj, h2);
            h1 = fma(jj, fma(al[j], sj, -(be[j] * cj)), h1);
        }
        if (j + 1 < KF) {
            const double cn = fma(tc, cj, -cp), sn = fma(tc, sj, -sp);
            cp = cj;
            sp = sj;
            cj = cn;
            sj = sn;
        }
    }
}

// h alone (no phShift derivatives), bit-identical to tpl_terms_fourier's h
template <int KF>
__device__ __forceinline__ void tpl_value_fourier(const double (&al)[KF], const double (&be)[KF], double s1, double c1,
                                                  double& h) {
    const double tc = c1 + c1;
    double cj = c1, sj = s1, cp = 1.0, sp = 0.0;
#pragma unroll
    for (int j = 0; j < KF; ++j) {
        const double tj = fma(al[j], cj, be[j] * sj);
        h = j == 0 ? tj : h + tj;
        if (j + 1 < KF) {
            const double cn = fma(tc, cj, -cp), sn = fma(tc, sj, -sp);
            cp = cj;
            sp = sj;
            cj = cn;
            sj = sn;
        }
    }
}

// One block per group of <= 4 points of one interval; lanes stride the photons. fp64.
// Coefficient table per point (LDS): fourier  a_j = A cos(ph_j - j phi), b_j = -A sin(ph_j - j phi)
//                                    cauchy/vm a_j = cos(cen_j + phi),   b_j = sin(cen_j + phi)
__global__ __launch_bounds__(kPtsBlock) void k_toa_points(const double* __restrict__ x,
                                                          const int64_t* __restrict__ offsets,
                                                          const TplDev* __restrict__ T,
                                                          const int64_t* __restrict__ grp_int,
                                                          const int64_t* __restrict__ grp_first,
                                                          const int32_t* __restrict__ grp_np,
                                                          const double* __restrict__ pt_norm,
                                                          const double* __restrict__ pt_phi, double* __restrict__ out) {
    __shared__ double coef[kPtsPerGroup][2][CRIMP_MAX_COMP];
    __shared__ double red[kPtsBlock / 64][kPtsPerGroup][8];
#if CRIMP_FIT_TABLE
    __shared__ double2 stab[kSinTab];
    sintab_fill(stab);
#endif
    const int gi = blockIdx.x;
    const int64_t iv = grp_int[gi];
    const int64_t p0 = grp_first[gi];
    const int np = grp_np[gi];
    const int model = T->model, K = T->K;
    const int tid = threadIdx.x;
    if (tid < kPtsPerGroup * K) {
        const int p = tid / K, j = tid % K;
        const double phi = p < np ? pt_phi[p0 + p] : 0.0;
        tpl_coef(T, j, phi, coef[p][0][j], coef[p][1][j]);
    }
    __syncthreads();
    double nrm[kPtsPerGroup];
#pragma unroll
    for (int p = 0; p < kPtsPerGroup; ++p) nrm[p] = p < np ? pt_norm[p0 + p] : 1.0;
    double acc[kPtsPerGroup][7];
#pragma unroll
    for (int p = 0; p < kPtsPerGroup; ++p) {
#pragma unroll
        for (int q = 0; q < 6; ++q) acc[p][q] = 0.0;
        acc[p][6] = INFINITY;
    }
    const int64_t a = offsets[iv], b = offsets[iv + 1];
    for (int64_t i = a + tid; i < b; i += kPtsBlock) {
        double s1, c1;
#if CRIMP_FIT_TABLE
        photon_sincos_tab(model, stab, x[i], s1, c1);
#else
        photon_sincos(model, x[i], s1, c1);
#endif
#pragma unroll
        for (int p = 0; p < kPtsPerGroup; ++p) {
            if (p >= np) break;
            double h, h1, h2;
            tpl_terms(T, model, K, coef[p][0], coef[p][1], s1, c1, h, h1, h2);
            const double mv = nrm[p] + h;
            const double q = lk_rcp(mv);
            acc[p][0] += log(mv);
            acc[p][1] += q;
            acc[p][2] += h1 * q;
            acc[p][3] -= q * q;
            acc[p][4] -= h1 * q * q;
            acc[p][5] += h2 * q - h1 * h1 * q * q;
            acc[p][6] = fmin(acc[p][6], mv);
        }
    }
    const int wid = tid >> 6, lane = tid & 63;
#pragma unroll
    for (int p = 0; p < kPtsPerGroup; ++p) {
#pragma unroll
        for (int q = 0; q < 6; ++q) {
            const double v = wave_sum(acc[p][q]);
            if (lane == 0) red[wid][p][q] = v;
        }
        const double v = wave_min(acc[p][6]);
        if (lane == 0) red[wid][p][6] = v;
    }
    __syncthreads();
    if (tid < kPtsPerGroup * 7) {
        const int p = tid / 7, q = tid % 7;
        if (p < np) {
            double v = red[0][p][q];
            for (int w = 1; w < kPtsBlock / 64; ++w) v = (q == 6) ? fmin(v, red[w][p][q]) : v + red[w][p][q];
            out[(p0 + p) * 8 + q] = v;
            if (q == 0) out[(p0 + p) * 8 + 7] = (double)(b - a);
        }
    }
}

// Brute grid (fp32 model and log2, fp64 fold every 32 photons). One lane per phShift value,
// photons of a 128-photon tile broadcast from LDS; NN norms per lane. The fp32 adds, multiplies and FMAs run
// as packed pairs (v_pk_add/mul/fma_f32: two lane-ops per issue, the only way to the f32 VALU peak) -- the
// template over photon pairs, the norm products over norm pairs -- with each lane's operation order unchanged,
// so the sums are bit-identical to the scalar form.
constexpr int kGridBlock = 128;
constexpr int kGridNN = 20;
constexpr int kGridKMax = 8;
constexpr int kGridProd = 4;
constexpr int64_t kGridTarget = 16384;  // brute-grid blocks per launch (toa_grid_partials)
static_assert(kGridNN % 2 == 0 && kGridProd == 4, "norm pairs; photons in two pairs per product");
constexpr int kGridNNSmall = 4;  // the pruned brute grid's norms per lane (crimp_toa_fit)
#ifndef CRIMP_GRID_MFMA
#define CRIMP_GRID_MFMA 1  // Fourier brute grid on the f16 matrix cores (k_toa_grid_mf)
#endif
#ifndef CRIMP_GRID_PPL
#define CRIMP_GRID_PPL 2
#endif
constexpr int kGridPPL = CRIMP_GRID_PPL;  // phShift values per lane of the pruned grid (k_toa_grid)

typedef float f32x2 __attribute__((ext_vector_type(2)));

// MODEL and (Fourier) the template size KF are template arguments: registers only for the model's own coefficients,
// no per-harmonic branches; KF = 0 reads K from the template at run time. NN (even, <= kGridNN) norms per lane:
// the device fit evaluates only the norms that can hold each phShift's maximum (crimp_toa_fit), usually 2.
// PPL phShift values per lane (1 or 2; the block has kGridBlock / PPL threads and always covers kGridBlock phShift
// values): with 2, every broadcast basis read feeds twice the FMAs. Each (phShift, norm) sum is formed in the same
// operation order whatever PPL, so the sums are bit-identical.
template <int KMAX, int MODEL, int KF, int NN, int PPL>
__global__ __launch_bounds__(kGridBlock) __attribute__((amdgpu_waves_per_eu(4))) void k_toa_grid(const double* __restrict__ x,
                                                         const int64_t* __restrict__ offsets,
                                                         const TplDev* __restrict__ T, const double* __restrict__ norm,
                                                         int nnorm, int a0, int na, const double* __restrict__ phi,
                                                         int nphi, int64_t chunk, int nint,
                                                         double* __restrict__ lnsum, double* __restrict__ hmin) {
    constexpr int TB = kGridBlock / PPL;  // threads per block
    // bas[pair][2j (+1)] = {photon 2 pair, photon 2 pair + 1}: cos / sin of harmonic j+1 (Fourier) or of the phase
    // (j = 0, other models). A photon pair's whole basis is 16 K contiguous bytes, read by broadcast ds_read_b128
    // (cos and sin of one harmonic for both photons) at immediate offsets from one address per pair.
    __shared__ __attribute__((aligned(16))) f32x2 bas[kGridBlock / 2][2 * KMAX];
    float* const basf = reinterpret_cast<float*>(&bas[0][0]);
    auto bset = [&](int photon, int row, float v) { basf[((photon >> 1) * 2 * KMAX + row) * 2 + (photon & 1)] = v; };
    auto bget = [&](int photon, int row) { return basf[((photon >> 1) * 2 * KMAX + row) * 2 + (photon & 1)]; };
    const int tid = threadIdx.x;
    const int64_t iv = blockIdx.y;
    const int64_t split = blockIdx.z;
    constexpr int model = MODEL;
    const int K = KF > 0 ? KF : T->K;
    int bphi[PPL];
    float ca[PPL][KMAX], cb[PPL][KMAX], amp[KMAX], chj[KMAX], kpj[KMAX];
#pragma unroll
    for (int p = 0; p < PPL; ++p) {
        bphi[p] = blockIdx.x * kGridBlock + p * TB + tid;
        const double ph = phi[bphi[p] < nphi ? bphi[p] : nphi - 1];
#pragma unroll
        for (int j = 0; j < KMAX; ++j) {
            ca[p][j] = cb[p][j] = 0.0f;
            if (p == 0) amp[j] = chj[j] = kpj[j] = 0.0f;
            if (j < K) {
                if (model == CRIMP_MODEL_FOURIER) {
                    const double d = T->loc[j] - (double)(j + 1) * ph;
                    ca[p][j] = (float)(T->amp[j] * cos(d));
                    cb[p][j] = (float)(-T->amp[j] * sin(d));
                } else {
                    const double d = T->loc[j] + ph;
                    ca[p][j] = (float)cos(d);
                    cb[p][j] = (float)sin(d);
                    if (p == 0) {
                        amp[j] = (float)T->amp[j];
                        chj[j] = (float)T->ch[j];
                        kpj[j] = (float)(T->kap[j] * 1.4426950408889634);  // exp(k*cu) = exp2(k*log2e*cu)
                    }
                }
            }
        }
    }
    f32x2 nr[NN / 2];
#pragma unroll
    for (int a = 0; a < NN; ++a) nr[a / 2][a % 2] = (a < na) ? (float)norm[iv * nnorm + a0 + a] : 1.0f;
    double acc[PPL][NN];
    float hmn[PPL];
#pragma unroll
    for (int p = 0; p < PPL; ++p) {
        hmn[p] = INFINITY;
#pragma unroll
        for (int a = 0; a < NN; ++a) acc[p][a] = 0.0;
    }
    const int64_t beg = offsets[iv] + split * chunk;
    const int64_t end = std::min<int64_t>(offsets[iv + 1], beg + chunk);
    for (int64_t base = beg; base < end; base += kGridBlock) {
        const int cnt = (int)std::min<int64_t>(kGridBlock, end - base);
        __syncthreads();
#pragma unroll
        for (int q = 0; q < PPL; ++q) {
            const int ph_i = tid + q * TB;  // photon of the tile this thread fills
            if (ph_i < cnt) {
                const double xv = x[base + ph_i];
                double rv = (model == CRIMP_MODEL_FOURIER) ? xv : xv * 0.15915494309189533577;  // cycles
                rv -= rint(rv);
                float s1, c1;
                sincos_rev_poly((float)rv, s1, c1);
                if (model == CRIMP_MODEL_FOURIER) {
                    float cj = c1, sj = s1;
#pragma unroll
                    for (int j = 0; j < KMAX; ++j) {
                        bset(ph_i, 2 * j, cj);
                        bset(ph_i, 2 * j + 1, sj);
                        const float cn = __builtin_fmaf(cj, c1, -sj * s1);
                        sj = __builtin_fmaf(sj, c1, cj * s1);
                        cj = cn;
                    }
                } else {
                    bset(ph_i, 0, c1);
                    bset(ph_i, 1, s1);
                }
            }
        }
        __syncthreads();
        auto hval = [&](int p, int i) {
            float h = 0.0f;
            if (model == CRIMP_MODEL_FOURIER) {
#pragma unroll
                for (int j = 0; j < KMAX; ++j)
                    if (j < K) h = __builtin_fmaf(ca[p][j], bget(i, 2 * j), __builtin_fmaf(cb[p][j], bget(i, 2 * j + 1), h));
            } else {
                const float cx = bget(i, 0), sx = bget(i, 1);
#pragma unroll
                for (int j = 0; j < KMAX; ++j) {
                    if (j < K) {
                        const float cu = __builtin_fmaf(cx, ca[p][j], sx * cb[p][j]);
                        if (model == CRIMP_MODEL_CAUCHY)
                            h += amp[j] * __builtin_amdgcn_rcpf(chj[j] - cu);
                        else
                            h += amp[j] * __builtin_amdgcn_exp2f(kpj[j] * cu);
                    }
                }
            }
            return h;
        };
        // photons i, i+1 (i even) for every phShift of the lane: the Fourier template as packed FMAs, same order per
        // photon as hval; one basis read serves all PPL phShifts
        auto hval2 = [&](int i, f32x2 (&h)[PPL]) {
            if (model == CRIMP_MODEL_FOURIER) {
#pragma unroll
                for (int p = 0; p < PPL; ++p) h[p] = f32x2{0.0f, 0.0f};
#pragma unroll
                for (int j = 0; j < KMAX; ++j)
                    if (j < K) {
                        const f32x2 cj = bas[i >> 1][2 * j], sj = bas[i >> 1][2 * j + 1];   // i is even
#pragma unroll
                        for (int p = 0; p < PPL; ++p)
                            h[p] = __builtin_elementwise_fma(f32x2{ca[p][j], ca[p][j]}, cj,
                                                             __builtin_elementwise_fma(f32x2{cb[p][j], cb[p][j]}, sj, h[p]));
                    }
            } else {
#pragma unroll
                for (int p = 0; p < PPL; ++p) h[p] = f32x2{hval(p, i), hval(p, i + 1)};
            }
        };
        for (int i0 = 0; i0 < cnt; i0 += 32) {
            f32x2 pa[PPL][NN / 2];
#pragma unroll
            for (int p = 0; p < PPL; ++p)
#pragma unroll
                for (int a = 0; a < NN / 2; ++a) pa[p][a] = f32x2{0.0f, 0.0f};
            const int i1 = std::min(cnt, i0 + 32);
            int i = i0;
            // log2 of a product of kGridProd model values instead of kGridProd logs (v_log issues at quarter
            // rate): one photon costs an add and a multiply per norm plus 1/kGridProd of a log and an add.
            // Four factors of (norm + h) <= 2^31 cannot overflow fp32; the product adds <= 3 roundings.
            for (; i + kGridProd <= i1; i += kGridProd) {
                f32x2 h01[PPL], h23[PPL];
                hval2(i, h01);
                hval2(i + 2, h23);
#pragma unroll
                for (int p = 0; p < PPL; ++p) {
                    hmn[p] = fminf(fminf(fminf(fminf(hmn[p], h01[p].x), h01[p].y), h23[p].x), h23[p].y);
#pragma unroll
                    for (int b = 0; b < NN / 2; ++b) {
                        f32x2 pr = nr[b] + h01[p].x;
                        pr *= nr[b] + h01[p].y;
                        pr *= nr[b] + h23[p].x;
                        pr *= nr[b] + h23[p].y;
                        pa[p][b] += f32x2{__builtin_amdgcn_logf(pr.x), __builtin_amdgcn_logf(pr.y)};
                    }
                }
            }
            for (; i < i1; ++i) {
#pragma unroll
                for (int p = 0; p < PPL; ++p) {
                    const float h = hval(p, i);
                    hmn[p] = fminf(hmn[p], h);
#pragma unroll
                    for (int b = 0; b < NN / 2; ++b) {
                        const f32x2 pr = nr[b] + h;
                        pa[p][b] += f32x2{__builtin_amdgcn_logf(pr.x), __builtin_amdgcn_logf(pr.y)};
                    }
                }
            }
#pragma unroll
            for (int p = 0; p < PPL; ++p)
#pragma unroll
                for (int a = 0; a < NN; ++a) acc[p][a] += (double)pa[p][a / 2][a % 2];
        }
    }
#pragma unroll
    for (int p = 0; p < PPL; ++p) {
        if (bphi[p] < nphi) {
#pragma unroll
            for (int a = 0; a < NN; ++a)
                if (a < na) lnsum[((split * nint + iv) * nnorm + a0 + a) * nphi + bphi[p]] = acc[p][a];
            if (a0 == 0) hmin[(split * nint + iv) * nphi + bphi[p]] = (double)hmn[p];
        }
    }
}

// Brute grid of a Fourier template on the f16 matrix cores (the default for Fourier templates of <= 8 harmonics;
// CRIMP_GRID_MFMA=0 builds the VALU kernel above for them too). The template part of every (photon, phShift)
// point is a product of the photon's basis (cos jx, sin jx) and the phShift's coefficients (a_j, b_j):
// h = sum_j a_j cos jx + b_j sin jx, i.e. one (32 photons x 2K) . (2K x 32 phShifts) matrix product per tile. Each
// fp32 factor is carried as hi + lo f16 (f16_split.h split_xy; |x - hi - lo| <= 2^-22 |x|) and the four exact
// products hi.hi, hi.lo, lo.hi, lo.lo of each term fill K = 8 per harmonic of v_mfma_f32_32x32x16_f16 (two harmonics
// per instruction, fp32 accumulation). The VALU is left with the likelihood part: per point and evaluated norm an
// add, 3/4 of a multiply and 1/4 of a v_log_f32 (log2 of products of 4 photons, as k_toa_grid), and the min -- or,
// on crimp_toa_fit's certified modes, 7/8 of a multiply and 1/8 of a log (PROD 8), no add (CIN: the accumulators
// start at the norm) and no min (HMIN false).
// Block: 4 waves, wave w owns the 32 phShift columns 128 bx + 32 w + (lane & 31); a kGmTile-photon tile's A fragments
// (per photon and harmonic 16 bytes: hi, hi, lo, lo of cos then of sin) are built once per tile in LDS by the whole
// block. MFMA result i of lane l is photon (i & 3) + 8 (i >> 2) + 4 (l >> 5) of the 32-photon chunk, phShift column
// l & 31, so each lane multiplies 4 consecutive photons per group; the two lane halves' sums of a column are added
// (half 0 + half 1) at the end. fp64 folds every 32-photon chunk; deterministic, not bit-identical to k_toa_grid.
// Scale: the coefficients and the norms enter multiplied by s = 2^se (grid_mf_scale: the largest amplitude brought into
// [1, 4096] when it lies outside), so that faint templates keep the split's 2^-22 relative accuracy (a lo part below
// 2^-14 would be an f16 subnormal) and bright ones cannot overflow f16; every factor norm + h is then s (norm + h)
// exactly, so the log2 sums lose se per photon (subtracted exactly at the end) and min h is hmn / s. se = 0 (the
// amplitudes already in range, e.g. the bundled template) is the unscaled kernel, bit for bit.
// Tile: CRIMP_GM_TILE photons per LDS tile, built by the block's 256 threads -- 256: one thread per photon computes all
// of its harmonics (one sin/cos and one recurrence per photon); 128 (round 3): two threads per photon, each storing
// half of the harmonics but running the recurrence up to its own. Each photon row has one spare 16-byte slot
// (kGmPad): the 16 lanes of a b128 read pass take 16 consecutive rows, whose start banks are then 16 distinct
// multiples of 4 (row strides of 3, 5, 7, 9 slots for K <= 2, 4, 6, 8; without the pad 2, 4, 6, 8 slots put 2-8 rows
// on the same banks).
#ifndef CRIMP_GM_TILE
#define CRIMP_GM_TILE 256
#endif
#ifndef CRIMP_GM_PAD
#define CRIMP_GM_PAD 1
#endif
// CRIMP_GM_CIN: with one evaluated norm on the eight-factor kernel, the MFMA accumulators start at s norm instead of 0,
// so the matrix cores return the factors s (norm + h) themselves (no add per point; the min h is then
// min(s (norm + h)) - s norm, exact in fp64). The factor is the MFMA's fp32 sum with the norm inside instead of
// fl(norm + fl(h)): rounding-level changes of the lattice LL, held to the full kernel's brute argmax by the tests.
#ifndef CRIMP_GM_CIN
#define CRIMP_GM_CIN 1
#endif
// CRIMP_GM_PREF: each thread loads its photon of the next tile right after building the current one, so the global
// load's latency passes under the current tile's chunks instead of stalling every wave of the block at the build.
// (1.85 -> 1.82 ms per 1250 config-5 grids, profiles/r04/ab_toa_pipe.log.) CRIMP_GM_PIPE=1 (A/B build): a wave
// issues the next chunk's MFMAs before the VALU work on the current chunk's results; it measured slower (1.88 ms):
// the five resident waves per SIMD already overlap one wave's MFMAs with another's VALU work.
#ifndef CRIMP_GM_PREF
#define CRIMP_GM_PREF 1
#endif
#ifndef CRIMP_GM_PIPE
#define CRIMP_GM_PIPE 0
#endif
constexpr int kGmTile = CRIMP_GM_TILE, kGmPad = CRIMP_GM_PAD;
static_assert(kGmTile == 128 || kGmTile == 256, "k_toa_grid_mf: one or two of the block's 256 threads per photon");
static_assert(kGridBlock == 32 * 4, "k_toa_grid_mf: 4 waves of 32 phShift columns cover a block's kGridBlock columns");
// HMIN: track min h per phShift (the public crimp_toa_grid; the device fit skips it when the template's lower bound
// already keeps every evaluated norm + h positive, k_toa_grid_best then takes that bound). PROD: model values per log2
// (4, or 8 when the host has checked that a product of eight factors stays a normal fp32, grid_prod8_ok): the min is
// ~29 % and the logs ~15 % of the likelihood part's VALU.
template <int KF, int NN, bool HMIN = true, int PROD = 4>
__global__ __launch_bounds__(256) void k_toa_grid_mf(const double* __restrict__ x, const int64_t* __restrict__ offsets,
                                                     const TplDev* __restrict__ T, const double* __restrict__ norm,
                                                     int nnorm, int a0, int na, const double* __restrict__ phi, int nphi,
                                                     int64_t chunk, int nint, int se, int a_first,
                                                     double* __restrict__ lnsum, double* __restrict__ hmin) {
    constexpr int NM = (KF + 1) / 2;  // MFMAs per 32-photon chunk (two harmonics each)
    __shared__ __attribute__((aligned(16))) u32x4 afr[kGmTile][2 * NM + kGmPad];  // [photon][harmonic]
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, hk = lane >> 5;
    const int64_t iv = blockIdx.y, split = blockIdx.z;
    const int bphi = blockIdx.x * kGridBlock + 32 * wv + (lane & 31);
    const double sc = ldexp(1.0, se);
    // B fragments: the lane's phShift coefficients of harmonics 2m + hk + 1 (zero past K)
    f16x8 bf[NM];
    {
        const double ph = phi[bphi < nphi ? bphi : nphi - 1];
#pragma unroll
        for (int m = 0; m < NM; ++m) {
            const int j = 2 * m + hk;
            float ca = 0.0f, cb = 0.0f;
            if (j < KF) {
                const double d = T->loc[j] - (double)(j + 1) * ph;
                ca = (float)(T->amp[j] * cos(d) * sc);
                cb = (float)(-T->amp[j] * sin(d) * sc);
            }
            uint32_t dh, dl;
            split_xy<false>(ca, cb, dh, dl);
            const uint32_t wc = (dh & 0xffffu) | (dl << 16), ws = (dh >> 16) | (dl & 0xffff0000u);
            const u32x4 w = {wc, wc, ws, ws};
            bf[m] = __builtin_bit_cast(f16x8, w);
        }
    }
    // PROD 4: the norms in pairs (f32x2 over two norms); PROD 8: one norm at a time over photon pairs (f32x2 over two
    // photons), so that an odd number of norms (a single one after k_toa_grid_best's lazy norms) costs no dead lane
    constexpr int NP = NN > 1 ? NN / 2 : 1;
    constexpr bool CIN = CRIMP_GM_CIN && PROD == 8 && NN == 1;
    f32x2 nr[NP];
    float nrs[NN];
#pragma unroll
    for (int a = 0; a < NN; ++a) {
        nrs[a] = (a < na) ? (float)(norm[iv * nnorm + a0 + a] * sc) : 1.0f;
        nr[a / 2][a % 2] = nrs[a];
    }
    if (NN == 1) nr[0][1] = 1.0f;
    double acc[NN];
#pragma unroll
    for (int a = 0; a < NN; ++a) acc[a] = 0.0;
    float hmn = INFINITY;
    const int64_t beg = offsets[iv] + split * chunk;
    const int64_t end = std::min<int64_t>(offsets[iv + 1], beg + chunk);
    const int pt = tid & (kGmTile - 1);  // this thread's photon of a tile
    double xpre = (CRIMP_GM_PREF && beg + pt < end) ? x[beg + pt] : 0.0;
    for (int64_t base = beg; base < end; base += kGmTile) {
        const int cnt = (int)std::min<int64_t>(kGmTile, end - base);
        __syncthreads();
        {   // A fragments: thread (photon p = tid % kGmTile, part g = tid / kGmTile) builds harmonics [g JP, (g+1) JP)
            constexpr int JP = kGmTile == 256 ? 2 * NM : 4;
            const int p = pt, g = kGmTile == 256 ? 0 : tid >> 7;
            float c1 = 1.0f, s1 = 0.0f;
            if (p < cnt) {
                double rv = CRIMP_GM_PREF ? xpre : x[base + p];
                rv -= rint(rv);
                sincos_rev_poly((float)rv, s1, c1);
            }
            if (CRIMP_GM_PREF) xpre = base + kGmTile + p < end ? x[base + kGmTile + p] : 0.0;
            float cj = c1, sj = s1;
#pragma unroll
            for (int j = 0; j < 2 * NM; ++j) {
                if (j >= JP * g && j < JP * g + JP) {
                    uint32_t dh, dl;
                    split_xy<false>(cj, sj, dh, dl);
                    // {hi, hi}, {lo, lo} of cos (low halves of dh, dl), then of sin (high halves): one v_perm each
                    afr[p][j] = u32x4{__builtin_amdgcn_perm(dh, dh, 0x01000100u), __builtin_amdgcn_perm(dl, dl, 0x01000100u),
                                      __builtin_amdgcn_perm(dh, dh, 0x03020302u), __builtin_amdgcn_perm(dl, dl, 0x03020302u)};
                }
                const float cn = __builtin_fmaf(cj, c1, -sj * s1);
                sj = __builtin_fmaf(sj, c1, cj * s1);
                cj = cn;
            }
        }
        __syncthreads();
        // one 32-photon chunk's template part (32 photons x the wave's 32 phShift columns) on the matrix cores
        auto chunk_mfma = [&](int q0) -> f32x16 {
            f32x16 h = {};
            if constexpr (CIN) {
#pragma unroll
                for (int r = 0; r < 16; ++r) h[r] = nrs[0];
            }
#pragma unroll
            for (int m = 0; m < NM; ++m) {
                const f16x8 av = __builtin_bit_cast(f16x8, afr[q0 + (lane & 31)][2 * m + hk]);
                h = __builtin_amdgcn_mfma_f32_32x32x16_f16(av, bf[m], h, 0, 0, 0);
            }
            return h;
        };
        // the likelihood part of one chunk on the VALU (hv: the chunk's MFMA results)
        auto chunk_valu = [&](const f32x16& hv, int q0) {
            if constexpr (PROD == 8) {
                // photon pairs: per norm, the 16 factors norm + h of the lane's chunk as 8 f32x2, multiplied down a tree
                // to two products of eight (even and odd photons), one v_log_f32 each
                f32x2 pl[NN];
#pragma unroll
                for (int b = 0; b < NN; ++b) pl[b] = f32x2{0.0f, 0.0f};
                if (q0 + 32 <= cnt) {
                    if constexpr (HMIN) {
#pragma unroll
                        for (int r = 0; r < 16; ++r) hmn = fminf(hmn, hv[r]);
                    }
#pragma unroll
                    for (int b = 0; b < NN; ++b) {
                        const f32x2 n2 = f32x2{nrs[b], nrs[b]};
                        f32x2 f[8];
#pragma unroll
                        for (int k = 0; k < 8; ++k) {
                            f[k] = f32x2{hv[2 * k], hv[2 * k + 1]};
                            if constexpr (!CIN) f[k] += n2;
                        }
                        f[0] *= f[1];
                        f[2] *= f[3];
                        f[4] *= f[5];
                        f[6] *= f[7];
                        f[0] *= f[2];
                        f[4] *= f[6];
                        f[0] *= f[4];
                        pl[b] += f32x2{__builtin_amdgcn_logf(f[0].x), __builtin_amdgcn_logf(f[0].y)};
                    }
                } else {  // the tile's last, partial chunk: photons past cnt contribute a factor 1 (products of four)
#pragma unroll
                    for (int gi = 0; gi < 4; ++gi) {
                        float pr[NN];
#pragma unroll
                        for (int b = 0; b < NN; ++b) pr[b] = 1.0f;
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const int row = q0 + r + 8 * gi + 4 * hk;
                            if (row < cnt) {
                                const float h = hv[4 * gi + r];
                                if constexpr (HMIN) hmn = fminf(hmn, h);
#pragma unroll
                                for (int b = 0; b < NN; ++b) pr[b] *= CIN ? h : nrs[b] + h;
                            }
                        }
#pragma unroll
                        for (int b = 0; b < NN; ++b) pl[b].x += __builtin_amdgcn_logf(pr[b]);
                    }
                }
#pragma unroll
                for (int a = 0; a < NN; ++a) acc[a] += (double)pl[a].x + (double)pl[a].y;
                return;
            }
            f32x2 pa[NP];
#pragma unroll
            for (int b = 0; b < NP; ++b) pa[b] = f32x2{0.0f, 0.0f};
            if (q0 + 32 <= cnt) {
#pragma unroll
                for (int gi = 0; gi < 4; ++gi) {
                    if constexpr (HMIN) {
#pragma unroll
                        for (int r = 0; r < 4; ++r) hmn = fminf(hmn, hv[4 * gi + r]);
                    }
#pragma unroll
                    for (int b = 0; b < NP; ++b) {
                        f32x2 pr = nr[b] + hv[4 * gi];
#pragma unroll
                        for (int r = 1; r < 4; ++r) pr *= nr[b] + hv[4 * gi + r];
                        pa[b] += f32x2{__builtin_amdgcn_logf(pr.x), __builtin_amdgcn_logf(pr.y)};
                    }
                }
            } else {  // the tile's last, partial chunk: photons past cnt contribute a factor 1
#pragma unroll
                for (int gi = 0; gi < 4; ++gi) {
                    f32x2 pr[NP];
#pragma unroll
                    for (int b = 0; b < NP; ++b) pr[b] = f32x2{1.0f, 1.0f};
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int row = q0 + r + 8 * gi + 4 * hk;
                        if (row < cnt) {
                            const float h = hv[4 * gi + r];
                            if constexpr (HMIN) hmn = fminf(hmn, h);
#pragma unroll
                            for (int b = 0; b < NP; ++b) pr[b] *= nr[b] + h;
                        }
                    }
#pragma unroll
                    for (int b = 0; b < NP; ++b)
                        pa[b] += f32x2{__builtin_amdgcn_logf(pr[b].x), __builtin_amdgcn_logf(pr[b].y)};
                }
            }
#pragma unroll
            for (int a = 0; a < NN; ++a) acc[a] += (double)pa[a / 2][a % 2];
        };
        if constexpr (CRIMP_GM_PIPE) {  // ping-pong: chunk q + 1's MFMAs issue before chunk q's VALU work
            f32x16 ha = chunk_mfma(0), hb = {};
            for (int q0 = 0; q0 < cnt; q0 += 64) {
                if (q0 + 32 < cnt) hb = chunk_mfma(q0 + 32);
                chunk_valu(ha, q0);
                if (q0 + 32 >= cnt) break;
                if (q0 + 64 < cnt) ha = chunk_mfma(q0 + 64);
                chunk_valu(hb, q0 + 32);
            }
        } else {
            for (int q0 = 0; q0 < cnt; q0 += 32) chunk_valu(chunk_mfma(q0), q0);
        }
    }
    // the column's two lane halves: half 0 + half 1
#pragma unroll
    for (int a = 0; a < NN; ++a) {
        const double o = __shfl_xor(acc[a], 32);
        acc[a] = hk == 0 ? acc[a] + o : o + acc[a];
    }
    hmn = fminf(hmn, __shfl_xor(hmn, 32));
    if (se != 0) {  // every photon's factor carried s = 2^se: log2 s per photon of the split, exactly
        const double drop = (double)se * (double)(end > beg ? end - beg : 0);
#pragma unroll
        for (int a = 0; a < NN; ++a) acc[a] -= drop;
    }
    if (hk == 0 && bphi < nphi) {
#pragma unroll
        for (int a = 0; a < NN; ++a)
            if (a < na) lnsum[((split * nint + iv) * nnorm + a0 + a) * nphi + bphi] = acc[a];
        // the first evaluated norm block writes the min (a_first: past toa_grid_partials' lazy norms)
        if (HMIN && a0 == a_first)
            hmin[(split * nint + iv) * nphi + bphi] = ldexp(CIN ? (double)hmn - (double)nrs[0] : (double)hmn, -se);
    }
}

// np.histogram(x, bins=edges) for uniform edges (numpy/lib/_histograms_impl.py semantics).
// Per-interval phase histogram (np.histogram semantics, binphases.py). Block (iv, y) of a (nint, ns) grid counts
// photons offsets[iv] + 256 y + tid + k 256 ns into one LDS histogram per wave (4-way fewer LDS atomic collisions
// than one per block, the bins being few), then adds its bins to the zeroed int64 counts: integer sums, so the split
// into ns blocks per interval cannot change a count. (One 256-thread block per interval with one shared histogram:
// 0.6 ms for config 5's 1250 x 1e5 photons, ~1.7 TB/s.)
constexpr int kBinWaves = 4;
constexpr int kBinRegs = 16;
__global__ __launch_bounds__(64 * kBinWaves) void k_binphases(const double* __restrict__ x,
                                                              const int64_t* __restrict__ offsets,
                                                              const double* __restrict__ edges, int nb,
                                                              unsigned long long* __restrict__ counts) {
    __shared__ unsigned int cnt[kBinWaves][256];
    __shared__ double se[257];
    const int64_t iv = blockIdx.x;
    const int tid = threadIdx.x, w = tid >> 6;
    for (int b = tid; b < kBinWaves * 256; b += blockDim.x) cnt[b >> 8][b & 255] = 0;
    for (int b = tid; b <= nb; b += blockDim.x) se[b] = edges[b];
    __syncthreads();
    const double first = se[0], last = se[nb];
    const double scale = (double)nb / (last - first);
    // np.histogram's bin: the estimate floor((v - first) / (last - first) * nb), then its two corrections against the
    // edges (v below its left edge: one down; at or above its right edge, unless the last bin: one up). Any estimate
    // within one bin of the true one ends on the same bin, so the product with the reciprocal (a few ulps from numpy's
    // quotient) gives numpy's counts without an fp64 division per photon.
    auto bin = [&](double v) -> int {
        int idx = (int)((v - first) * scale);
        idx = idx < nb ? idx : nb - 1;
        if (v < se[idx]) idx -= 1;
        if (idx != nb - 1 && v >= se[idx + 1]) idx += 1;
        return idx;
    };
    const int64_t stride = (int64_t)blockDim.x * gridDim.y;
    const int64_t beg = offsets[iv] + (int64_t)blockIdx.y * blockDim.x + tid, end = offsets[iv + 1];
    if (nb <= kBinRegs) {
        // up to kBinRegs bins (measuretoas' default 15): per-thread 8-bit counters, bins 0-7 in lo and 8-15 in hi
        // (one shift and a 64-bit add per photon), moved to 32-bit registers every 32 iterations of two photons (a
        // byte holds 64 at most), added to the wave's LDS histogram once at the end
        uint32_t rc[kBinRegs];
#pragma unroll
        for (int b = 0; b < kBinRegs; ++b) rc[b] = 0;
        uint64_t lo = 0, hi = 0;
        int pend = 0;
        auto count = [&](double v) {
            if (!(v >= first && v <= last)) return;
            const int idx = bin(v);
            const uint64_t one = 1ull << (8 * (idx & 7));
            lo += idx < 8 ? one : 0ull;
            hi += idx < 8 ? 0ull : one;
        };
        auto flush = [&]() {
#pragma unroll
            for (int b = 0; b < 8; ++b) {
                rc[b] += (uint32_t)(lo >> (8 * b)) & 0xffu;
                rc[b + 8] += (uint32_t)(hi >> (8 * b)) & 0xffu;
            }
            lo = hi = 0;
            pend = 0;
        };
        for (int64_t i = beg; i < end; i += 2 * stride) {
            const double v0 = x[i];
            const double v1 = i + stride < end ? x[i + stride] : NAN;
            count(v0);
            count(v1);
            if (++pend == 32) flush();
        }
        flush();
#pragma unroll
        for (int b = 0; b < kBinRegs; ++b)
            if (rc[b]) atomicAdd(&cnt[w][b], rc[b]);
    } else {
        for (int64_t i = beg; i < end; i += stride) {
            const double v = x[i];
            if (v >= first && v <= last) atomicAdd(&cnt[w][bin(v)], 1u);
        }
    }
    __syncthreads();
    for (int b = tid; b < nb; b += blockDim.x) {
        unsigned long long c = 0;
#pragma unroll
        for (int k = 0; k < kBinWaves; ++k) c += cnt[k][b];
        if (c) atomicAdd(&counts[iv * nb + b], c);
    }
}

// photon splits per interval for k_binphases: about 8 blocks per CU over the whole call, at least 4096 photons per block
static int64_t bin_splits(int64_t ntot, int64_t nint) {
    const int64_t per = (ntot + nint - 1) / nint;
    return std::max<int64_t>(1, std::min<int64_t>({(2048 + nint - 1) / nint, (per + 4095) / 4096, 65535}));
}

// Many independent one-trial searches (measureToAs.py:210-212: PeriodSearch(TIME_toa*86400, [f(ToA_mid)], 5).htest()
// per interval): set i is t[offsets[i] : offsets[i+1]] with its own t0 = (t[first] + t[last])/2 (periodsearch.py:54)
// and trial frequency freq[i]. One block per set; fp64 as k_search_f64 (harmonic groups of 8 from exact phases,
// fp64 angle addition inside a group), block-reduced fp64 sums, statistic in the reference's formula order.
constexpr int kSetBlock = 256;
__global__ __launch_bounds__(kSetBlock) void k_search_sets(const double* __restrict__ t,
                                                           const int64_t* __restrict__ offsets,
                                                           const double* __restrict__ freq, int m, int stat,
                                                           double tscale, double* __restrict__ out) {
#pragma clang fp contract(off)  // t * tscale rounded before the subtraction, as the host's TIME_toa * 86400
    __shared__ double red[kSetBlock / 64][16];
    const int64_t set = blockIdx.x;
    const int64_t a = offsets[set], b = offsets[set + 1];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    // tscale 1 (seconds) or 86400 (days: the reference's TIME_toa * 86400, measureToAs.py:211, in the same multiply)
    const double t0 = (t[a] * tscale + t[b - 1] * tscale) / 2;
    const double f = freq[set];
    const double w = 2.0 / (double)(b - a);
    double zsum = 0.0, cum = 0.0, best = -INFINITY;
    for (int k0 = 1; k0 <= m; k0 += 8) {
        const int G = m - k0 + 1 < 8 ? m - k0 + 1 : 8;
        double C[8], S[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) C[k] = S[k] = 0.0;
        for (int64_t i = a + tid; i < b; i += kSetBlock) {
            const double ph = f * (t[i] * tscale - t0);
            double s1, c1, s, c;
            sincospi(2.0 * (ph - rint(ph)), &s1, &c1);
            if (k0 == 1) {
                s = s1;
                c = c1;
            } else {
                const double pk = ph * (double)k0;
                sincospi(2.0 * (pk - rint(pk)), &s, &c);
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                if (k < G) {
                    C[k] += c;
                    S[k] += s;
                    const double cn = fma(c, c1, -s * s1);
                    s = fma(s, c1, c * s1);
                    c = cn;
                }
            }
        }
        for (int k = 0; k < G; ++k) {
            const double cw = wave_sum(C[k]), sw = wave_sum(S[k]);
            if (lane == 0) {
                red[wid][2 * k] = cw;
                red[wid][2 * k + 1] = sw;
            }
        }
        __syncthreads();
        if (tid == 0) {
            for (int k = 0; k < G; ++k) {
                double c = 0.0, s = 0.0;
                for (int q = 0; q < kSetBlock / 64; ++q) {
                    c += red[q][2 * k];
                    s += red[q][2 * k + 1];
                }
                const double z = c * c + s * s;
                if (stat == CRIMP_STAT_Z2) {
                    zsum += z;
                } else {
                    cum += z * w;
                    const double v = cum - 4.0 * (double)(k0 - 1 + k);
                    best = v > best ? v : best;
                }
            }
        }
        __syncthreads();
    }
    if (tid == 0) out[set] = (stat == CRIMP_STAT_Z2) ? zsum * w : best;
}

// fp64 fix-up of a few trials over many photons (the exact path's flagged trials): block (t, split) sums the
// harmonics k0 .. k0+G-1 of trial tidx[t] over photons of its split with fp64 sincospi of the exact phase of k0 and
// fp64 angle addition (as k_search_f64), reduced across the block in a fixed order into part[split][2m][count].
constexpr int kFixBlock = 256;
template <int G, bool TWOD>
__global__ __launch_bounds__(kFixBlock) void k_search_f64_few(
    const double* __restrict__ dt, const double* __restrict__ dt2, int64_t n, int64_t chunk,
    const double* __restrict__ freq, int64_t nf, const double* __restrict__ c2row, int64_t first,
    const int64_t* __restrict__ tidx, int64_t count, int k0, int ncomp, double* __restrict__ part) {
    __shared__ double red[kFixBlock / 64][2 * G];
    const int64_t t = blockIdx.x;
    const int64_t split = blockIdx.y;
    const int64_t g = first + tidx[t];
    const int64_t row = TWOD ? g / nf : 0;
    const double f = freq[g - row * nf];
    const double c2 = TWOD ? c2row[row] : 0.0;
    const int64_t i0 = split * chunk;
    const int64_t i1 = i0 + chunk < n ? i0 + chunk : n;
    double C[G], S[G];
#pragma unroll
    for (int k = 0; k < G; ++k) C[k] = S[k] = 0.0;
    for (int64_t i = i0 + threadIdx.x; i < i1; i += kFixBlock) {
        const double ph = TWOD ? fma(f, dt[i], c2 * dt2[i]) : f * dt[i];
        double s1 = 0.0, c1 = 1.0, s, c;
        if (G > 1) sincospi(2.0 * (ph - rint(ph)), &s1, &c1);
        if (k0 == 1 && G > 1) {
            s = s1;
            c = c1;
        } else {
            const double pk = ph * (double)k0;
            sincospi(2.0 * (pk - rint(pk)), &s, &c);
        }
#pragma unroll
        for (int k = 0; k < G; ++k) {
            C[k] += c;
            S[k] += s;
            const double cn = fma(c, c1, -s * s1);
            s = fma(s, c1, c * s1);
            c = cn;
        }
    }
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < G; ++k) {
        const double cw = wave_sum(C[k]), sw = wave_sum(S[k]);
        if (lane == 0) {
            red[wid][2 * k] = cw;
            red[wid][2 * k + 1] = sw;
        }
    }
    __syncthreads();
    if (threadIdx.x < 2 * G) {
        double v = 0.0;
        for (int w = 0; w < kFixBlock / 64; ++w) v += red[w][threadIdx.x];
        part[(split * ncomp + 2 * (k0 - 1) + threadIdx.x) * count + t] = v;
    }
}

#include "toa_fit.h"
#include "toa_shape.h"

// ============================================================== 6. C-ABI
static hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }
// A second stream per device for crimp_toa_fit's overlapped halves (created once, kept for the process)
static hipStream_t aux_stream() {
    static hipStream_t st[64] = {};
    int d = 0;
    if (hipGetDevice(&d) != hipSuccess || d < 0 || d >= 64) return nullptr;
    if (!st[d] && hipStreamCreateWithFlags(&st[d], hipStreamNonBlocking) != hipSuccess) st[d] = nullptr;
    return st[d];
}

extern "C" double crimp_last_kernel_ms(void) { return g_last_kernel_ms; }

extern "C" int crimp_last_kernel_times(double* ms, int32_t cap) {
    const int n = (int)g_kernel_times.size();
    for (int i = 0; i < n && i < cap; ++i) ms[i] = g_kernel_times[(size_t)i];
    return n;
}

extern "C" int crimp_version(void) { return CRIMP_VERSION; }

extern "C" int64_t crimp_last_fixups(void) { return g_last_fixups; }
extern "C" int64_t crimp_last_toa_grid_norms(void) { return g_last_grid_norms; }
extern "C" int64_t crimp_last_toa_grid_fast(void) { return g_last_grid_fast; }

extern "C" int crimp_release_scratch(void) {
    std::lock_guard<std::mutex> lk(g_mutex);
    release_idle_blocks(-1);
    return CRIMP_OK;
}

extern "C" const char* crimp_last_error(void) { return g_err.c_str(); }

extern "C" int crimp_device_count(int32_t* count) {
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (count) *count = (e == hipSuccess) ? n : 0;
    if (e != hipSuccess) return set_err(CRIMP_ERR_NODEV, std::string("hipGetDeviceCount: ") + hipGetErrorString(e));
    return CRIMP_OK;
}

static int finish(hipStream_t s, uint32_t flags) {
    (void)flags;
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(s));  // every call returns with its stream drained (scratch reuse)
    return CRIMP_OK;
}

extern "C" int crimp_calcphase(const double* t_mjd, int64_t n, const crimp_timing_model* model, int32_t parts,
                               double* total, double* folded, uint32_t flags, void* stream) {
    ARGCHK(n >= 0, "n < 0");
    ARGCHK(model != nullptr && total != nullptr && (t_mjd != nullptr || n == 0), "null argument");
    ARGCHK(model->n_glitch >= 0 && model->n_glitch <= CRIMP_MAX_GLITCH, "n_glitch out of range");
    ARGCHK(model->n_wave >= 0 && model->n_wave <= CRIMP_MAX_WAVE, "n_wave out of range");
    if (n == 0) return CRIMP_OK;
    std::lock_guard<std::mutex> lk(g_mutex);
    if (flags & CRIMP_FLAG_TIME_KERNELS) {
        g_kernel_times.clear();
        g_last_kernel_ms = -1.0;
    }
    const bool dev = flags & CRIMP_FLAG_DEVICE_PTRS;
    hipStream_t s = as_stream(stream);
    CPModel hm{};
    hm.pepoch = model->pepoch;
    hm.nterms = 0;
    double fact = 1.0;
    for (int k = 0; k < 13; ++k) {
        fact *= (double)(k + 1);
        hm.coef[k] = (1.0 / fact) * model->f[k];
        if (model->f[k] != 0.0) hm.nterms = k + 1;
    }
    hm.parts = parts;
    hm.n_glitch = model->n_glitch;
    std::memcpy(hm.glitch, model->glitch, sizeof(hm.glitch));
    hm.n_wave = model->n_wave;
    hm.wave_epoch = model->wave_epoch;
    hm.wave_om = model->wave_om;
    hm.f0 = model->f[0];
    std::memcpy(hm.wave_ab, model->wave_ab, sizeof(hm.wave_ab));
    {
        Scratch sc(s);
        const double* dt = nullptr;
        double *dtot = nullptr, *dfol = nullptr;
        HIPCHK(stage_in(sc, t_mjd, (size_t)n, dev, &dt));
        HIPCHK(stage_out(sc, total, (size_t)n, dev, &dtot));
        HIPCHK(stage_out(sc, folded, (size_t)n, dev, &dfol));
        const bool vec = ((reinterpret_cast<uintptr_t>(dt) | reinterpret_cast<uintptr_t>(dtot) |
                           reinterpret_cast<uintptr_t>(dfol)) & 15u) == 0 && (n % 2 == 0);
        const int blocks = (int)std::min<int64_t>(cdiv(vec ? n / 2 : n, 256), int64_t(1) << 20);
        KernelTimer kt(s, flags & CRIMP_FLAG_TIME_KERNELS);
        kt.start();
        // CRIMP_FLAG_FOLD_RADIANS: the folded phase times 2 pi, the host's `folded * (2 * np.pi)` of the Cauchy and
        // von Mises fits (measureToAs.py:195, :200) in the same fp64 multiply
        const double fscale = (flags & CRIMP_FLAG_FOLD_RADIANS) ? 2.0 * 3.141592653589793 : 1.0;
        if (vec)
            k_calcphase_vec<<<blocks, 256, 0, s>>>(reinterpret_cast<const double2*>(dt), n / 2, hm,
                                                     reinterpret_cast<double2*>(dtot), reinterpret_cast<double2*>(dfol),
                                                     fscale);
        else
            k_calcphase_scalar<<<blocks, 256, 0, s>>>(dt, n, hm, dtot, dfol, fscale);
        HIPCHK(hipGetLastError());
        kt.stop();
        HIPCHK(copy_back(s, total, dtot, (size_t)n, dev));
        HIPCHK(copy_back(s, folded, dfol, (size_t)n, dev));
    }
    return finish(s, flags);
}

template <bool TWOD>
static void launch_f64(int G, dim3 grid, hipStream_t s, const double* dt, const double* dt2, int64_t n, int64_t chunk,
                       const double* fr, int64_t nf, const double* c2, int64_t first, const int64_t* tidx,
                       int64_t count, int k0, int ncomp, double* part) {
#define CRIMP_LF(GG)                                                                                             \
    k_search_f64<GG, TWOD><<<grid, kSearchBlock, 0, s>>>(dt, dt2, n, chunk, fr, nf, c2, first, tidx, count, k0, \
                                                         ncomp, part)
    if (G == 8) CRIMP_LF(8); else if (G == 4) CRIMP_LF(4); else if (G == 2) CRIMP_LF(2); else CRIMP_LF(1);
#undef CRIMP_LF
}

// Per-trial device buffers of a search (fp64 per-split partial sums of the fp64 kernel, int64 totals of the exact
// kernel) are bounded by this many bytes (CRIMP_SEARCH_BUDGET_MB, default 2048): a larger trial range
// is computed in blocks of trials.
static int64_t part_budget() {
    static int64_t b = -1;
    if (b < 0) {
        const char* e = getenv("CRIMP_SEARCH_BUDGET_MB");
        const long long mb = e ? atoll(e) : 2048;
        b = (int64_t)(mb > 0 ? mb : 2048) << 20;
    }
    return b;
}

// Relative error the exact path certifies per trial before the fp64 fix-up (CRIMP_FIXUP_REL, default 1e-6; a
// larger value is a test hook that sends more trials through the fix-up).
static double fixup_rel() {
    static double r = -1.0;
    if (r < 0.0) {
        const char* e = getenv("CRIMP_FIXUP_REL");
        r = e ? atof(e) : 1e-6;
        if (!(r > 0.0)) r = 1e-6;
    }
    return r;
}

// Direct (one lane per trial) fp64 search over trials first + (tidx ? tidx[t] : t), t < count, of any grid, into
// out[t] (or out[tidx[t]] with scatter). The photon split count is a function of the photon count only.
static int direct_search(Scratch& sc, hipStream_t s, const double* dt, const double* dt2, int64_t n,
                         const double* freq, int64_t nf, const double* c2, bool twod, int nharm, int stat,
                         int64_t first, const int64_t* tidx, int64_t count, double* out, bool scatter,
                         KernelTimer* kt) {
    const int64_t splits0 = std::max<int64_t>(1, std::min<int64_t>(64, n / 16384));
    const int64_t chunk = cdiv(cdiv(n, splits0), kSearchFold) * kSearchFold;
    const int64_t splits = cdiv(n, chunk);
    const int ncomp = 2 * nharm;
    const int64_t cbmax = std::max<int64_t>(kSearchBlock, part_budget() / (8 * splits * ncomp));
    const int64_t cb = std::min<int64_t>(count, cdiv(cdiv(count, cdiv(count, cbmax)), kSearchBlock) * kSearchBlock);
    double* part = nullptr;
    HIPCHK(sc.alloc(&part, (size_t)(splits * ncomp * cb)));
    if (kt) kt->start();
    for (int64_t b0 = 0; b0 < count; b0 += cb) {
        const int64_t bc = std::min<int64_t>(cb, count - b0);
        const int64_t* bt = tidx ? tidx + b0 : nullptr;
        const int64_t bfirst = tidx ? first : first + b0;
        dim3 grid((unsigned)cdiv(bc, kSearchBlock), (unsigned)splits);
        for (int k0 = 1; k0 <= nharm;) {  // groups of 8, 4, 2, 1 harmonics, each started from its exact phase
            const int rem = nharm - k0 + 1;
            const int G = rem >= 8 ? 8 : rem >= 4 ? 4 : rem >= 2 ? 2 : 1;
            if (twod) launch_f64<true>(G, grid, s, dt, dt2, n, chunk, freq, nf, c2, bfirst, bt, bc, k0, ncomp, part);
            else launch_f64<false>(G, grid, s, dt, dt2, n, chunk, freq, nf, c2, bfirst, bt, bc, k0, ncomp, part);
            HIPCHK(hipGetLastError());
            k0 += G;
        }
        if (kt && b0 + cb >= count) kt->stop();
        k_search_finalize<<<(unsigned)cdiv(bc, 256), 256, 0, s>>>(part, bc, (int)splits, nharm, stat, (double)n,
                                                                 scatter ? bt : nullptr, scatter ? out : out + b0);
        HIPCHK(hipGetLastError());
    }
    return CRIMP_OK;
}

// fp64 fix-up of the trials first + tidx[t] (t < count), a few trials over all photons: photon splits of >= 4096
// photons (up to 1024), one block per (trial, split), the splits combined by k_search_finalize into out[tidx[t]].
static int fixup_search(Scratch& sc, hipStream_t s, const double* dt, const double* dt2, int64_t n, const double* freq,
                        int64_t nf, const double* c2, bool twod, int nharm, int stat, int64_t first,
                        const int64_t* tidx, int64_t count, double* out) {
    const int64_t splits0 = std::max<int64_t>(1, std::min<int64_t>(1024, n / 4096));
    const int64_t chunk = cdiv(n, splits0);
    const int64_t splits = cdiv(n, chunk);
    const int ncomp = 2 * nharm;
    const int64_t cbmax = std::max<int64_t>(1, std::min<int64_t>(65535, part_budget() / (8 * splits * ncomp)));
    double* part = nullptr;
    HIPCHK(sc.alloc(&part, (size_t)(splits * ncomp * std::min<int64_t>(count, cbmax))));
    for (int64_t b0 = 0; b0 < count; b0 += cbmax) {
        const int64_t bc = std::min<int64_t>(cbmax, count - b0);
        dim3 grid((unsigned)bc, (unsigned)splits);
        for (int k0 = 1; k0 <= nharm;) {
            const int rem = nharm - k0 + 1;
            const int G = rem >= 8 ? 8 : rem >= 4 ? 4 : rem >= 2 ? 2 : 1;
#define CRIMP_FX(GG)                                                                                                \
    if (twod)                                                                                                       \
        k_search_f64_few<GG, true><<<grid, kFixBlock, 0, s>>>(dt, dt2, n, chunk, freq, nf, c2, first, tidx + b0, bc, \
                                                              k0, ncomp, part);                                     \
    else                                                                                                            \
        k_search_f64_few<GG, false><<<grid, kFixBlock, 0, s>>>(dt, dt2, n, chunk, freq, nf, c2, first, tidx + b0,   \
                                                               bc, k0, ncomp, part)
            if (G == 8) { CRIMP_FX(8); } else if (G == 4) { CRIMP_FX(4); } else if (G == 2) { CRIMP_FX(2); } else { CRIMP_FX(1); }
#undef CRIMP_FX
            HIPCHK(hipGetLastError());
            k0 += G;
        }
        k_search_finalize<<<(unsigned)cdiv(bc, 256), 256, 0, s>>>(part, bc, (int)splits, nharm, stat, (double)n,
                                                                 tidx + b0, out);
        HIPCHK(hipGetLastError());
    }
    return CRIMP_OK;
}

// Best trial of a power array, np.argmax semantics (periodsearch.py's callers take the maximum and its index): the
// largest value, ties to the lowest index, a NaN above every number (the first NaN wins). k_best_blocks reduces
// grid-stride slices (eight loads in flight per thread) to one candidate per block, k_best_final the candidates.
struct BestCand {
    double v;
    int64_t i;
};
__device__ __forceinline__ bool best_better(double v1, int64_t i1, double v2, int64_t i2) {
    const bool n1 = isnan(v1), n2 = isnan(v2);
    if (n1 != n2) return n1;
    if (!n1 && v1 != v2) return v1 > v2;
    return i1 < i2;
}
__device__ __forceinline__ BestCand best_block_reduce(BestCand c) {
    for (int o = 32; o > 0; o >>= 1) {
        const double v = __shfl_xor(c.v, o);
        const int64_t i = __shfl_xor(c.i, o);
        if (best_better(v, i, c.v, c.i)) c = {v, i};
    }
    __shared__ BestCand red[4];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
    __syncthreads();
    c = red[0];
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w)
        if (best_better(red[w].v, red[w].i, c.v, c.i)) c = red[w];
    return c;
}
constexpr int kBestBlocks = 1024;
__global__ __launch_bounds__(256) void k_best_blocks(const double* __restrict__ x, int64_t n, BestCand* __restrict__ part) {
    constexpr int U = 8;
    BestCand c = {-INFINITY, INT64_MAX};
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t j0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j0 < n; j0 += U * stride) {
        double v[U];
#pragma unroll
        for (int q = 0; q < U; ++q) v[q] = x[j0 + q * stride < n ? j0 + q * stride : n - 1];
#pragma unroll
        for (int q = 0; q < U; ++q) {
            const int64_t j = j0 + q * stride;
            if (j < n && best_better(v[q], j, c.v, c.i)) c = {v[q], j};
        }
    }
    c = best_block_reduce(c);
    if (threadIdx.x == 0) part[blockIdx.x] = c;
}
__global__ __launch_bounds__(256) void k_best_final(const BestCand* __restrict__ part, int nb, double* __restrict__ out) {
    BestCand c = {-INFINITY, INT64_MAX};
    for (int b = threadIdx.x; b < nb; b += blockDim.x)
        if (best_better(part[b].v, part[b].i, c.v, c.i)) c = part[b];
    c = best_block_reduce(c);
    if (threadIdx.x == 0) {
        out[0] = c.v;
        out[1] = (double)c.i;
    }
}

// the best trial of x[n] (device) into dout[0..1] (device): k_best_blocks + k_best_final on the stream, no sync
static int launch_best(Scratch& sc, hipStream_t s, const double* x, int64_t n, double* dout) {
    BestCand* part = nullptr;
    HIPCHK(sc.alloc(&part, (size_t)kBestBlocks));
    const int nb = (int)std::min<int64_t>(cdiv(n, 256 * 8), kBestBlocks);
    k_best_blocks<<<nb, 256, 0, s>>>(x, n, part);
    HIPCHK(hipGetLastError());
    k_best_final<<<1, 256, 0, s>>>(part, nb, dout);
    HIPCHK(hipGetLastError());
    return CRIMP_OK;
}

// Arithmetic-progression check of the (device) frequency grid: 16 ulp of max|f| (k_ap_check, k_ap_final). Writes
// delta into ap[0] on the device (read by the factorised kernels) and returns whether the grid qualifies. With nu_t
// (a NUFFT search) the NUFFT's own checks -- photon order (k_nu_sorted, MFMA-slot plans only) and the plan's
// scalars (k_ap_final) -- are queued with it and read back in the same transfer: nu_hs = [delta, f0, dt[0],
// dt[n-1], unsorted flag]. No memset: k_ap_check zeroes the order flag, k_ap_final writes the rest.
static int grid_is_progression(Scratch& sc, hipStream_t s, const double* freq, int64_t nf, double** ap, bool* ok,
                               const double* nu_t = nullptr, double t0 = 0.0, int64_t n = 0, double* nu_hs = nullptr,
                               bool nu_sorted_check = true, int* nuflags = nullptr, const NuExpect* ex = nullptr);
#include "search_nufft.h"
static int grid_is_progression(Scratch& sc, hipStream_t s, const double* freq, int64_t nf, double** ap, bool* ok,
                               const double* nu_t, double t0, int64_t n, double* nu_hs, bool nu_sorted_check,
                               int* nuflags, const NuExpect* ex) {
    *ok = false;
    // info: [delta, max deviation, max |f|, NUFFT: delta, f_0, dt[0], dt[n-1], order flag (int bits)], then the
    // block partials of k_ap_check
    double* info = nullptr;
    HIPCHK(sc.alloc(&info, 8 + 2 * kApBlocks));
    *ap = info;
    if (nf < 2) return CRIMP_OK;
    double2* part = reinterpret_cast<double2*>(info + 8);
    int* order = reinterpret_cast<int*>(info + 7);
    const int nb = (int)std::min<int64_t>(cdiv(nf, 256 * 8), kApBlocks);
    k_ap_check<<<nb, 256, 0, s>>>(freq, nf, part, nu_t ? order : nullptr);
    HIPCHK(hipGetLastError());
    if (nu_t && nu_sorted_check)
        k_nu_sorted<<<(unsigned)std::min<int64_t>(cdiv(n, 256), 2048), 256, 0, s>>>(nu_t, t0, n, order);
    NuExpect none{};
    k_ap_final<<<1, 256, 0, s>>>(freq, nf, part, nb, info, nu_t, t0, n, info + 3, order, ex ? *ex : none, nuflags);
    HIPCHK(hipGetLastError());
    if (ex && ex->on) {  // a cached NUFFT plan runs on: no read-back, the device checks the plan (nuflags[1])
        *ok = true;
        return CRIMP_OK;
    }
    double h[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    HIPCHK(d2h(s, h, info, (nu_t ? 8 : 3) * sizeof(double)));
    *ok = std::isfinite(h[0]) && h[0] != 0.0 && h[1] <= 16.0 * 2.220446049250313e-16 * h[2];
    if (nu_t) std::memcpy(nu_hs, h + 3, 5 * sizeof(double));
    return CRIMP_OK;
}

// Default path: the exact integer-MFMA kernel (search_exact.h) over an arithmetic-progression grid, then the
// fp64 fix-up of the trials whose power is too small for the kernel's error bound (k_search_finalize_exact).
// int64 totals in units of 2^-36 hold |C_k| <= n exactly for n < 2^27 photons; a larger search runs its photons in
// chunks of < 2^27, each into its own totals, summed exactly by the finalize (periodsearch.py:57-71 has no limit).
static const int64_t kExactMaxPhotons = int64_t(1) << 27;
static const int64_t kExFoldMaxBlocks = 8192;  // fold scratch of one launch <= 1 GiB
static const int64_t kExFoldPhotons = (int64_t)kExFold * kExChunk;  // photons between int64 folds (search_exact.h)
static const int64_t kExNoFoldMaxBlocks = 131072;  // blocks per launch when splits need no fold scratch
// Photon splits of the exact kernel (one 256-thread block per CU): >= 4096 photons per split and >= 8 rounds of
// the device's CUs, and among those counts (up to 4x the smallest) the one whose last round of blocks is fullest:
// a grid of 8.2 rounds runs as long as 9 (config 3: 123 block columns x 17 splits = 2091 blocks on 256 CUs wasted
// 9 %; 29 splits = 3567 blocks fill 13.93 rounds).
static void exact_splits(int64_t n, int64_t bpg, int64_t* chunk_out, int64_t* splits_out) {
    static int ncu = 0;
    if (!ncu) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
            ncu = 256;
    }
    const int64_t smax_n = std::max<int64_t>(1, std::min<int64_t>(cdiv(n, 4096), 65535));
    const int64_t srounds = cdiv(8 * (int64_t)ncu, bpg);
    // Preferred: splits of <= kExFoldPhotons photons, which never fold into the int64 scratch (a block's only
    // global traffic is then its final atomics, 128 KB; each intermediate fold would add 128 KB each way).
    const int64_t snofold = cdiv(n, kExFoldPhotons);
    static const bool long_splits = getenv("CRIMP_EXACT_LONG_SPLITS") != nullptr;  // test hook: the fold path
    if (!long_splits && snofold <= 65535 && bpg * snofold <= kExNoFoldMaxBlocks) {
        const int64_t lo = std::max<int64_t>(1, std::max<int64_t>(snofold, std::min<int64_t>(srounds, smax_n)));
        int64_t best_chunk = 0, best_splits = 0;
        double best_eff = -1.0;
        for (int64_t want = lo; want <= std::min<int64_t>(smax_n, lo + lo / 4 + 1); ++want) {
            const int64_t chunk = cdiv(cdiv(n, want), kExChunk) * kExChunk;
            const int64_t splits = cdiv(n, chunk);
            const int64_t blocks = bpg * splits;
            const double eff = (double)blocks / (double)(cdiv(blocks, ncu) * ncu);
            if (chunk <= kExFoldPhotons && eff > best_eff + 0.005) {
                best_eff = eff;
                best_chunk = chunk;
                best_splits = splits;
            }
        }
        if (best_splits > 0) {
            *chunk_out = best_chunk;
            *splits_out = best_splits;
            return;
        }
    }
    const int64_t smax = std::max<int64_t>(1, std::min<int64_t>(smax_n, kExFoldMaxBlocks / bpg));
    const int64_t smin = std::max<int64_t>(1, std::min<int64_t>(srounds, smax));
    int64_t best_chunk = 0, best_splits = 0;
    double best_eff = -1.0;
    for (int64_t want = smin; want <= std::min<int64_t>(smax, 4 * smin); ++want) {
        const int64_t chunk = cdiv(cdiv(n, want), kExChunk) * kExChunk;
        const int64_t splits = cdiv(n, chunk);
        const int64_t blocks = bpg * splits;
        const double eff = (double)blocks / (double)(cdiv(blocks, ncu) * ncu);
        if (eff > best_eff + 0.005) {
            best_eff = eff;
            best_chunk = chunk;
            best_splits = splits;
        }
    }
    *chunk_out = best_chunk;
    *splits_out = best_splits;
}

static int exact_search(Scratch& sc, hipStream_t s, const double* dt, const double* dt2, int64_t n, const double* freq,
                        int64_t nf, const double* c2, const double* ap, bool twod, int nharm, int stat, int64_t first,
                        int64_t count, double* out, KernelTimer* kt, int64_t* nfixed, bool no_fixup) {
    const int64_t tpr = cdiv(nf, kExTileTrials);
    const int ncomp = 2 * nharm;
    // photon chunks of < 2^27 (one for every search below that), each with its own int64 totals
    const int64_t nchunk = cdiv(n, kExactMaxPhotons - 1);
    const int64_t pc = cdiv(n, nchunk);
    // Trial blocks are bounded by the int64 totals buffer (part_budget) and by the tiles one launch may hold
    // (<= kExFoldMaxBlocks block columns, so that a fold scratch stays <= 1 GiB: a 2-D grid's rows each start a
    // new tile, so a block of short rows holds more tiles than its trial count suggests); whole tiles.
    int64_t want = std::max<int64_t>(kExTileTrials, part_budget() / (8 * ncomp * nchunk)), cb = 0;
    struct Blk { int64_t bfirst, bcount, tf, nt, bpg, chunk, splits; };
    std::vector<Blk> blks;
    int64_t fold_blocks = 0;  // the largest bpg * splits of the blocks whose splits fold into the int64 scratch
    for (;;) {
        cb = std::min<int64_t>(count, cdiv(cdiv(count, cdiv(count, want)), kExTileTrials) * kExTileTrials);
        blks.clear();
        fold_blocks = 0;
        bool fits = true;
        for (int64_t b0 = 0; b0 < count && fits; b0 += cb) {
            Blk k;
            k.bfirst = first + b0;
            k.bcount = std::min<int64_t>(cb, count - b0);
            const int64_t last = k.bfirst + k.bcount - 1;
            k.tf = (k.bfirst / nf) * tpr + (k.bfirst % nf) / kExTileTrials;
            const int64_t tl = (last / nf) * tpr + (last % nf) / kExTileTrials;
            k.nt = tl - k.tf + 1;
            k.bpg = cdiv(k.nt, kExWaves);
            fits = k.bpg <= kExFoldMaxBlocks;
            exact_splits(pc, k.bpg, &k.chunk, &k.splits);
            if (k.chunk > kExFoldPhotons) fold_blocks = std::max<int64_t>(fold_blocks, k.bpg * k.splits);
            blks.push_back(k);
        }
        if (fits) break;
        if (cb <= kExTileTrials) return set_err(CRIMP_ERR_ARG, "exact search: trial block does not fit one launch");
        want = cb / 2;
    }
    if (fold_blocks > kExFoldMaxBlocks) return set_err(CRIMP_ERR_HIP, "exact search: fold scratch bound");
    unsigned long long* tot = nullptr;
    long long* fold = nullptr;
    int64_t* flagged = nullptr;
    int* nflag = nullptr;
    HIPCHK(sc.alloc(&tot, (size_t)(ncomp * cb * nchunk)));
    HIPCHK(sc.alloc(&flagged, (size_t)count));
    HIPCHK(sc.alloc(&nflag, 1));
    // fold scratch only when some block's splits are longer than one fold period; shorter splits never touch it
    if (fold_blocks > 0) HIPCHK(sc.alloc(&fold, (size_t)(fold_blocks * kExWaves * kExFoldVals * 64)));
    HIPCHK(hipMemsetAsync(nflag, 0, sizeof(int), s));
    const double sigc = std::sqrt((double)n) * 1e-9;  // standard deviation of the error of C_k (search_exact.h)
    if (kt) kt->start();
    for (size_t bi = 0; bi < blks.size(); ++bi) {
        const Blk& k = blks[bi];
        const int64_t b0 = k.bfirst - first;
        const int64_t cstride = (int64_t)ncomp * k.bcount;  // one chunk's totals
        HIPCHK(hipMemsetAsync(tot, 0, (size_t)(cstride * nchunk) * sizeof(unsigned long long), s));
        dim3 grid((unsigned)k.bpg, (unsigned)k.splits);
        for (int64_t pch = 0; pch < nchunk; ++pch) {
            const int64_t p0 = pch * pc, np_ = std::min<int64_t>(pc, n - p0);
            unsigned long long* tc = tot + pch * cstride;
            for (int h = 1; h <= nharm; ++h) {
                if (twod)
                    k_search_exact<true><<<grid, kExBlock, 0, s>>>(dt + p0, dt2 ? dt2 + p0 : nullptr, np_, k.chunk, freq,
                                                                   nf, c2, ap, k.tf, k.nt, tpr, k.bfirst, k.bcount, h, tc,
                                                                   fold);
                else
                    k_search_exact<false><<<grid, kExBlock, 0, s>>>(dt + p0, dt2 ? dt2 + p0 : nullptr, np_, k.chunk,
                                                                    freq, nf, c2, ap, k.tf, k.nt, tpr, k.bfirst, k.bcount,
                                                                    h, tc, fold);
                HIPCHK(hipGetLastError());
            }
        }
        if (kt && bi + 1 == blks.size()) kt->stop();
        k_search_finalize_exact<<<(unsigned)cdiv(k.bcount, 256), 256, 0, s>>>(
            reinterpret_cast<const long long*>(tot), k.bcount, nharm, stat, (double)n, sigc, fixup_rel(), b0, out + b0,
            nflag, flagged, (int)nchunk, cstride);
        HIPCHK(hipGetLastError());
    }
    int nf_h = 0;
    HIPCHK(d2h(s, &nf_h, nflag, sizeof(int)));
    *nfixed = nf_h;
    if (nf_h == 0 || no_fixup) return CRIMP_OK;
    return fixup_search(sc, s, dt, dt2, n, freq, nf, c2, twod, nharm, stat, first, flagged, nf_h, out);
}

extern "C" int crimp_best(const double* x, int64_t n, double* best, uint32_t flags, void* stream) {
    ARGCHK(n >= 1, "need at least one value");
    ARGCHK(x != nullptr && best != nullptr, "null argument");
    ARGCHK(n <= (int64_t(1) << 53), "n above 2^53 (the index is returned as a double)");
    const bool dev = flags & CRIMP_FLAG_DEVICE_PTRS;
    std::lock_guard<std::mutex> lk(g_mutex);
    hipStream_t s = as_stream(stream);
    {
        Scratch sc(s);
        const double* dx = nullptr;
        HIPCHK(stage_in(sc, x, (size_t)n, dev, &dx));
        double* dout = nullptr;
        HIPCHK(sc.alloc(&dout, 2));
        const int rc = launch_best(sc, s, dx, n, dout);
        if (rc) return rc;
        HIPCHK(d2h(s, best, dout, 2 * sizeof(double)));
    }
    return finish(s, flags);
}

extern "C" int crimp_last_search_path(void) { return g_last_search_path; }

extern "C" int crimp_last_nufft_plan(int64_t* fft_length, int32_t* moments, int32_t* gather) {
    if (fft_length) *fft_length = g_last_nufft_n;
    if (moments) *moments = g_last_nufft_p;
    if (gather) *gather = g_last_nufft_gather;
    return CRIMP_OK;
}

extern "C" int crimp_last_nufft_work(double* work, int32_t cap) {
    for (int i = 0; i < kNuCls && i < cap; ++i) work[i] = g_nu_work[i];
    return kNuCls;
}

static int search_impl(const double* t, int64_t n, double t0, const double* freq, int64_t nf,
                       const double* log10_negfdot, int64_t nfd, int32_t nharm, int32_t stat, int64_t first,
                       int64_t count, double* out, uint32_t flags, void* stream, double* best);

extern "C" int crimp_search(const double* t, int64_t n, double t0, const double* freq, int64_t nf,
                            const double* log10_negfdot, int64_t nfd, int32_t nharm, int32_t stat, int64_t first,
                            int64_t count, double* out, uint32_t flags, void* stream) {
    return search_impl(t, n, t0, freq, nf, log10_negfdot, nfd, nharm, stat, first, count, out, flags, stream, nullptr);
}

extern "C" int crimp_search_best(const double* t, int64_t n, double t0, const double* freq, int64_t nf,
                                 const double* log10_negfdot, int64_t nfd, int32_t nharm, int32_t stat, int64_t first,
                                 int64_t count, double* out, double* best, uint32_t flags, void* stream) {
    ARGCHK(best != nullptr, "null argument");
    ARGCHK(count >= 1, "the best trial of an empty range");
    ARGCHK(count <= (int64_t(1) << 53), "count above 2^53 (the index is returned as a double)");
    return search_impl(t, n, t0, freq, nf, log10_negfdot, nfd, nharm, stat, first, count, out, flags, stream, best);
}

static int search_impl(const double* t, int64_t n, double t0, const double* freq, int64_t nf,
                       const double* log10_negfdot, int64_t nfd, int32_t nharm, int32_t stat, int64_t first,
                       int64_t count, double* out, uint32_t flags, void* stream, double* best) {
    ARGCHK(n >= 1, "need at least one photon (periodsearch.py:54 reads time[0], time[-1])");
    ARGCHK(nf >= 1, "need at least one trial frequency");
    ARGCHK(nharm >= 1 && nharm <= 256, "nbrHarm must be in 1..256");
    ARGCHK(stat == CRIMP_STAT_Z2 || stat == CRIMP_STAT_H, "unknown statistic");
    ARGCHK(t != nullptr && freq != nullptr && out != nullptr, "null argument");
    const bool twod = log10_negfdot != nullptr && nfd > 0;
    const int64_t total = (twod ? nfd : 1) * nf;
    ARGCHK(first >= 0 && count >= 0 && first + count <= total, "trial range outside the grid");
    const bool f64 = flags & CRIMP_FLAG_F64;
    const bool exact_only = flags & CRIMP_FLAG_EXACT;
    ARGCHK(!(flags & CRIMP_FLAG_RETIRED_FAST), "the fp32 fast search path (flag bits 4, 16, 512) was retired: slower and "
                                                "less precise than the default path");
    ARGCHK(!((flags & CRIMP_FLAG_NUFFT) && f64), "CRIMP_FLAG_NUFFT excludes CRIMP_FLAG_F64");
    ARGCHK(!(exact_only && (f64 || (flags & CRIMP_FLAG_NUFFT))), "CRIMP_FLAG_EXACT excludes CRIMP_FLAG_F64 and _NUFFT");
    // the NUFFT is tried first unless a precision flag excludes it (CRIMP_FLAG_NUFFT asks for the default explicitly)
    const bool nufft = !f64 && !exact_only;
    if (count == 0) return CRIMP_OK;
    std::lock_guard<std::mutex> lk(g_mutex);
    if (flags & CRIMP_FLAG_TIME_KERNELS) {
        g_kernel_times.clear();
        g_last_kernel_ms = -1.0;
    }
    const bool dev = flags & CRIMP_FLAG_DEVICE_PTRS;
    hipStream_t s = as_stream(stream);
    g_last_fixups = 0;
    {
        Scratch sc(s);
        const double *dtm = nullptr, *dfr = nullptr;
        double* dout = nullptr;
        HIPCHK(stage_in(sc, t, (size_t)n, dev, &dtm));
        HIPCHK(stage_in(sc, freq, (size_t)nf, dev, &dfr));
        HIPCHK(stage_out(sc, out, (size_t)count, dev, &dout));
        // fdot term per row, formed on the host exactly as periodsearch.py:95: 0.5*(-1*10**fd)
        double* dc2 = nullptr;
        if (twod) {
            std::vector<double> fdh((size_t)nfd), c2h((size_t)nfd);
            if (dev) {
                HIPCHK(d2h(s, fdh.data(), log10_negfdot, nfd * sizeof(double)));
            } else {
                std::memcpy(fdh.data(), log10_negfdot, nfd * sizeof(double));
            }
            for (int64_t r = 0; r < nfd; ++r) c2h[r] = 0.5 * (-1.0 * std::pow(10.0, fdh[r]));
            HIPCHK(sc.alloc(&dc2, (size_t)nfd));
            HIPCHK(h2d(dc2, c2h.data(), nfd * sizeof(double)));
        }
        // dt = t - t0 (and dt^2) for the exact / fp64 kernels; the NUFFT forms dt in its kernels and skips this
        double *ddt = nullptr, *ddt2 = nullptr;
        auto prep = [&]() -> hipError_t {
            hipError_t e = sc.alloc(&ddt, (size_t)n);
            if (e == hipSuccess && twod) e = sc.alloc(&ddt2, (size_t)n);
            if (e != hipSuccess) return e;
            k_search_prep<<<(int)std::min<int64_t>(cdiv(n, 256), 4096), 256, 0, s>>>(dtm, n, t0, ddt, ddt2);
            return hipGetLastError();
        };
        if (!nufft) HIPCHK(prep());

        // Routing by properties of the whole grid (not of this call's trial range), so that every shard of a
        // sharded search takes the kernel an unsharded search takes:
        //   default (and CRIMP_FLAG_NUFFT): the NUFFT for progressions of >= 64 trials per row (per shard segment),
        //            time-sorted photons and a plan within range (nu_plan); where it declines, the exact rule below;
        //   exact:   exact i8 kernel for progressions of >= 256 trials per row (any length with FORCE_MFMA), fp64
        //            kernel otherwise (a 2-D grid of short rows would fill its 2048-trial tiles with dead columns);
        //   f64:     fp64 kernel.
        KernelTimer kt(s, flags & CRIMP_FLAG_TIME_KERNELS);
        const bool exact_grid = nf >= 256 || (flags & CRIMP_FLAG_FORCE_MFMA);
        bool progression = false;
        double* ap = nullptr;
        double nu_hs[5] = {0, 0, 0, 0, 0};
        int rc = CRIMP_OK;
        bool done = false, best_done = false;
        const bool nu_try = nufft && nf >= 64;
        int* nuflags = nullptr;  // the NUFFT's device flags (fix-up count, photon order / plan check, best trial)
        if (nu_try) HIPCHK(sc.alloc(&nuflags, 8));
        const bool gather_form = nu_gather_form(twod ? nfd : 1);
        // A repeated search over the same buffers reuses its last plan (nu_spec_find): the progression check and
        // the plan's scalars are recomputed on the device and compared there (k_ap_final), every NUFFT kernel that
        // reads photon-derived tables exits if they differ, and the host, reading the result flags anyway at the
        // end, redoes the search from a fresh plan -- one host round trip per search instead of two.
        NuSpecKey key{};
        bool spec_mismatch = false;
        if (nu_try && !f64) {
            key = nu_spec_key(dtm, n, t0, dfr, nf, twod ? nfd : 0, nharm, stat, first, count, gather_form);
            NuExpect ex{};
            if (nu_spec_find(key, nu_hs)) {
                for (int q = 0; q < 4; ++q) ex.v[q] = nu_hs[q];
                ex.on = 1;
                ex.check_order = gather_form ? 0 : 1;
                rc = grid_is_progression(sc, s, dfr, nf, &ap, &progression, dtm, t0, n, nu_hs, !gather_form, nuflags,
                                         &ex);
                if (rc) return rc;
                int64_t nfix = 0;
                rc = nufft_search(sc, s, dtm, t0, n, dfr, nf, twod ? nfd : 1, dc2, nu_hs, twod, nharm, stat, first,
                                  count, dout, flags & CRIMP_FLAG_TIME_KERNELS, &nfix,
                                  (flags & CRIMP_FLAG_NO_FIXUP) != 0, &done, best, &best_done, nuflags, &spec_mismatch);
                if (rc) return rc;
                if (done) g_last_fixups = nfix;
                if (spec_mismatch) nu_spec_drop(key);
                // not done and no mismatch: photons out of order under a still-valid progression (the exact rule)
            }
        }
        if (!done && (!progression || spec_mismatch) && !f64 && (exact_grid || nu_try)) {
            progression = false;
            rc = grid_is_progression(sc, s, dfr, nf, &ap, &progression, nufft ? dtm : nullptr, t0, n, nu_hs,
                                     !gather_form, nuflags, nullptr);
            if (rc) return rc;
            if (progression && nu_try) {  // NUFFT; unsorted photons or no plan fall through to the exact rule
                int64_t nfix = 0;
                bool mm = false;
                rc = nufft_search(sc, s, dtm, t0, n, dfr, nf, twod ? nfd : 1, dc2, nu_hs, twod, nharm, stat, first,
                                  count, dout, flags & CRIMP_FLAG_TIME_KERNELS, &nfix,
                                  (flags & CRIMP_FLAG_NO_FIXUP) != 0, &done, best, &best_done, nuflags, &mm);
                if (rc) return rc;
                if (done) {
                    g_last_fixups = nfix;
                    nu_spec_store(key, nu_hs);
                }
            }
        }
        const bool factorised = !done && progression && exact_grid;
        if ((flags & CRIMP_FLAG_FORCE_MFMA) && !done && !factorised)
            return set_err(CRIMP_ERR_ARG, "factorised search not applicable (grid is not an arithmetic progression)");
        if (nufft && !done) HIPCHK(prep());  // the NUFFT did not apply: the exact / fp64 kernels read dt
        if (done) {
        } else if (factorised) {
            g_last_search_path = 1;
            int64_t nfix = 0;
            rc = exact_search(sc, s, ddt, ddt2, n, dfr, nf, dc2, ap, twod, nharm, stat, first, count, dout, &kt, &nfix,
                              (flags & CRIMP_FLAG_NO_FIXUP) != 0);
            g_last_fixups = nfix;
        } else {
            g_last_search_path = 0;
            rc = direct_search(sc, s, ddt, ddt2, n, dfr, nf, dc2, twod, nharm, stat, first, nullptr, count, dout,
                               false, &kt);
        }
        if (rc) return rc;
        if (best && !best_done) {  // the exact / fp64 paths, or a NUFFT whose fix-up rewrote powers after its read-back
            double* db = nullptr;
            HIPCHK(sc.alloc(&db, 2));
            rc = launch_best(sc, s, dout, count, db);
            if (rc) return rc;
            HIPCHK(d2h(s, best, db, 2 * sizeof(double)));
        }
        HIPCHK(copy_back(s, out, dout, (size_t)count, dev));
    }
    return finish(s, flags);
}

extern "C" int crimp_search_sets(const double* t, const int64_t* offsets, int64_t nset, const double* freq,
                                 int32_t nharm, int32_t stat, double* out, uint32_t flags, void* stream) {
    ARGCHK(nset >= 0, "nset < 0");
    ARGCHK(nharm >= 1 && nharm <= 256, "nbrHarm must be in 1..256");
    ARGCHK(stat == CRIMP_STAT_Z2 || stat == CRIMP_STAT_H, "unknown statistic");
    ARGCHK(t != nullptr && offsets != nullptr && freq != nullptr && out != nullptr, "null argument");
    ARGCHK(nset <= 2147483647LL, "too many sets");
    if (nset == 0) return CRIMP_OK;
    std::lock_guard<std::mutex> lk(g_mutex);
    if (flags & CRIMP_FLAG_TIME_KERNELS) {
        g_kernel_times.clear();
        g_last_kernel_ms = -1.0;
    }
    const bool dev = flags & CRIMP_FLAG_DEVICE_PTRS;
    hipStream_t s = as_stream(stream);
    std::vector<int64_t> hoff((size_t)nset + 1);
    if (dev) {
        HIPCHK(d2h(s, hoff.data(), offsets, (nset + 1) * sizeof(int64_t)));
    } else {
        std::memcpy(hoff.data(), offsets, (nset + 1) * sizeof(int64_t));
    }
    for (int64_t i = 0; i < nset; ++i)
        ARGCHK(hoff[i + 1] > hoff[i] && hoff[i] >= 0, "every set needs photons (periodsearch.py:54 reads time[0])");
    {
        Scratch sc(s);
        const double *dt = nullptr, *df = nullptr;
        const int64_t* doff = nullptr;
        double* dout = nullptr;
        HIPCHK(stage_in(sc, t, (size_t)hoff[nset], dev, &dt));
        HIPCHK(stage_in(sc, offsets, (size_t)nset + 1, dev, &doff));
        HIPCHK(stage_in(sc, freq, (size_t)nset, dev, &df));
        HIPCHK(stage_out(sc, out, (size_t)nset, dev, &dout));
        k_search_sets<<<(unsigned)nset, kSetBlock, 0, s>>>(dt, doff, df, nharm, stat,
                                                           (flags & CRIMP_FLAG_TIME_DAYS) ? 86400.0 : 1.0, dout);
        HIPCHK(hipGetLastError());
        HIPCHK(copy_back(s, out, dout, (size_t)nset, dev));
        // CRIMP_FLAG_ASYNC: with device pointers the call stages nothing and takes no scratch block (a block handed
        // back while the kernel still ran could be given to another call on another stream), so it may return with
        // the kernel queued
        if (dev && (flags & CRIMP_FLAG_ASYNC) && sc.held.empty()) return CRIMP_OK;
    }
    return finish(s, flags);
}

static int make_tpl(const crimp_template* tpl, TplDev* T) {
    ARGCHK(tpl != nullptr, "null template");
    ARGCHK(tpl->ncomp >= 1 && tpl->ncomp <= CRIMP_MAX_COMP, "ncomp out of range");
    ARGCHK(tpl->model >= 0 && tpl->model <= 2, "unknown template model");
    std::memset(T, 0, sizeof(*T));
    T->model = tpl->model;
    T->K = tpl->ncomp;
    const double twopi = 6.283185307179586476925286766559;
    for (int j = 0; j < tpl->ncomp; ++j) {
        const double a = tpl->amp[j] * tpl->amp_shift;
        T->loc[j] = tpl->loc[j];
        if (tpl->model == CRIMP_MODEL_FOURIER) {
            T->amp[j] = a;
        } else if (tpl->model == CRIMP_MODEL_CAUCHY) {
            T->amp[j] = (a / twopi) * std::sinh(tpl->wid[j]);
            T->ch[j] = std::cosh(tpl->wid[j]);
        } else {
            T->amp[j] = a / (twopi * tpl->i0[j]);
            T->kap[j] = 1.0 / (tpl->wid[j] * tpl->wid[j]);
        }
    }
    return CRIMP_OK;
}

// Bounds hmin <= h <= hmax of the template part h = model - norm over every phase and phShift
// (templatemodels.py:64-82, :166-185, :271-290 with TplDev's folded amplitudes)
// A lower bound of the template part h over every phase and phShift, from the template's own shape: min over u of
// h(u) (h(x; phShift) is h shifted in phase for every model, so its minimum does not depend on phShift) sampled on
// 2^16 points per turn, less the largest change between neighbouring samples (a smooth h cannot dip further between
// two samples than it moves across one step). Tighter than tpl_bounds' -sum|amp_j| for Fourier templates.
static double tpl_hmin_scan_uncached(const TplDev& T);
static double tpl_hmin_scan(const TplDev& T) {  // cached for the last template (a fit batch reuses one template)
    static TplDev last;
    static double val = 0.0;
    static bool have = false;
    if (have && std::memcmp(&last, &T, sizeof(T)) == 0) return val;
    val = tpl_hmin_scan_uncached(T);
    std::memcpy(&last, &T, sizeof(T));
    have = true;
    return val;
}
static double tpl_hmin_scan_uncached(const TplDev& T) {
    const int M = 1 << 16;
    double mn = INFINITY, dmax = 0.0, prev = 0.0, first = 0.0;
    for (int i = 0; i <= M; ++i) {
        const double u = 2.0 * M_PI * (double)(i % M) / (double)M;
        double h = 0.0;
        for (int j = 0; j < T.K; ++j) {
            if (T.model == CRIMP_MODEL_FOURIER)
                h += T.amp[j] * std::cos((double)(j + 1) * u + T.loc[j]);
            else if (T.model == CRIMP_MODEL_CAUCHY)
                h += T.amp[j] / (T.ch[j] - std::cos(u - T.loc[j]));
            else
                h += T.amp[j] * std::exp(T.kap[j] * std::cos(u - T.loc[j]));
        }
        if (i == 0) first = h;
        if (i > 0) dmax = std::max(dmax, std::fabs(h - prev));
        mn = std::min(mn, h);
        prev = h;
    }
    (void)first;
    return mn - dmax - 1e-12 * (std::fabs(mn) + dmax);
}

// Lazy-norm certificate (crimp_toa_fit_redchi2): per phShift phi_k of the brute lattice and histogram bin b = [e_b,
// e_{b+1}], an upper bound of the Fourier template part over every photon bin b can hold at phi_k,
// max_{x in bin} h0(x - phi_k / 2 pi) with h0(u) = sum_j amp_j cos(2 pi (j+1) u + loc_j) (k_toa_grid_mf's h): the
// largest of 8192 samples per cycle over the covering sample range plus the Lipschitz bound L / 8192,
// L = sum_j 2 pi (j+1) |amp_j|. out[k * nb + b]. Cached for the last (template, lattice, edges).
static const std::vector<double>& tpl_bin_max(const TplDev& T, const std::vector<double>& phi, const double* edges,
                                              int nb) {
    static TplDev last;
    static std::vector<double> lphi, ledg, val;
    static bool have = false;
    std::vector<double> edg(edges, edges + nb + 1);
    if (have && std::memcmp(&last, &T, sizeof(T)) == 0 && lphi == phi && ledg == edg) return val;
    constexpr int G = 8192;
    std::vector<double> hs(G);
    double L = 0.0;
    for (int j = 0; j < T.K; ++j) L += 2.0 * M_PI * (double)(j + 1) * std::fabs(T.amp[j]);
    for (int g = 0; g < G; ++g) {
        double h = 0.0;
        for (int j = 0; j < T.K; ++j) h += T.amp[j] * std::cos(2.0 * M_PI * (double)(j + 1) * ((double)g / G) + T.loc[j]);
        hs[(size_t)g] = h;
    }
    val.assign(phi.size() * (size_t)nb, 0.0);
    for (size_t k = 0; k < phi.size(); ++k) {
        const double sh = phi[k] / (2.0 * M_PI);
        for (int b = 0; b < nb; ++b) {
            const int64_t g0 = (int64_t)std::floor((edg[(size_t)b] - sh) * G) - 1;
            const int64_t g1 = (int64_t)std::ceil((edg[(size_t)b + 1] - sh) * G) + 1;
            double mx = -INFINITY;
            for (int64_t g = g0; g <= g1; ++g) mx = std::max(mx, hs[(size_t)(((g % G) + G) % G)]);
            val[k * (size_t)nb + (size_t)b] = mx + L / G;
        }
    }
    std::memcpy(&last, &T, sizeof(T));
    lphi = phi;
    ledg = edg;
    have = true;
    return val;
}

static void tpl_bounds(const TplDev& T, double* hmin, double* hmax) {
    double lo = 0.0, hi = 0.0;
    for (int j = 0; j < T.K; ++j) {
        const double a = std::fabs(T.amp[j]);
        if (T.model == CRIMP_MODEL_FOURIER) {
            lo -= a;
            hi += a;
        } else if (T.model == CRIMP_MODEL_CAUCHY) {  // a / (cosh w - cos u), cos u in [-1, 1]
            lo += T.amp[j] / (T.ch[j] + 1.0);
            hi += T.amp[j] / (T.ch[j] - 1.0);
        } else {                                     // a exp(k cos u)
            lo += T.amp[j] * std::exp(-T.kap[j]);
            hi += T.amp[j] * std::exp(T.kap[j]);
        }
    }
    *hmin = std::min(lo, hi);
    *hmax = std::max(lo, hi);
}

extern "C" int crimp_toa_points(const double* x, const int64_t* offsets, int64_t nint, const crimp_template* tpl,
                                const int64_t* pt_interval, const double* pt_norm, const double* pt_phi, int64_t npts,
                                double* out, uint32_t flags, void* stream) {
    ARGCHK(nint >= 1 && npts >= 0, "bad sizes");
    ARGCHK(x != nullptr && offsets != nullptr && pt_interval != nullptr && pt_norm != nullptr && pt_phi != nullptr &&
               out != nullptr,
           "null argument");
    TplDev T;
    int rc = make_tpl(tpl, &T);
    if (rc) return rc;
    if (npts == 0) return CRIMP_OK;
    std::lock_guard<std::mutex> lk(g_mutex);
    if (flags & CRIMP_FLAG_TIME_KERNELS) {
        g_kernel_times.clear();
        g_last_kernel_ms = -1.0;
    }
    const bool dev = flags & CRIMP_FLAG_DEVICE_PTRS;
    hipStream_t s = as_stream(stream);
    // groups of <= 4 consecutive points sharing an interval (host needs the interval ids)
    std::vector<int64_t> pint((size_t)npts), hoff((size_t)nint + 1);
    if (dev) {
        HIPCHK(d2h(s, pint.data(), pt_interval, npts * sizeof(int64_t)));
        HIPCHK(d2h(s, hoff.data(), offsets, (nint + 1) * sizeof(int64_t)));
        HIPCHK(hipStreamSynchronize(s));
    } else {
        std::memcpy(pint.data(), pt_interval, npts * sizeof(int64_t));
        std::memcpy(hoff.data(), offsets, (nint + 1) * sizeof(int64_t));
    }
    for (int64_t i = 0; i < nint; ++i) ARGCHK(hoff[i + 1] >= hoff[i] && hoff[i] >= 0, "offsets must be non-decreasing");
    std::vector<int64_t> gint, gfirst;
    std::vector<int32_t> gnp;
    for (int64_t p = 0; p < npts;) {
        ARGCHK(pint[p] >= 0 && pint[p] < nint, "point interval out of range");
        int64_t q = p + 1;
        while (q < npts && q - p < kPtsPerGroup && pint[q] == pint[p]) ++q;
        gint.push_back(pint[p]);
        gfirst.push_back(p);
        gnp.push_back((int32_t)(q - p));
        p = q;
    }
    const int64_t ng = (int64_t)gint.size();
    {
        Scratch sc(s);
        const double *dx = nullptr, *dn = nullptr, *dp = nullptr;
        const int64_t* doff = nullptr;
        double* dout = nullptr;
        HIPCHK(stage_in(sc, x, (size_t)hoff[nint], dev, &dx));
        HIPCHK(stage_in(sc, offsets, (size_t)nint + 1, dev, &doff));
        HIPCHK(stage_in(sc, pt_norm, (size_t)npts, dev, &dn));
        HIPCHK(stage_in(sc, pt_phi, (size_t)npts, dev, &dp));
        HIPCHK(stage_out(sc, out, (size_t)npts * 8, dev, &dout));
        TplDev* dT = nullptr;
        int64_t *dgi = nullptr, *dgf = nullptr;
        int32_t* dgn = nullptr;
        HIPCHK(sc.alloc(&dT, 1));
        HIPCHK(sc.alloc(&dgi, (size_t)ng));
        HIPCHK(sc.alloc(&dgf, (size_t)ng));
        HIPCHK(sc.alloc(&dgn, (size_t)ng));
        HIPCHK(h2d(dT, &T, sizeof(T)));
        HIPCHK(h2d(dgi, gint.data(), ng * sizeof(int64_t)));
        HIPCHK(h2d(dgf, gfirst.data(), ng * sizeof(int64_t)));
        HIPCHK(h2d(dgn, gnp.data(), ng * sizeof(int32_t)));
        k_toa_points<<<(unsigned)ng, kPtsBlock, 0, s>>>(dx, doff, dT, dgi, dgf, dgn, dn, dp, dout);
        HIPCHK(hipGetLastError());
        HIPCHK(copy_back(s, out, dout, (size_t)npts * 8, dev));
        HIPCHK(hipStreamSynchronize(s));  // host vectors above are read by queued copies
    }
    return finish(s, flags);
}

// k_toa_grid_mf's power-of-two coefficient scale: 0 when the largest |amp_j| is in [1, 4096], otherwise the exponent
// that brings it there; *ok = false where even that is out of reach (the exponent is clamped to [-64, 20], so that
// s x 500 stays far from fp32 overflow in the kernel's products of four factors): those go to the VALU kernel.
static int grid_mf_scale(const TplDev& T, bool* ok) {
    double m = 0.0;
    for (int j = 0; j < T.K; ++j) m = std::max(m, std::fabs(T.amp[j]));
    *ok = std::isfinite(m) && m > 0.0;
    if (!*ok) return 0;
    int e = 0;
    while (std::ldexp(m, e) < 1.0 && e < 20) ++e;
    while (std::ldexp(m, e) > 4096.0 && e > -64) --e;
    const double ms = std::ldexp(m, e);
    *ok = ms >= 1.0 && ms <= 4096.0;
    return e;
}

// Per-split brute-grid partial sums (k_toa_grid) for nint <= 65535 intervals of at most maxn photons:
// pl[((split*nint + i)*nnorm + a)*nphi + b] (log2 sums), ph[(split*nint + i)*nphi + b] (min h).
// mode (crimp_toa_fit's brute grid, Fourier templates on k_toa_grid_mf only): bit 0 (kGridNoMin) -- no per-phShift
// min h (*ph = nullptr: the host's template bound certifies every candidate norm + h > 0); bit 1 (kGridProd8) -- log2 of
// products of eight model values (the host certified that every factor of a valid lattice point stays inside
// [2^-15, 2^15] after the coefficient scale, or k_toa_grid_best checks it where the min decides validity)
// bit 2 (kGridCert) -- no per-phShift min either: the lazy norms' points are shown invalid by the phase histogram
// (k_toa_grid_best with lzmask; crimp_toa_fit_redchi2's histogram, tpl_bin_max)
constexpr int kGridNoMin = 1, kGridProd8 = 2, kGridCert = 4;
// a_first: the lazy norms [0, a_first) of every interval are not evaluated (their lnsum entries are left unwritten;
// k_toa_grid_best knows them invalid from the min, or has the grid rerun in full)
static int toa_grid_partials(Scratch& sc, hipStream_t s, const double* dx, const int64_t* doff, const TplDev* dT,
                             const TplDev& T, const double* dnrm, int64_t nnorm, const double* dphi, int64_t nphi,
                             int64_t nint, int64_t maxn, double** pl, double** ph, int64_t* splits_out,
                             int mode = 0, int* mode_out = nullptr, int64_t a_first = 0) {
    const int model = T.model, K = T.K;
    bool mf_ok = false;
    const int se = grid_mf_scale(T, &mf_ok);
    const int64_t pblocks = cdiv(nphi, kGridBlock);
    // photon splits: aim at kGridTarget blocks (2 waves each; 4 waves/SIMD fit, 2048 resident blocks), so
    // that the last round of waves is a small part of the launch (config 5: 1250 intervals x 14 splits = 8.5
    // rounds; targets of 12288..32768 blocks measured within 1 %, profiles/r02/ab_toa_target.log), splits of
    // >= 1024 photons
    int64_t splits = std::max<int64_t>(1, std::min<int64_t>(cdiv(kGridTarget, pblocks * nint),
                                                            cdiv(std::max<int64_t>(maxn, 1), 1024)));
    splits = std::min<int64_t>(splits, 65535);
    int64_t chunk = cdiv(std::max<int64_t>(maxn, 1), splits);
    chunk = cdiv(chunk, kGridBlock) * kGridBlock;
    splits = cdiv(std::max<int64_t>(maxn, 1), chunk);
    HIPCHK(sc.alloc(pl, (size_t)(splits * nint * nnorm * nphi)));
    const bool mf = model == CRIMP_MODEL_FOURIER && CRIMP_GRID_MFMA && K <= kGridKMax && mf_ok;
    if (!mf) mode = 0;
    if (!(mode & kGridProd8)) a_first = 0;  // lazy norms only on the eight-factor kernel (its caller checks them)
    if (!(mode & kGridProd8)) mode &= ~kGridCert;
    if (mode_out) *mode_out = mode;
    const bool hm = !(mode & (kGridNoMin | kGridCert)), p8 = mode & kGridProd8;
    if (!hm)
        *ph = nullptr;
    else
        HIPCHK(sc.alloc(ph, (size_t)(splits * nint * nphi)));
    dim3 grid((unsigned)pblocks, (unsigned)nint, (unsigned)splits);
    // norms per lane: 2 or kGridNNSmall for a pruned grid (crimp_toa_fit; 1 left after its lazy norms, on the eight-
    // factor kernel), otherwise kGridNN per launch
    const int64_t neval = nnorm - a_first;
    const int nn = (neval == 1 && mf && (mode & kGridProd8)) ? 1 : neval <= 2 ? 2 : neval <= kGridNNSmall ? kGridNNSmall
                                                                                                       : kGridNN;
    for (int64_t a0 = a_first; a0 < nnorm; a0 += nn) {
        const int na = (int)std::min<int64_t>(nn, nnorm - a0);
#define CRIMP_LG1(MD, KK, NNV, PP) k_toa_grid<kGridKMax, MD, KK, NNV, PP><<<grid, kGridBlock / PP, 0, s>>>(dx, doff, dT, dnrm, \
                                                          (int)nnorm, (int)a0, na, dphi, (int)nphi, chunk, (int)nint, *pl, *ph)
#define CRIMP_LG(MD, KK) do { if (nn == 2) CRIMP_LG1(MD, KK, 2, kGridPPL); \
                              else if (nn == kGridNNSmall) CRIMP_LG1(MD, KK, kGridNNSmall, kGridPPL); \
                              else CRIMP_LG1(MD, KK, kGridNN, 1); } while (0)
        if (mf) {
#define CRIMP_LM2(KK, NNV, HM, PR) k_toa_grid_mf<KK, NNV, HM, PR><<<grid, 256, 0, s>>>(dx, doff, dT, dnrm, (int)nnorm, \
                                                        (int)a0, na, dphi, (int)nphi, chunk, (int)nint, se, (int)a_first, \
                                                        *pl, *ph)
#define CRIMP_LM1(KK, NNV) do { \
        if (!hm && p8) CRIMP_LM2(KK, NNV, false, 8); \
        else if (p8) CRIMP_LM2(KK, NNV, true, 8); \
        else if (!hm) CRIMP_LM2(KK, NNV, false, 4); \
        else CRIMP_LM2(KK, NNV, true, 4); } while (0)
#define CRIMP_LM(KK) do { if (nn == 1) { if (hm) CRIMP_LM2(KK, 1, true, 8); else CRIMP_LM2(KK, 1, false, 8); } \
                          else if (nn == 2) CRIMP_LM1(KK, 2); else if (nn == kGridNNSmall) CRIMP_LM1(KK, kGridNNSmall); \
                          else CRIMP_LM1(KK, kGridNN); } while (0)
            switch (K) {
                case 1: CRIMP_LM(1); break;
                case 2: CRIMP_LM(2); break;
                case 3: CRIMP_LM(3); break;
                case 4: CRIMP_LM(4); break;
                case 5: CRIMP_LM(5); break;
                case 6: CRIMP_LM(6); break;
                case 7: CRIMP_LM(7); break;
                default: CRIMP_LM(8); break;
            }
#undef CRIMP_LM
#undef CRIMP_LM1
#undef CRIMP_LM2
        } else if (model == CRIMP_MODEL_FOURIER) {
            switch (K) {
                case 1: CRIMP_LG(CRIMP_MODEL_FOURIER, 1); break;
                case 2: CRIMP_LG(CRIMP_MODEL_FOURIER, 2); break;
                case 3: CRIMP_LG(CRIMP_MODEL_FOURIER, 3); break;
                case 4: CRIMP_LG(CRIMP_MODEL_FOURIER, 4); break;
                case 5: CRIMP_LG(CRIMP_MODEL_FOURIER, 5); break;
                case 6: CRIMP_LG(CRIMP_MODEL_FOURIER, 6); break;
                case 7: CRIMP_LG(CRIMP_MODEL_FOURIER, 7); break;
                default: CRIMP_LG(CRIMP_MODEL_FOURIER, 8); break;
            }
        } else if (model == CRIMP_MODEL_CAUCHY) {
            CRIMP_LG(CRIMP_MODEL_CAUCHY, 0);
        } else {
            CRIMP_LG(CRIMP_MODEL_VONMISES, 0);
        }
#undef CRIMP_LG
#undef CRIMP_LG1
        HIPCHK(hipGetLastError());
    }
    *splits_out = splits;
    return CRIMP_OK;
}

// crimp_toa_fit_redchi2's binned part: np.histogram edges and bin centres (binphases), free parameters, output
struct RedChi2Req {
    const double *edges, *centers;
    int32_t nbins, nfree;
    double* out;
};

struct EventGuard {  // an event destroyed on every return path (destruction waits for nothing unless wait is set)
    hipEvent_t e = nullptr;
    bool wait = false;  // synchronise before destroying: the event marks work that uses scratch blocks of this call
    ~EventGuard() {
        if (e && wait) (void)hipEventSynchronize(e);
        if (e) (void)hipEventDestroy(e);
    }
};

__global__ __launch_bounds__(64) void k_toa_chi2(const unsigned long long* __restrict__ counts, const TplDev T,
                                                 const double* __restrict__ expo, const double* __restrict__ rec,
                                                 const double* __restrict__ centers, int nb, int nfree,
                                                 double* __restrict__ out);

// CRIMP_TOA_HOST_TRACE=1 (diagnostic): host-side phase times of each crimp_toa_fit(_redchi2) call on stderr
struct HostTrace {
    bool on;
    std::chrono::steady_clock::time_point t0, last;
    std::string line;
    HostTrace() : on(getenv("CRIMP_TOA_HOST_TRACE") != nullptr) {
        if (on) t0 = last = std::chrono::steady_clock::now();
    }
    void mark(const char* what) {
        if (!on) return;
        const auto t = std::chrono::steady_clock::now();
        char b[96];
        snprintf(b, sizeof(b), " %s %.1f", what, std::chrono::duration<double, std::micro>(t - last).count());
        line += b;
        last = t;
    }
    ~HostTrace() {
        if (on) fprintf(stderr, "toa host trace (us):%s total %.1f\n", line.c_str(),
                        std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    }
};

static int toa_fit_impl(const double* x, const int64_t* offsets, int64_t nint, const crimp_template* tpl,
                        const double* exposure, double norm0, int32_t ph_shift_res, int32_t options, double* out,
                        uint32_t flags, void* stream, const RedChi2Req* rq) {
    ARGCHK(nint >= 1, "bad sizes");
    ARGCHK(ph_shift_res >= 1, "phShiftRes must be >= 1");
    ARGCHK(norm0 > 0.0, "template norm must be positive");
    ARGCHK(x != nullptr && offsets != nullptr && exposure != nullptr && out != nullptr, "null argument");
    ARGCHK(nint <= 2147483647LL, "too many intervals");
    TplDev T;
    int rc = make_tpl(tpl, &T);
    if (rc) return rc;
    const bool brutemin = options & CRIMP_TOA_BRUTE, vary_amps = options & CRIMP_TOA_VARY_AMPS;
    if (brutemin) ARGCHK(T.K <= kGridKMax, "brute grid supports at most 8 template components");
    std::lock_guard<std::mutex> lk(g_mutex);
    if (flags & CRIMP_FLAG_TIME_KERNELS) {
        g_kernel_times.clear();
        g_last_kernel_ms = -1.0;
    }
    const bool dev = flags & CRIMP_FLAG_DEVICE_PTRS;
    hipStream_t s = as_stream(stream);
    HostTrace ht;
    g_last_grid_norms = 0;
    g_last_grid_fast = 0;
    // the host's copies of the offsets, exposures and (crimp_toa_fit_redchi2) histogram edges: one stream drain for all
    std::vector<int64_t> hoff((size_t)nint + 1);
    std::vector<double> hexp0((size_t)nint), hedg0(rq ? (size_t)rq->nbins + 1 : 0);
    pin_begin((size_t)65536 + (size_t)nint * 340 + hedg0.size() * 8);
    if (dev) {
        const size_t bo = (nint + 1) * sizeof(int64_t), be = nint * sizeof(double), bg = hedg0.size() * sizeof(double);
        const size_t need = ((bo + 255) & ~size_t(255)) + ((be + 255) & ~size_t(255)) + ((bg + 255) & ~size_t(255));
        if (g_pin.p && need <= g_pin.cap) {  // three async reads into the staging buffer, one drain
            char* q = g_pin.p;
            HIPCHK(hipMemcpyAsync(q, offsets, bo, hipMemcpyDeviceToHost, s));
            HIPCHK(hipMemcpyAsync(q + ((bo + 255) & ~size_t(255)), exposure, be, hipMemcpyDeviceToHost, s));
            if (rq)
                HIPCHK(hipMemcpyAsync(q + ((bo + 255) & ~size_t(255)) + ((be + 255) & ~size_t(255)), rq->edges, bg,
                                      hipMemcpyDeviceToHost, s));
            HIPCHK(hipStreamSynchronize(s));
            std::memcpy(hoff.data(), q, bo);
            std::memcpy(hexp0.data(), q + ((bo + 255) & ~size_t(255)), be);
            if (rq) std::memcpy(hedg0.data(), q + ((bo + 255) & ~size_t(255)) + ((be + 255) & ~size_t(255)), bg);
        } else {
            HIPCHK(hipStreamSynchronize(s));
            HIPCHK(hipMemcpy(hoff.data(), offsets, bo, hipMemcpyDeviceToHost));
            HIPCHK(hipMemcpy(hexp0.data(), exposure, be, hipMemcpyDeviceToHost));
            if (rq) HIPCHK(hipMemcpy(hedg0.data(), rq->edges, bg, hipMemcpyDeviceToHost));
        }
    } else {
        std::memcpy(hoff.data(), offsets, (nint + 1) * sizeof(int64_t));
        std::memcpy(hexp0.data(), exposure, nint * sizeof(double));
        if (rq) std::memcpy(hedg0.data(), rq->edges, hedg0.size() * sizeof(double));
    }
    for (int64_t i = 0; i < nint; ++i)
        ARGCHK(hoff[i + 1] > hoff[i] && hoff[i] >= 0,
               "every ToA interval needs photons (measureToAs.py:182 fails on an empty one)");
    g_pin.used = 0;  // the reads are in the host's vectors: the staging buffer starts over for the uploads
    ht.mark("offsets");
    // measureToAs.py:715-725 / :757-771 (readvaryparam=False) and :320-376
    FitCfg C;
    C.lo = norm0 / 100.0;
    C.hi = 500.0;
    C.pb = T.model == CRIMP_MODEL_FOURIER ? M_PI : 1.5 * M_PI;
    C.step = (2.0 * M_PI) / (double)ph_shift_res;
    C.kcap = (double)ph_shift_res / 2.0;
    C.sum_amp = 0.0;
    for (int j = 0; j < tpl->ncomp; ++j) C.sum_amp += tpl->amp[j] * tpl->amp_shift;
    C.amp_lo = T.model == CRIMP_MODEL_FOURIER ? 0.01 : 0.0;                                  // :308, :461, :605
    C.amp_hi = T.model == CRIMP_MODEL_FOURIER ? 100.0 : T.model == CRIMP_MODEL_CAUCHY ? INFINITY : 500.0;
    C.mom_r = kMomR;
    if (const char* e = getenv("CRIMP_FIT_MOM_R")) C.mom_r = atof(e);  // test hook: 0 = iterative norm profiles
    {
        Scratch sc(s);
        const double *dx = nullptr, *de = nullptr;
        const int64_t* doff = nullptr;
        double* dout = nullptr;
        HIPCHK(stage_in(sc, x, (size_t)hoff[nint], dev, &dx));
        HIPCHK(stage_in(sc, offsets, (size_t)nint + 1, dev, &doff));
        HIPCHK(stage_in(sc, exposure, (size_t)nint, dev, &de));
        HIPCHK(stage_out(sc, out, (size_t)nint * 8, dev, &dout));
        // redChi2's histogram (crimp_toa_fit_redchi2) needs only the photons: it runs on the auxiliary stream beside
        // the brute grid and the fits, in the partly empty last round of the fit's workgroups (timed calls: on this
        // stream before the grid's timer starts, so that the kernel times stay those of the grid and the fit alone).
        // The brute grid's lazy-norm certificate reads it too (kGridCert).
        const double *dedg = nullptr, *dcen = nullptr;
        double* dred = nullptr;
        unsigned long long* dcnt = nullptr;
        // destroyed before sc releases its blocks: on an error return between the histogram's launch on the
        // auxiliary stream and the caller stream's wait for it, dcnt stays held until the histogram has finished
        EventGuard ebin;
        ebin.wait = true;
        bool hist_pending = false;
        if (rq) {
            HIPCHK(stage_in(sc, rq->edges, (size_t)rq->nbins + 1, dev, &dedg));
            HIPCHK(stage_in(sc, rq->centers, (size_t)rq->nbins, dev, &dcen));
            HIPCHK(stage_out(sc, rq->out, (size_t)nint, dev, &dred));
            HIPCHK(sc.alloc(&dcnt, (size_t)(nint * rq->nbins)));
            HIPCHK(hipMemsetAsync(dcnt, 0, (size_t)(nint * rq->nbins) * sizeof(unsigned long long), s));
            if (!(flags & CRIMP_FLAG_TIME_KERNELS)) {
                // launched by launch_hist() once the grid's uploads are queued: launched here, its blocks held every
                // CU while the uploads' copy kernels waited for one (the grid started ~180 us late, rocprofv3 trace)
                hist_pending = true;
            } else {
                k_binphases<<<dim3((unsigned)nint, (unsigned)bin_splits(hoff[nint], nint)), 64 * kBinWaves, 0, s>>>(
                    dx, doff, dedg, rq->nbins, dcnt);
                HIPCHK(hipGetLastError());
            }
        }
        ht.mark("stage+hist");
        TplDev* dT = nullptr;
        double* dstart = nullptr;
        HIPCHK(sc.alloc(&dT, 1));
        HIPCHK(h2d_async(s, dT, &T, sizeof(T)));
        HIPCHK(sc.alloc(&dstart, (size_t)(2 * nint)));
        std::vector<double> hphi, hnrm, hstart, grid_n;
        // the brute grid's state, used by the launches below the setup (run_brute)
        int64_t nphi = 0, nc = 0, nlazy = 0;
        double hb = 0.0, gsc = 1.0;
        int grid_mode = 0, lattice_start = 0;
        double *dphi = nullptr, *dnrm = nullptr;
        int* dunsafe = nullptr;
        uint64_t* dlzmask = nullptr;
        int* dlzrow = nullptr;
        std::function<int(int, hipStream_t, int64_t, int64_t)> run_brute;
        if (brutemin) {
            // lmfit brute lattices (measureToAs.py:292-295): scipy mgrid phShift = k*0.05 - bound, 20 norms
            nphi = (int64_t)std::ceil((2.0 * C.pb) / (0.05 * 1.0));
            const int64_t nn = 20;
            hphi.resize((size_t)nphi);
            for (int64_t k = 0; k < nphi; ++k) hphi[(size_t)k] = (double)k * 0.05 + (-C.pb);
            grid_n.resize((size_t)nn);
            for (int64_t a = 0; a < nn; ++a) grid_n[(size_t)a] = (double)a * ((C.hi - C.lo) / (double)(nn - 1)) + C.lo;
            // Pruned norm axis. At fixed phShift the extended LL is -nE + sum_i ln(n + h_i) + const (every model:
            // templatemodels.py:109-121, :213-226, :318-329), strictly concave in n, with its maximum n* where
            // sum_i 1/(n* + h_i) = E, so n* lies in [N/E - hmax, N/E - hmin] for any bounds hmin <= h_i <= hmax. The
            // lattice maximum over the norms at that phShift is then at one of the grid norms adjacent to that
            // interval: every other grid norm is strictly lower (a whole grid step, ~26 norm units, from a
            // bracketing one), so the brute grid's argmax (lmfit brute, measureToAs.py:292-295) is found among them.
            // Config 5 and the worked example: 2 of the 20 norms.
            double hlo = 0.0, hhi = 0.0;
            tpl_bounds(T, &hlo, &hhi);
            const std::vector<double>& hexp = hexp0;
            std::vector<int64_t> alo((size_t)nint), acnt((size_t)nint);
            int64_t ncand = 1;
            for (int64_t i = 0; i < nint; ++i) {
                const double r = (double)(hoff[i + 1] - hoff[i]) / hexp[(size_t)i];
                const double lo_n = r - hhi, hi_n = r - hlo, eps = 1e-9 * (1.0 + std::fabs(r) + hhi - hlo);
                int64_t a0 = 0, a1 = nn - 1;
                if (std::isfinite(lo_n) && std::isfinite(hi_n) && hexp[(size_t)i] > 0.0) {
                    while (a0 + 1 < nn && grid_n[(size_t)(a0 + 1)] <= lo_n - eps) ++a0;
                    while (a1 > a0 && grid_n[(size_t)(a1 - 1)] >= hi_n + eps) --a1;
                }
                alo[(size_t)i] = a0;
                acnt[(size_t)i] = a1 - a0 + 1;
                ncand = std::max(ncand, a1 - a0 + 1);
            }
            if (ncand > kGridNNSmall || getenv("CRIMP_TOA_FULL_GRID")) {  // (test hook: evaluate all 20 norms)
                for (int64_t i = 0; i < nint; ++i) {
                    alo[(size_t)i] = 0;
                    acnt[(size_t)i] = nn;
                }
                ncand = nn;
            }
            // compacted per-interval norms: the candidates in grid order, padded by repeating the last (a repeat
            // comes later in norm-outer order, so it never wins a tie)
            nc = ncand <= 2 ? 2 : ncand <= kGridNNSmall ? kGridNNSmall : ncand;
            g_last_grid_norms = nc;
            hnrm.resize((size_t)(nint * nc));
            for (int64_t i = 0; i < nint; ++i)
                for (int64_t c = 0; c < nc; ++c)
                    hnrm[(size_t)(i * nc + c)] = grid_n[(size_t)(alo[(size_t)i] + std::min(c, acnt[(size_t)i] - 1))];
            HIPCHK(sc.alloc(&dphi, (size_t)nphi));
            HIPCHK(sc.alloc(&dnrm, (size_t)(nint * nc)));
            HIPCHK(h2d_async(s, dphi, hphi.data(), nphi * sizeof(double)));
            HIPCHK(h2d_async(s, dnrm, hnrm.data(), nint * nc * sizeof(double)));
            // test hook: start the ascent at the brute lattice point itself (not at the rate norm + parabola vertex)
            lattice_start = getenv("CRIMP_TOA_LATTICE_START") != nullptr;
            // Fast brute grid (k_toa_grid_mf, Fourier): without the per-phShift min h when a lower bound hb of h keeps
            // every candidate lattice point valid (norm + h > 0) and decides k_toa_grid_best's start rule as the min
            // would (hb + N/E > N/E / 2 for every interval); with log2 of products of eight model values when every
            // factor s (norm + h) of a valid point stays in [2^-15, 2^15], so that a product of eight is a normal fp32:
            // certified here from hb and the template's upper bound for the norms above -hb, and checked by
            // k_toa_grid_best (from the min) for the others -- a lattice point there that could have underflowed sends
            // the grid back to the four-factor kernel (test hook CRIMP_TOA_GRID_SLOW: always the full kernel).
            hb = tpl_hmin_scan(T);
            int mode = 0;
            bool mf_ok = false;
            gsc = std::ldexp(1.0, grid_mf_scale(T, &mf_ok));
            // the fast modes exist on k_toa_grid_mf only (toa_grid_partials' own test): decided once here, so that
            // a Cauchy / von Mises / K > kGridKMax fit sets up no mode state, certificate or unsafe readback
            const bool mf_grid = T.model == CRIMP_MODEL_FOURIER && CRIMP_GRID_MFMA && T.K <= kGridKMax && mf_ok;
            if (mf_grid && getenv("CRIMP_TOA_GRID_SLOW") == nullptr && std::isfinite(hb)) {
                bool nomin = true, prod8 = true;
                for (const double nv : hnrm) {
                    nomin = nomin && nv + hb > 0.0;
                    prod8 = prod8 && (nv + hhi) * gsc <= std::ldexp(1.0, 15) &&
                            (nv + hb <= 0.0 || (nv + hb) * gsc >= std::ldexp(1.0, -15));
                }
                for (int64_t i = 0; i < nint && nomin; ++i) {
                    const double r = (double)(hoff[i + 1] - hoff[i]) / hexp[(size_t)i];
                    nomin = hb + r > 0.5 * r;
                }
                mode = (nomin ? kGridNoMin : 0) | (prod8 ? kGridProd8 : 0);
            }
            // Lazy norms: the leading candidate norms of every interval with norm + hb <= 0 are left out of the grid.
            // Their lattice points are valid only where the per-phShift min h exceeds -norm; k_toa_grid_best marks the
            // rest -inf, as the full grid does, and a valid one sends the grid back to the full evaluation. (Config 5:
            // lmfit's lowest grid norm, norm0/100, is a candidate of every interval and invalid everywhere.)
            // lazy_uniform: every interval has exactly nlazy leading lazy norms. The certificate below needs it: an
            // interval with more would have evaluated norms with norm + hb <= 0 that k_toa_grid_best, without the min,
            // could not judge.
            bool lazy_uniform = false;
            if ((mode & kGridProd8) && !(mode & kGridNoMin)) {
                nlazy = nc;
                int64_t zmax = 0;
                for (int64_t i = 0; i < nint; ++i) {
                    int64_t z = 0;
                    while (z < nc && hnrm[(size_t)(i * nc + z)] + hb <= 0.0) ++z;
                    nlazy = std::min(nlazy, z);
                    zmax = std::max(zmax, z);
                }
                lazy_uniform = zmax == nlazy;
                if (nlazy >= nc) nlazy = 0;  // every candidate lazy: evaluate them all
            }
            // Lazy-norm certificate (crimp_toa_fit_redchi2, whose histogram is at hand; CRIMP_TOA_NO_CERT: off): a lazy
            // point (norm n0, phi_k) is invalid when some photon has h <= -n0; it does where a bin b holds photons and
            // the template's bound over that bin at phi_k (tpl_bin_max) is <= -n0 - margin (1e-3 + 1e-5 of the
            // amplitude sum and n0: it covers the kernel's fp32 h). With the start rule decided by hb too (as kGridNoMin), the grid then needs no min h:
            // k_toa_grid_best marks those points -inf from the counts, and one it cannot show invalid reruns the grid
            // with the min (the flag below). Used only when every (lazy norm, phi_k) has such a bin.
            if (rq && nlazy > 0 && lazy_uniform && mode == kGridProd8 && rq->nbins <= 64 &&
                getenv("CRIMP_TOA_NO_CERT") == nullptr) {
                bool srule = true;
                for (int64_t i = 0; i < nint && srule; ++i) {
                    const double r = (double)(hoff[i + 1] - hoff[i]) / hexp[(size_t)i];
                    srule = hb + r > 0.5 * r;
                }
                if (srule) {
                    const int nb = rq->nbins;
                    const std::vector<double>& hedg = hedg0;
                    const std::vector<double>& bm = tpl_bin_max(T, hphi, hedg.data(), nb);
                    std::vector<double> vals;  // the distinct lazy norms (lattice values)
                    std::vector<int> hrow((size_t)(nint * nlazy));
                    for (int64_t i = 0; i < nint; ++i)
                        for (int64_t z = 0; z < nlazy; ++z) {
                            const double v = hnrm[(size_t)(i * nc + z)];
                            size_t r = 0;
                            while (r < vals.size() && vals[r] != v) ++r;
                            if (r == vals.size()) vals.push_back(v);
                            hrow[(size_t)(i * nlazy + z)] = (int)r;
                        }
                    std::vector<uint64_t> hmask(vals.size() * (size_t)nphi, 0);
                    // margin over the kernel's h: its f16 hi/lo terms and fp32 sums err by <~ 1e-6 of the amplitude
                    // sum and of the norm inside the accumulators (k_toa_grid_mf), so 1e-5 of them plus 1e-3
                    double asum = 0.0;
                    for (int j = 0; j < T.K; ++j) asum += std::fabs(T.amp[j]);
                    bool all_k = true;
                    for (size_t r = 0; r < vals.size(); ++r)
                        for (int64_t k = 0; k < nphi; ++k) {
                            const double margin = 1e-3 + 1e-5 * (asum + std::fabs(vals[r]));
                            uint64_t m = 0;
                            for (int b = 0; b < nb; ++b)
                                if (bm[(size_t)k * nb + b] + margin <= -vals[r]) m |= 1ull << b;
                            hmask[r * (size_t)nphi + (size_t)k] = m;
                            all_k = all_k && m != 0;
                        }
                    if (all_k) {
                        HIPCHK(sc.alloc(&dlzmask, hmask.size()));
                        HIPCHK(sc.alloc(&dlzrow, hrow.size()));
                        HIPCHK(h2d_async(s, dlzmask, hmask.data(), hmask.size() * sizeof(uint64_t)));
                        HIPCHK(h2d_async(s, dlzrow, hrow.data(), hrow.size() * sizeof(int)));
                        mode |= kGridCert;
                    }
                }
            }
            // dunsafe -- k_toa_grid_best: a valid lattice point whose min factor is below 2^-15 / s, or of a lazy norm
            HIPCHK(sc.alloc(&dunsafe, 1));
            HIPCHK(hipMemsetAsync(dunsafe, 0, sizeof(int), s));
            // brute grid of intervals [i0, i0 + n) on stream st (k_toa_grid_mf / k_toa_grid + k_toa_grid_best)
            auto brute = [&](int md, hipStream_t st, int64_t b0, int64_t bn) -> int {
                for (int64_t i0 = b0; i0 < b0 + bn; i0 += 65535) {
                    const int64_t nb = std::min<int64_t>(65535, b0 + bn - i0);
                    int64_t maxn = 0;
                    for (int64_t i = i0; i < i0 + nb; ++i) maxn = std::max(maxn, hoff[i + 1] - hoff[i]);
                    double *pl = nullptr, *ph = nullptr;
                    int64_t splits = 0;
                    int ran = 0;
                    const int64_t lz = (md & kGridProd8) ? nlazy : 0;
                    const int r2 = toa_grid_partials(sc, st, dx, doff + i0, dT, T, dnrm + i0 * nc, nc, dphi, nphi, nb,
                                                     maxn, &pl, &ph, &splits, md, &ran, lz);
                    if (r2) return r2;
                    g_last_grid_fast = ran;
                    g_last_grid_norms = nc - ((ran & kGridProd8) ? lz : 0);  // the lazy norms are not evaluated
                    const bool cert = ran & kGridCert;
                    if (cert && ebin.e) HIPCHK(hipStreamWaitEvent(st, ebin.e, 0));  // the histogram's counts
                    k_toa_grid_best<<<(unsigned)nb, 256, 0, st>>>(pl, ph, dnrm + i0 * nc, dphi, doff + i0, de + i0, (int)nc,
                                                                 (int)nphi, (int)nb, (int)splits, T.model, C.sum_amp,
                                                                 grid_n[0], C.lo, C.hi, lattice_start, hb,
                                                                 (ran & kGridProd8) ? gsc : 0.0,
                                                                 (ran & kGridProd8) ? (int)lz : 0, dunsafe,
                                                                 cert ? dlzmask : nullptr, cert ? dlzrow + i0 * lz : nullptr,
                                                                 cert ? dcnt + i0 * rq->nbins : nullptr, cert ? rq->nbins : 0,
                                                                 dstart + 2 * i0);
                    HIPCHK(hipGetLastError());
                }
                return CRIMP_OK;
            };
            grid_mode = mode;
            run_brute = brute;
        } else {  // Nelder-Mead starts from the template (norm0, phShift 0) (measureToAs.py:301)
            hstart.resize((size_t)(2 * nint));
            for (int64_t i = 0; i < nint; ++i) {
                hstart[(size_t)(2 * i)] = norm0;
                hstart[(size_t)(2 * i + 1)] = 0.0;
            }
            HIPCHK(h2d_async(s, dstart, hstart.data(), 2 * nint * sizeof(double)));
        }
        // the fit kernel over intervals [f0, f0 + fn) on stream st
        double* hcache = nullptr;  // per-photon template part for the iterative norm profiles of the 1-sigma scan (only
                                   // the CRIMP_FIT_MOMENTS=0 build caches it; the moment profile needs none)
        if (!vary_amps && !CRIMP_FIT_MOMENTS) HIPCHK(sc.alloc(&hcache, (size_t)hoff[nint]));
        auto fit = [&](hipStream_t st, int64_t f0, int64_t fn) {
            if (vary_amps) {
                k_toa_fit_amp<<<(unsigned)fn, kFitBlock, 0, st>>>(dx, doff + f0, dT, de + f0, dstart + 2 * f0, C,
                                                                  dout + 8 * f0);
                return;
            }
#define CRIMP_LF(MD, KK) k_toa_fit<MD, KK><<<(unsigned)fn, kFitBlock, 0, st>>>(dx, doff + f0, dT, de + f0, dstart + 2 * f0, \
                                                                             C, dout + 8 * f0, hcache)
            if (T.model == CRIMP_MODEL_FOURIER) {
#if CRIMP_FIT_GENERIC  // A/B build: the template size read at run time
                CRIMP_LF(CRIMP_MODEL_FOURIER, 0);
#else
                switch (T.K) {
                    case 1: CRIMP_LF(CRIMP_MODEL_FOURIER, 1); break;
                    case 2: CRIMP_LF(CRIMP_MODEL_FOURIER, 2); break;
                    case 3: CRIMP_LF(CRIMP_MODEL_FOURIER, 3); break;
                    case 4: CRIMP_LF(CRIMP_MODEL_FOURIER, 4); break;
                    case 5: CRIMP_LF(CRIMP_MODEL_FOURIER, 5); break;
                    case 6: CRIMP_LF(CRIMP_MODEL_FOURIER, 6); break;
                    case 7: CRIMP_LF(CRIMP_MODEL_FOURIER, 7); break;
                    case 8: CRIMP_LF(CRIMP_MODEL_FOURIER, 8); break;
                    default: CRIMP_LF(CRIMP_MODEL_FOURIER, 0); break;
                }
#endif
            } else if (T.model == CRIMP_MODEL_CAUCHY) {
                CRIMP_LF(CRIMP_MODEL_CAUCHY, 0);
            } else {
                CRIMP_LF(CRIMP_MODEL_VONMISES, 0);
            }
#undef CRIMP_LF
        };
        // Brute grid, then fits, in sequence on the caller's stream. CRIMP_TOA_OVERLAP=1 (A/B build switch, read per
        // call) runs the intervals in two halves on two streams instead, the second half's grid beside the first half's
        // fits (every interval's fit is independent of its batch, so the records are those of the sequential order):
        // measured slower on config 5 (6.1 vs 5.7 ms per 1250 intervals, profiles/r04/toa_breakdown.log) -- each half's
        // fit runs 1.2 rounds of the resident workgroups and its grid half as many blocks, so the tails grow, not shrink
        auto all = [&](int md) -> int {
            const bool timed = flags & CRIMP_FLAG_TIME_KERNELS;
            const bool overlap = run_brute && !timed && nint >= 2 * 512 && getenv("CRIMP_TOA_OVERLAP") != nullptr;
            if (!overlap) {
                KernelTimer kg(s, timed);  // brute grid: k_toa_grid(_mf) + k_toa_grid_best
                kg.start();
                if (run_brute) {
                    const int r2 = run_brute(md, s, 0, nint);
                    if (r2) return r2;
                }
                if (run_brute) kg.stop();
                KernelTimer kf(s, timed);  // the fit kernel
                kf.start();
                fit(s, 0, nint);
                HIPCHK(hipGetLastError());
                kf.stop();
                return CRIMP_OK;
            }
            hipStream_t s1 = aux_stream();
            if (!s1) return set_err(CRIMP_ERR_HIP, "cannot create the auxiliary stream");
            hipEvent_t e0 = nullptr, e1 = nullptr;
            HIPCHK(hipEventCreateWithFlags(&e0, hipEventDisableTiming));
            HIPCHK(hipEventCreateWithFlags(&e1, hipEventDisableTiming));
            const int64_t h = nint / 2;
            int r2 = run_brute(md, s, 0, h);
            if (!r2) {
                HIPCHK(hipEventRecord(e0, s));
                fit(s, 0, h);
                HIPCHK(hipGetLastError());
                HIPCHK(hipStreamWaitEvent(s1, e0, 0));
                r2 = run_brute(md, s1, h, nint - h);
            }
            if (!r2) {
                fit(s1, h, nint - h);
                HIPCHK(hipGetLastError());
                HIPCHK(hipEventRecord(e1, s1));
                HIPCHK(hipStreamWaitEvent(s, e1, 0));
            }
            (void)hipEventDestroy(e0);  // destruction waits for nothing; the events complete in stream order
            (void)hipEventDestroy(e1);
            return r2;
        };
        ht.mark("setup");
        if (hist_pending) {  // redChi2's histogram on the auxiliary stream, beside the grid and the fits
            hipStream_t s1 = aux_stream();
            if (!s1) return set_err(CRIMP_ERR_HIP, "cannot create the auxiliary stream");
            EventGuard e0;
            HIPCHK(hipEventCreateWithFlags(&e0.e, hipEventDisableTiming));
            HIPCHK(hipEventRecord(e0.e, s));
            HIPCHK(hipStreamWaitEvent(s1, e0.e, 0));
            k_binphases<<<dim3((unsigned)nint, (unsigned)bin_splits(hoff[nint], nint)), 64 * kBinWaves, 0, s1>>>(
                dx, doff, dedg, rq->nbins, dcnt);
            HIPCHK(hipGetLastError());
            HIPCHK(hipEventCreateWithFlags(&ebin.e, hipEventDisableTiming));
            HIPCHK(hipEventRecord(ebin.e, s1));
        }
        rc = all(grid_mode);
        if (rc) return rc;
        ht.mark("launch");
        if (run_brute && (grid_mode & kGridProd8) && !(grid_mode & kGridNoMin)) {
            // the runtime half of the certificates (eight factors, lazy norms): a flagged lattice point reruns the
            // grid and the fits with the full four-factor kernel
            int unsafe = 0;
            HIPCHK(d2h(s, &unsafe, dunsafe, sizeof(int)));
            HIPCHK(hipStreamSynchronize(s));
            if (unsafe) {
                rc = all(grid_mode & ~(kGridProd8 | kGridCert));
                if (rc) return rc;
            }
        }
        ht.mark("unsafe");
        if (rq) {  // redChi2 from the final records
            if (ebin.e) HIPCHK(hipStreamWaitEvent(s, ebin.e, 0));
            k_toa_chi2<<<(unsigned)nint, 64, 0, s>>>(dcnt, T, de, dout, dcen, rq->nbins, rq->nfree, dred);
            HIPCHK(hipGetLastError());
            HIPCHK(copy_back(s, rq->out, dred, (size_t)nint, dev));
        }
        HIPCHK(copy_back(s, out, dout, (size_t)nint * 8, dev));
        HIPCHK(hipStreamSynchronize(s));
        ht.mark("chi2+sync");
    }
    return finish(s, flags);
}

extern "C" int crimp_toa_fit(const double* x, const int64_t* offsets, int64_t nint, const crimp_template* tpl,
                             const double* exposure, double norm0, int32_t ph_shift_res, int32_t options, double* out,
                             uint32_t flags, void* stream) {
    return toa_fit_impl(x, offsets, nint, tpl, exposure, norm0, ph_shift_res, options, out, flags, stream, nullptr);
}

extern "C" int crimp_toa_fit_redchi2(const double* x, const int64_t* offsets, int64_t nint, const crimp_template* tpl,
                                     const double* exposure, double norm0, int32_t ph_shift_res, int32_t options,
                                     const double* edges, const double* centers, int32_t nbins, int32_t nfree,
                                     double* out, double* redchi2, uint32_t flags, void* stream) {
    ARGCHK(nbins >= 1 && nbins <= 256, "bad sizes (nbins must be 1..256)");
    ARGCHK(edges != nullptr && centers != nullptr && redchi2 != nullptr, "null argument");
    const RedChi2Req rq{edges, centers, nbins, nfree, redchi2};
    return toa_fit_impl(x, offsets, nint, tpl, exposure, norm0, ph_shift_res, options, out, flags, stream, &rq);
}

extern "C" int crimp_toa_grid(const double* x, const int64_t* offsets, int64_t nint, const crimp_template* tpl,
                              const double* norm, int64_t nnorm, const double* phi, int64_t nphi, double* lnsum,
                              double* hmin, uint32_t flags, void* stream) {
    ARGCHK(nint >= 1 && nnorm >= 1 && nphi >= 1, "bad sizes");
    ARGCHK(nphi <= (1 << 24) && nnorm <= (1 << 20), "grid too large");
    ARGCHK(x != nullptr && offsets != nullptr && norm != nullptr && phi != nullptr && lnsum != nullptr &&
               hmin != nullptr,
           "null argument");
    TplDev T;
    int rc = make_tpl(tpl, &T);
    if (rc) return rc;
    ARGCHK(T.K <= kGridKMax, "brute grid supports at most 8 template components");
    std::lock_guard<std::mutex> lk(g_mutex);
    if (flags & CRIMP_FLAG_TIME_KERNELS) {
        g_kernel_times.clear();
        g_last_kernel_ms = -1.0;
    }
    const bool dev = flags & CRIMP_FLAG_DEVICE_PTRS;
    hipStream_t s = as_stream(stream);
    std::vector<int64_t> hoff((size_t)nint + 1);
    if (dev) {
        HIPCHK(d2h(s, hoff.data(), offsets, (nint + 1) * sizeof(int64_t)));
        HIPCHK(hipStreamSynchronize(s));
    } else {
        std::memcpy(hoff.data(), offsets, (nint + 1) * sizeof(int64_t));
    }
    int64_t maxn = 0;
    for (int64_t i = 0; i < nint; ++i) {
        ARGCHK(hoff[i + 1] >= hoff[i] && hoff[i] >= 0, "offsets must be non-decreasing");
        maxn = std::max(maxn, hoff[i + 1] - hoff[i]);
    }
    {
        Scratch sc(s);
        const double *dx = nullptr, *dnrm = nullptr, *dphi = nullptr;
        const int64_t* doff = nullptr;
        HIPCHK(stage_in(sc, x, (size_t)hoff[nint], dev, &dx));
        HIPCHK(stage_in(sc, offsets, (size_t)nint + 1, dev, &doff));
        HIPCHK(stage_in(sc, norm, (size_t)(nint * nnorm), dev, &dnrm));
        HIPCHK(stage_in(sc, phi, (size_t)nphi, dev, &dphi));
        ARGCHK(nint <= 65535, "at most 65535 intervals per brute-grid call");
        TplDev* dT = nullptr;
        HIPCHK(sc.alloc(&dT, 1));
        HIPCHK(h2d(dT, &T, sizeof(T)));
        double *pl = nullptr, *ph = nullptr;
        int64_t splits = 0;
        rc = toa_grid_partials(sc, s, dx, doff, dT, T, dnrm, nnorm, dphi, nphi, nint, maxn, &pl, &ph, &splits);
        if (rc) return rc;
        // combine splits on the host in a fixed order (deterministic)
        std::vector<double> hl((size_t)(splits * nint * nnorm * nphi)), hh((size_t)(splits * nint * nphi));
        HIPCHK(d2h(s, hl.data(), pl, hl.size() * sizeof(double)));
        HIPCHK(d2h(s, hh.data(), ph, hh.size() * sizeof(double)));
        HIPCHK(hipStreamSynchronize(s));
        const int64_t L = nint * nnorm * nphi, H = nint * nphi;
        std::vector<double> rl((size_t)L), rh((size_t)H);
        for (int64_t k = 0; k < L; ++k) {
            double v = 0.0;
            for (int64_t sp = 0; sp < splits; ++sp) v += hl[(size_t)(sp * L + k)];
            rl[(size_t)k] = v * 0.69314718055994530942;  // log2 -> ln
        }
        for (int64_t k = 0; k < H; ++k) {
            double v = INFINITY;
            for (int64_t sp = 0; sp < splits; ++sp) v = std::min(v, hh[(size_t)(sp * H + k)]);
            rh[(size_t)k] = v;
        }
        if (dev) {
            HIPCHK(h2d(lnsum, rl.data(), L * sizeof(double)));
            HIPCHK(h2d(hmin, rh.data(), H * sizeof(double)));
            HIPCHK(hipStreamSynchronize(s));
        } else {
            std::memcpy(lnsum, rl.data(), L * sizeof(double));
            std::memcpy(hmin, rh.data(), H * sizeof(double));
        }
    }
    return finish(s, flags);
}

extern "C" int crimp_toa_shape_points(const double* x, const int64_t* offsets, int64_t nint, const crimp_template* tpls,
                                      const double* aux, const int64_t* pt_interval, const double* pt_norm,
                                      const double* pt_phi, int64_t npts, double* out, uint32_t flags, void* stream) {
    ARGCHK(nint >= 1 && npts >= 0, "bad sizes");
    ARGCHK(x != nullptr && offsets != nullptr && tpls != nullptr && pt_interval != nullptr && pt_norm != nullptr &&
               pt_phi != nullptr && out != nullptr,
           "null argument");
    ARGCHK(npts <= 2147483647LL, "too many points");
    if (npts == 0) return CRIMP_OK;
    // templates and point intervals are host arrays (checked here); photons, norms, phases and out may be device
    for (int64_t p = 0; p < npts; ++p) {
        ARGCHK(tpls[p].ncomp >= 1 && tpls[p].ncomp <= CRIMP_MAX_COMP, "ncomp out of range");
        ARGCHK(tpls[p].model >= 0 && tpls[p].model <= 2, "unknown template model");
        ARGCHK(pt_interval[p] >= 0 && pt_interval[p] < nint, "point interval out of range");
    }
    std::lock_guard<std::mutex> lk(g_mutex);
    if (flags & CRIMP_FLAG_TIME_KERNELS) {
        g_kernel_times.clear();
        g_last_kernel_ms = -1.0;
    }
    const bool dev = flags & CRIMP_FLAG_DEVICE_PTRS;
    hipStream_t s = as_stream(stream);
    std::vector<int64_t> hoff((size_t)nint + 1);
    if (dev) {
        HIPCHK(d2h(s, hoff.data(), offsets, (nint + 1) * sizeof(int64_t)));
        HIPCHK(hipStreamSynchronize(s));
    } else {
        std::memcpy(hoff.data(), offsets, (nint + 1) * sizeof(int64_t));
    }
    for (int64_t i = 0; i < nint; ++i) ARGCHK(hoff[i + 1] >= hoff[i] && hoff[i] >= 0, "offsets must be non-decreasing");
    {
        Scratch sc(s);
        const double *dx = nullptr, *dn = nullptr, *dp = nullptr;
        const int64_t* doff = nullptr;
        double* dout = nullptr;
        HIPCHK(stage_in(sc, x, (size_t)hoff[nint], dev, &dx));
        HIPCHK(stage_in(sc, offsets, (size_t)nint + 1, dev, &doff));
        HIPCHK(stage_in(sc, pt_norm, (size_t)npts, dev, &dn));
        HIPCHK(stage_in(sc, pt_phi, (size_t)npts, dev, &dp));
        HIPCHK(stage_out(sc, out, (size_t)npts * kShapeSums, dev, &dout));
        crimp_template* dT = nullptr;
        int64_t* dpi = nullptr;
        double* daux = nullptr;
        HIPCHK(sc.alloc(&dT, (size_t)npts));
        HIPCHK(sc.alloc(&dpi, (size_t)npts));
        HIPCHK(h2d(dT, tpls, npts * sizeof(crimp_template)));
        HIPCHK(h2d(dpi, pt_interval, npts * sizeof(int64_t)));
        if (aux != nullptr) {
            HIPCHK(sc.alloc(&daux, (size_t)npts * CRIMP_MAX_COMP));
            HIPCHK(h2d(daux, aux, npts * CRIMP_MAX_COMP * sizeof(double)));
        }
        // one launch per run of points sharing a model (the kernel is specialised per model)
        for (int64_t p0 = 0; p0 < npts;) {
            int64_t p1 = p0 + 1;
            while (p1 < npts && tpls[p1].model == tpls[p0].model) ++p1;
            const unsigned nb = (unsigned)(p1 - p0);
            const double* da = daux != nullptr ? daux + p0 * CRIMP_MAX_COMP : nullptr;
            if (tpls[p0].model == CRIMP_MODEL_FOURIER)
                k_toa_shape<CRIMP_MODEL_FOURIER><<<nb, kShapeBlock, 0, s>>>(dx, doff, dT + p0, da, dpi + p0, dn + p0,
                                                                            dp + p0, dout + p0 * kShapeSums);
            else if (tpls[p0].model == CRIMP_MODEL_CAUCHY)
                k_toa_shape<CRIMP_MODEL_CAUCHY><<<nb, kShapeBlock, 0, s>>>(dx, doff, dT + p0, da, dpi + p0, dn + p0,
                                                                           dp + p0, dout + p0 * kShapeSums);
            else
                k_toa_shape<CRIMP_MODEL_VONMISES><<<nb, kShapeBlock, 0, s>>>(dx, doff, dT + p0, da, dpi + p0, dn + p0,
                                                                             dp + p0, dout + p0 * kShapeSums);
            p0 = p1;
        }
        HIPCHK(hipGetLastError());
        HIPCHK(copy_back(s, out, dout, (size_t)npts * kShapeSums, dev));
        HIPCHK(hipStreamSynchronize(s));
    }
    return finish(s, flags);
}

// redChi2 of every fitted interval on the device (measureToAs.py:385-393 and the Cauchy / von Mises copies): against
// binphases' histogram (k_binphases, np.histogram semantics) the best-fit template curve at the bin centres;
// chi2 = sum_b (model_b - rate_b)^2 / err_b^2 with rate = cts / (E / nbins), err = sqrt(cts) / (E / nbins) (numpy's
// division: an empty bin gives inf, or nan where the model is 0 too), summed in bin order, redChi2 = chi2 / (nbins -
// nfree). One 64-thread block per interval; rec = the fit records (norm [0], phShift [1], ampShift [6]).
__global__ __launch_bounds__(64) void k_toa_chi2(const unsigned long long* __restrict__ counts, const TplDev T,
                                                 const double* __restrict__ expo, const double* __restrict__ rec,
                                                 const double* __restrict__ centers, int nb, int nfree,
                                                 double* __restrict__ out) {
    __shared__ double term[256];
    const int64_t iv = blockIdx.x;
    const double n = rec[iv * 8], ph = rec[iv * 8 + 1], A = rec[iv * 8 + 6];
    const double w = expo[iv] / (double)nb;
    for (int b = threadIdx.x; b < nb; b += 64) {
        const double xx = centers[b];
        double y = n;  // toafit.ToAFitter.curve: fourseries / wrapcauchy / vonmises (templatemodels.py:64-82, :166-185,
                       // :271-290); Fourier by angle subtraction as the host formed it
        for (int j = 0; j < T.K; ++j) {
            if (T.model == CRIMP_MODEL_FOURIER) {
                const double ang = (double)(j + 1) * 2.0 * M_PI * xx + T.loc[j], bph = (double)(j + 1) * ph;
                y = y + T.amp[j] * A * (cos(ang) * cos(bph) + sin(ang) * sin(bph));
            } else if (T.model == CRIMP_MODEL_CAUCHY) {
                y = y + T.amp[j] * A / (T.ch[j] - cos(xx - T.loc[j] - ph));
            } else {
                y = y + T.amp[j] * A * exp(T.kap[j] * cos(xx - T.loc[j] - ph));
            }
        }
        const double c = (double)counts[iv * nb + b];
        const double rate = c / w, err = sqrt(c) / w;
        term[b] = ((y - rate) * (y - rate)) / (err * err);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double chi2 = 0.0;
        for (int b = 0; b < nb; ++b) chi2 += term[b];
        out[iv] = chi2 / (double)(nb - nfree);
    }
}

extern "C" int crimp_toa_redchi2(const double* x, const int64_t* offsets, int64_t nint, const crimp_template* tpl,
                                 const double* exposure, const double* records, const double* edges,
                                 const double* centers, int32_t nbins, int32_t nfree, double* out, uint32_t flags,
                                 void* stream) {
    ARGCHK(nint >= 1 && nbins >= 1 && nbins <= 256, "bad sizes (nbins must be 1..256)");
    ARGCHK(x != nullptr && offsets != nullptr && exposure != nullptr && records != nullptr && edges != nullptr &&
               centers != nullptr && out != nullptr, "null argument");
    ARGCHK(nint <= 2147483647LL, "too many intervals");
    TplDev T;
    int rc = make_tpl(tpl, &T);
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(g_mutex);
    if (flags & CRIMP_FLAG_TIME_KERNELS) {
        g_kernel_times.clear();
        g_last_kernel_ms = -1.0;
    }
    const bool dev = flags & CRIMP_FLAG_DEVICE_PTRS;
    hipStream_t s = as_stream(stream);
    int64_t ntot = 0;
    if (dev) {
        HIPCHK(d2h(s, &ntot, offsets + nint, sizeof(int64_t)));
        HIPCHK(hipStreamSynchronize(s));
    } else {
        ntot = offsets[nint];
    }
    {
        Scratch sc(s);
        const double *dx = nullptr, *de = nullptr, *dc = nullptr, *dexp = nullptr, *drec = nullptr;
        const int64_t* doff = nullptr;
        double* dout = nullptr;
        unsigned long long* dcnt = nullptr;
        HIPCHK(stage_in(sc, x, (size_t)ntot, dev, &dx));
        HIPCHK(stage_in(sc, offsets, (size_t)nint + 1, dev, &doff));
        HIPCHK(stage_in(sc, exposure, (size_t)nint, dev, &dexp));
        HIPCHK(stage_in(sc, records, (size_t)nint * 8, dev, &drec));
        HIPCHK(stage_in(sc, edges, (size_t)nbins + 1, dev, &de));
        HIPCHK(stage_in(sc, centers, (size_t)nbins, dev, &dc));
        HIPCHK(stage_out(sc, out, (size_t)nint, dev, &dout));
        HIPCHK(sc.alloc(&dcnt, (size_t)(nint * nbins)));
        HIPCHK(hipMemsetAsync(dcnt, 0, (size_t)(nint * nbins) * sizeof(unsigned long long), s));
        const int64_t ns = bin_splits(ntot, nint);
        KernelTimer kt(s, flags & CRIMP_FLAG_TIME_KERNELS);
        kt.start();
        k_binphases<<<dim3((unsigned)nint, (unsigned)ns), 64 * kBinWaves, 0, s>>>(dx, doff, de, nbins, dcnt);
        k_toa_chi2<<<(unsigned)nint, 64, 0, s>>>(dcnt, T, dexp, drec, dc, nbins, nfree, dout);
        HIPCHK(hipGetLastError());
        kt.stop();
        HIPCHK(copy_back(s, out, dout, (size_t)nint, dev));
    }
    return finish(s, flags);
}

extern "C" int crimp_binphases(const double* x, const int64_t* offsets, int64_t nint, const double* edges,
                               int32_t nbins, int64_t* counts, uint32_t flags, void* stream) {
    ARGCHK(nint >= 1 && nbins >= 1 && nbins <= 256, "bad sizes (nbins must be 1..256)");
    ARGCHK(x != nullptr && offsets != nullptr && edges != nullptr && counts != nullptr, "null argument");
    ARGCHK(nint <= 2147483647LL, "too many intervals");
    std::lock_guard<std::mutex> lk(g_mutex);
    if (flags & CRIMP_FLAG_TIME_KERNELS) {
        g_kernel_times.clear();
        g_last_kernel_ms = -1.0;
    }
    const bool dev = flags & CRIMP_FLAG_DEVICE_PTRS;
    hipStream_t s = as_stream(stream);
    int64_t ntot = 0;
    if (dev) {
        HIPCHK(d2h(s, &ntot, offsets + nint, sizeof(int64_t)));
        HIPCHK(hipStreamSynchronize(s));
    } else {
        ntot = offsets[nint];
    }
    {
        Scratch sc(s);
        const double *dx = nullptr, *de = nullptr;
        const int64_t* doff = nullptr;
        int64_t* dc = nullptr;
        HIPCHK(stage_in(sc, x, (size_t)ntot, dev, &dx));
        HIPCHK(stage_in(sc, offsets, (size_t)nint + 1, dev, &doff));
        HIPCHK(stage_in(sc, edges, (size_t)nbins + 1, dev, &de));
        HIPCHK(stage_out(sc, counts, (size_t)(nint * nbins), dev, &dc));
        const int64_t ns = bin_splits(ntot, nint);
        HIPCHK(hipMemsetAsync(dc, 0, (size_t)(nint * nbins) * sizeof(int64_t), s));
        k_binphases<<<dim3((unsigned)nint, (unsigned)ns), 64 * kBinWaves, 0, s>>>(
            dx, doff, de, nbins, reinterpret_cast<unsigned long long*>(dc));
        HIPCHK(hipGetLastError());
        HIPCHK(copy_back(s, counts, dc, (size_t)(nint * nbins), dev));
    }
    return finish(s, flags);
}

// ============================================================== 7. interval selection (measureToAs.py:168-182)
// The photons of a ToA interval are TIME[(TIME >= start) & (TIME <= end)] (measureToAs.py:173-174); on time-sorted
// photons (event files are) that is the range [lower_bound(start), upper_bound(end)) -- two binary searches per
// interval instead of a pass over all photons per interval. crimp_is_sorted decides which applies.
__global__ __launch_bounds__(256) void k_unsorted(const double* __restrict__ t, int64_t n, int* __restrict__ flag) {
    constexpr int U = 4;  // pairs per thread and sweep, loads issued together
    int b = 0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i0 + 1 < n; i0 += U * stride) {
        double a[U], c[U];
#pragma unroll
        for (int q = 0; q < U; ++q) {
            const int64_t i = i0 + q * stride;
            a[q] = t[i + 1 < n ? i : 0];
            c[q] = t[i + 1 < n ? i + 1 : 0];
        }
#pragma unroll
        for (int q = 0; q < U; ++q)
            if (i0 + q * stride + 1 < n) b |= !(a[q] <= c[q]);  // a NaN is out of order, as np.all(T[1:] >= T[:-1])
    }
    if (__any(b) && (threadIdx.x & 63) == 0) atomicOr(flag, 1);
}

// lo[i] = first photon with t >= starts[i] (np.searchsorted side="left"), count[i] = photons up to the last with
// t <= ends[i] (side="right") less lo[i], at least 0; first_last[2i], [2i+1] = t of the interval's first and last
// photon (NaN when it holds none). A NaN bound selects nothing, as the reference's mask.
__global__ __launch_bounds__(256) void k_select_intervals(const double* __restrict__ t, int64_t n,
                                                          const double* __restrict__ starts,
                                                          const double* __restrict__ ends, int64_t nint,
                                                          int64_t* __restrict__ lo, int64_t* __restrict__ count,
                                                          double* __restrict__ first_last) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nint) return;
    const double s = starts[i], e = ends[i];
    int64_t a = 0, b = n;
    while (a < b) {  // lower bound of s
        const int64_t m = (a + b) >> 1;
        if (t[m] < s) a = m + 1; else b = m;
    }
    const int64_t l = a;
    b = n;
    while (a < b) {  // upper bound of e, from l
        const int64_t m = (a + b) >> 1;
        if (t[m] <= e) a = m + 1; else b = m;
    }
    const int64_t c = (s == s && e == e && a > l) ? a - l : 0;
    lo[i] = l;
    count[i] = c;
    if (first_last) {
        first_last[2 * i] = c > 0 ? t[l] : NAN;
        first_last[2 * i + 1] = c > 0 ? t[l + c - 1] : NAN;
    }
}

// out[offsets[i] + j] = t[lo[i] + j], j < offsets[i+1] - offsets[i]: the intervals' photons concatenated
__global__ __launch_bounds__(256) void k_gather_ranges(const double* __restrict__ t, const int64_t* __restrict__ lo,
                                                       const int64_t* __restrict__ offsets, double* __restrict__ out) {
    const int64_t i = blockIdx.x;
    const int64_t o = offsets[i], len = offsets[i + 1] - o;
    const double* src = t + lo[i];
    for (int64_t j = threadIdx.x; j < len; j += blockDim.x) out[o + j] = src[j];
}

extern "C" int crimp_is_sorted(const double* t, int64_t n, int32_t* unsorted, uint32_t flags, void* stream) {
    ARGCHK(n >= 0, "n < 0");
    ARGCHK(unsorted != nullptr && (t != nullptr || n == 0), "null argument");
    *unsorted = 0;
    if (n < 2) return CRIMP_OK;
    const bool dev = flags & CRIMP_FLAG_DEVICE_PTRS;
    std::lock_guard<std::mutex> lk(g_mutex);
    hipStream_t s = as_stream(stream);
    {
        Scratch sc(s);
        const double* dt = nullptr;
        int* dflag = nullptr;
        HIPCHK(stage_in(sc, t, (size_t)n, dev, &dt));
        HIPCHK(sc.alloc(&dflag, 1));
        HIPCHK(hipMemsetAsync(dflag, 0, sizeof(int), s));
        k_unsorted<<<(unsigned)std::min<int64_t>(cdiv(n, 256 * 4), 2048), 256, 0, s>>>(dt, n, dflag);
        HIPCHK(hipGetLastError());
        int h = 0;
        HIPCHK(d2h(s, &h, dflag, sizeof(int)));
        *unsorted = h ? 1 : 0;
    }
    return finish(s, flags);
}

extern "C" int crimp_select_intervals(const double* t, int64_t n, const double* starts, const double* ends,
                                      int64_t nint, int64_t* lo, int64_t* count, double* first_last, uint32_t flags,
                                      void* stream) {
    ARGCHK(n >= 0 && nint >= 0, "negative size");
    ARGCHK((t != nullptr || n == 0) && (nint == 0 || (starts && ends && lo && count)), "null argument");
    if (nint == 0) return CRIMP_OK;
    const bool dev = flags & CRIMP_FLAG_DEVICE_PTRS;
    std::lock_guard<std::mutex> lk(g_mutex);
    hipStream_t s = as_stream(stream);
    {
        Scratch sc(s);
        const double *dt = nullptr, *ds = nullptr, *de = nullptr;
        int64_t *dlo = nullptr, *dc = nullptr;
        double* dfl = nullptr;
        HIPCHK(stage_in(sc, t, (size_t)n, dev, &dt));
        HIPCHK(stage_in(sc, starts, (size_t)nint, dev, &ds));
        HIPCHK(stage_in(sc, ends, (size_t)nint, dev, &de));
        HIPCHK(stage_out(sc, lo, (size_t)nint, dev, &dlo));
        HIPCHK(stage_out(sc, count, (size_t)nint, dev, &dc));
        if (first_last) HIPCHK(stage_out(sc, first_last, (size_t)(2 * nint), dev, &dfl));
        k_select_intervals<<<(unsigned)cdiv(nint, 256), 256, 0, s>>>(dt, n, ds, de, nint, dlo, dc, dfl);
        HIPCHK(hipGetLastError());
        HIPCHK(copy_back(s, lo, dlo, (size_t)nint, dev));
        HIPCHK(copy_back(s, count, dc, (size_t)nint, dev));
        if (first_last) HIPCHK(copy_back(s, first_last, dfl, (size_t)(2 * nint), dev));
    }
    return finish(s, flags);
}

extern "C" int crimp_gather_ranges(const double* t, int64_t n, const int64_t* lo, const int64_t* offsets,
                                   int64_t nint, double* out, uint32_t flags, void* stream) {
    ARGCHK(n >= 0 && nint >= 0, "negative size");
    ARGCHK(nint <= 2147483647LL, "too many intervals");
    ARGCHK(nint == 0 || (t && lo && offsets && out), "null argument");
    if (nint == 0) return CRIMP_OK;
    const bool dev = flags & CRIMP_FLAG_DEVICE_PTRS;
    std::lock_guard<std::mutex> lk(g_mutex);
    hipStream_t s = as_stream(stream);
    // the ranges are checked on the host against the photon array before any copy is queued
    std::vector<int64_t> hlo((size_t)nint), hoff((size_t)nint + 1);
    if (dev) {
        HIPCHK(d2h(s, hlo.data(), lo, (size_t)nint * sizeof(int64_t)));
        HIPCHK(d2h(s, hoff.data(), offsets, ((size_t)nint + 1) * sizeof(int64_t)));
    } else {
        std::memcpy(hlo.data(), lo, (size_t)nint * sizeof(int64_t));
        std::memcpy(hoff.data(), offsets, ((size_t)nint + 1) * sizeof(int64_t));
    }
    ARGCHK(hoff[0] == 0, "offsets[0] must be 0");
    for (int64_t i = 0; i < nint; ++i) {
        const int64_t len = hoff[(size_t)i + 1] - hoff[(size_t)i];
        ARGCHK(len >= 0 && hlo[(size_t)i] >= 0 && hlo[(size_t)i] + len <= n, "a range lies outside the photon array");
    }
    const int64_t total = hoff[(size_t)nint];
    {
        Scratch sc(s);
        const double* dt = nullptr;
        const int64_t *dlo = nullptr, *doff = nullptr;
        double* dout = nullptr;
        HIPCHK(stage_in(sc, t, (size_t)n, dev, &dt));
        HIPCHK(stage_in(sc, lo, (size_t)nint, dev, &dlo));
        HIPCHK(stage_in(sc, offsets, (size_t)nint + 1, dev, &doff));
        HIPCHK(stage_out(sc, out, (size_t)total, dev, &dout));
        k_gather_ranges<<<(unsigned)nint, 256, 0, s>>>(dt, dlo, doff, dout);
        HIPCHK(hipGetLastError());
        HIPCHK(copy_back(s, out, dout, (size_t)total, dev));
    }
    return finish(s, flags);
}

/*
 * crimp_hip.h -- C-ABI of the MI355X-native CRIMP photon hot path (libcrimp_hip.so).
 *
 * The reference (georgeyounes/CRIMP v2.3.0) is pure Python with no FFI; its
 * "operator API" is the Python functions listed per entry point below. Each entry
 * point replaces the NumPy inner loops of one of them; the Python drop-ins in
 * crimp_amd/ keep the reference signatures and call these through ctypes.
 *
 * Conventions (all entry points):
 *   - return 0 (CRIMP_OK) or a negative status; crimp_last_error() gives the text
 *     (thread-local, valid until the next call on the same thread);
 *   - every buffer is caller-owned; with CRIMP_FLAG_DEVICE_PTRS all array
 *     arguments are device pointers on the current HIP device, otherwise they are
 *     host pointers and the library stages them through device memory itself;
 *   - `stream` is a hipStream_t (NULL = the null stream); kernels are queued on it
 *     and every call returns with that stream drained (host staging copies are
 *     blocking), so results are ready on return -- CRIMP_FLAG_SYNC is accepted and
 *     implied;
 *   - calls are serialised process-wide, all devices together (one internal mutex:
 *     the scratch pool and the measurement hooks are shared); the ctypes layer
 *     releases the GIL around them, so threads driving different devices queue.
 */
#ifndef CRIMP_HIP_H
#define CRIMP_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CRIMP_OK 0
#define CRIMP_ERR_ARG (-1)
#define CRIMP_ERR_HIP (-2)
#define CRIMP_ERR_NODEV (-3)

#define CRIMP_FLAG_DEVICE_PTRS 1u  /* array arguments are device pointers */
#define CRIMP_FLAG_SYNC 2u         /* synchronise the stream before returning */
/* Periodicity-search precision. Default: the NUFFT (search_nufft.h) on arithmetic-progression grids (ascending)
 * of >= 64 trials per row segment with time-sorted photons and a plan in range -- every trial certified within 1e-6
 * relative by a truncation bound, the uncertified ones recomputed in fp64 (crimp_last_fixups()). Where the NUFFT
 * declines: the exact i8-MFMA kernel on progressions of >= 256 trials (per-term error ~1e-9, integer sums; trials
 * whose 10-sigma bound cannot place them within 1e-6 relative are recomputed in fp64), the fp64 kernel otherwise.
 * crimp_last_search_path() says which ran. Tested within 1e-6 of the reference on every checked trial; the
 * reference's own fp64 argument rounding (~1e-6 of a noise-level H_20) is the floor of any fp64 implementation
 * (DESIGN.md section 8). */
#define CRIMP_FLAG_FORCE_MFMA 8u   /* search: fail unless a factorised kernel (NUFFT, or exact i8 MFMA at any row
                                    * length) applies */
#define CRIMP_FLAG_TIME_KERNELS 128u /* search / calcphase: time the kernels with hipEvents (crimp_last_kernel_ms) */
#define CRIMP_FLAG_F64 256u         /* search: fp64 kernel on every grid */
#define CRIMP_FLAG_NO_FIXUP 1024u   /* search (diagnostic): the exact kernel's / the NUFFT's raw powers, without the
                                       fp64 fix-up of the trials their error bound cannot certify (crimp_last_fixups
                                       counts them) */
/* Bits 4, 16 and 512 selected the fp32 "fast" search (round 1-4), retired in round 5: slower than the default exact
 * path and only within 1e-6 of the grid's mean power. A search call that sets any of them fails with CRIMP_ERR_ARG. */
#define CRIMP_FLAG_RETIRED_FAST (4u | 16u | 512u)
#define CRIMP_FLAG_ASYNC 2048u     /* crimp_search_sets with device pointers: return once the kernel is queued, without
                                     * draining the stream (the caller synchronises it before reading out) */

#define CRIMP_FLAG_NUFFT 4096u     /* search: the default routing, asked for explicitly (the NUFFT wherever it applies,
                                    * the exact rule otherwise); kept for callers of rounds 5 and earlier */
#define CRIMP_FLAG_EXACT 8192u     /* search: no NUFFT -- the exact i8-MFMA kernel on progressions of >= 256 trials,
                                    * the fp64 kernel otherwise (the default of rounds 1-5) */

#define CRIMP_FLAG_TIME_DAYS 16384u    /* crimp_search_sets: t in days (MJD); the kernel forms t * 86400 seconds as
                                        * measureToAs.py:211 does on the host (the same fp64 multiply) */
#define CRIMP_FLAG_FOLD_RADIANS 32768u /* crimp_calcphase: the folded phase times 2 pi (radians), the host's
                                        * `folded * (2 * np.pi)` of measureToAs.py:195, :200 in the same multiply */

#define CRIMP_STAT_Z2 0 /* Z^2_m  (periodsearch.py:57-71, :73-106) */
#define CRIMP_STAT_H 1  /* H-test (periodsearch.py:109-125)         */

#define CRIMP_MODEL_FOURIER 0  /* templatemodels.py:24-121, x in cycles  */
#define CRIMP_MODEL_CAUCHY 1   /* templatemodels.py:124-226, x in rad    */
#define CRIMP_MODEL_VONMISES 2 /* templatemodels.py:229-329, x in rad    */

#define CRIMP_MAX_GLITCH 32
#define CRIMP_MAX_WAVE 64
#define CRIMP_MAX_COMP 16

/* Values of a .par timing model as calcphase consumes them
 * (readtimingmodel.py:212-233; calcphase.py:73-149). */
typedef struct crimp_timing_model {
    double pepoch;                          /* PEPOCH (MJD) */
    double f[13];                           /* F0..F12; absent ones 0 */
    int32_t n_glitch;                       /* glitches 1..n (count of GLEP_ keys, calcphase.py:94) */
    double glitch[CRIMP_MAX_GLITCH][7];     /* GLEP, GLPH, GLF0, GLF1, GLF2, GLF0D, GLTD */
    int32_t n_wave;                         /* WAVE harmonics used = (#WAVE* keys) - 2 (calcphase.py:142) */
    double wave_epoch, wave_om;             /* WAVEEPOCH (MJD), WAVE_OM (rad/day) */
    double wave_ab[CRIMP_MAX_WAVE][2];      /* WAVEj A, B */
} crimp_timing_model;

/* A pulse-profile template (readPPtemplate.py:15-166) with its fixed shape. */
typedef struct crimp_template {
    int32_t model;                   /* CRIMP_MODEL_* */
    int32_t ncomp;                   /* harmonics / components, 1..CRIMP_MAX_COMP */
    double amp[CRIMP_MAX_COMP];      /* amp_j */
    double loc[CRIMP_MAX_COMP];      /* ph_j (fourier) or cen_j (cauchy, vonmises) */
    double wid[CRIMP_MAX_COMP];      /* wid_j (cauchy, vonmises) */
    double i0[CRIMP_MAX_COMP];       /* scipy.special.i0(1/wid_j^2) (vonmises) */
    double amp_shift;                /* ampShift (1 unless varied) */
} crimp_template;

/* Library identification. */
int crimp_version(void);
const char* crimp_last_error(void);
/* Duration (ms, hipEvents on the call's stream) of the harmonic-sum kernels of the last crimp_search, or of
 * the kernel of the last crimp_calcphase, made with CRIMP_FLAG_TIME_KERNELS; -1 if none. Measurement hook for
 * bench.py, not in the reference. */
double crimp_last_kernel_ms(void);
/* All timed spans of the last call made with CRIMP_FLAG_TIME_KERNELS (ms, in order: crimp_search -> the
 * harmonic-sum kernels; crimp_calcphase -> the kernel; crimp_toa_fit -> the brute grid, the fit kernel); writes
 * up to cap values, returns how many there are. Measurement hook for bench.py, not in the reference. */
int crimp_last_kernel_times(double* ms, int32_t cap);
/* Trials of the last crimp_search (default precision) whose power was recomputed by the fp64 fix-up. */
int64_t crimp_last_fixups(void);
/* Kernel family of the last crimp_search: 0 fp64 direct, 1 exact i8 MFMA, 2 NUFFT. With
 * CRIMP_FLAG_TIME_KERNELS a NUFFT search's crimp_last_kernel_times are: the whole pipeline, then the summed ms of its
 * seven kernel classes (cell starts, spread, merge, FFT pass 1, FFT pass 2, Horner sum, finalize), then their launch
 * counts. Measurement hook for tests and bench.py, not in the reference. */
int crimp_last_search_path(void);
/* The plan of the last NUFFT search: its (largest) FFT length n, moments P, and spread form (1 = cell gather, one lane
 * per wrapped cell on the VALU; 0 = MFMA slots). Measurement hook for bench.py, not in the reference. */
int crimp_last_nufft_plan(int64_t* fft_length, int32_t* moments, int32_t* gather);
/* The last NUFFT search's algorithmic work, up to cap of: [0] the spread's fp64 flops, then HBM bytes of [1] the
 * spread, [2] merge, [3] FFT pass 1, [4] FFT pass 2 (with the fused Horner sum), [5] the separate Horner sum, [6]
 * finalize; returns 7. For bench.py's rooflines, not in the reference. */
int crimp_last_nufft_work(double* work, int32_t cap);
/* Brute-grid norms evaluated per phShift by the last crimp_toa_fit with CRIMP_TOA_BRUTE (the pruned candidates of
 * lmfit's 20-norm lattice, padded to 2, 4 or 20, less the lazy norms the eight-factor grid leaves out; 0 without a
 * brute grid). Measurement hook for bench.py's
 * algorithmic work count, not in the reference. */
int64_t crimp_last_toa_grid_norms(void);
/* The form of the last crimp_toa_fit's brute grid (Fourier templates): bit 0 -- no per-phShift min of the template
 * part (the template's bound certified every candidate lattice point valid), bit 1 -- log2 of products of eight model
 * values instead of four (every factor certified inside [2^-15, 2^15]); 0 = the full kernel. Measurement hook for
 * bench.py, not in the reference. */
int64_t crimp_last_toa_grid_fast(void);
/* Frees the library's idle cached device scratch on every device (not in the reference). */
int crimp_release_scratch(void);
int crimp_device_count(int32_t* count);

/* calcphase(timeMJD, timMod) -> (total, folded)   [calcphase.py:152-176]
 * parts: bit0 Taylor expansion (:73-85), bit1 glitches (:87-126), bit2 waves (:128-149);
 * 7 = calcphase(). folded may be NULL. */
int crimp_calcphase(const double* t_mjd, int64_t n, const crimp_timing_model* model, int32_t parts,
                    double* total, double* folded, uint32_t flags, void* stream);

/* PeriodSearch(time, freq, nbrHarm).ztest()/.htest()/.twod_ztest(freq_dot)
 *   [periodsearch.py:40-125]
 * t: photon times (s) [n]; t0: (t[0]+t[n-1])/2 as periodsearch.py:54 (passed explicitly so that
 * shards of one search share it); freq [nf] (Hz); log10_negfdot [nfd] or NULL (1-D); the trial
 * grid is fd-outer/f-inner (periodsearch.py:264-278) and this call computes flat trials
 * [first, first+count) of it into out[count]. stat = CRIMP_STAT_Z2 or CRIMP_STAT_H (the latter
 * over the 2-D grid is this library's extension). Precision: the CRIMP_FLAG_F64 / _NUFFT notes
 * above; the kernel is chosen from the whole grid (nf, nfd, progression), not from [first, count), so a sharded
 * search computes every trial exactly as an unsharded one -- except that the NUFFT (the default) plans each row
 * segment of [first, count) on its own (a shard of a row is its own progression, so it costs its share): whole rows are
 * bit-identical, a cut row agrees within the plans' ~1e-13 error. */
int crimp_search(const double* t, int64_t n, double t0, const double* freq, int64_t nf,
                 const double* log10_negfdot, int64_t nfd, int32_t nharm, int32_t stat, int64_t first,
                 int64_t count, double* out, uint32_t flags, void* stream);

/* crimp_search and the best trial of its powers in one call: out[count] as crimp_search, best[0] = the largest of
 * out, best[1] = its index within [first, first+count) as a double (np.argmax semantics, as crimp_best), best a host
 * pointer. A NUFFT search reads the best trial back with its fix-up count (one stream sync less than crimp_search +
 * crimp_best; sharding.sharded_search(gather='best')). */
int crimp_search_best(const double* t, int64_t n, double t0, const double* freq, int64_t nf,
                      const double* log10_negfdot, int64_t nfd, int32_t nharm, int32_t stat, int64_t first,
                      int64_t count, double* out, double* best, uint32_t flags, void* stream);

/* Best trial of a power array x[n] (crimp_search's out): best[0] = max, best[1] = its index as a double (exact:
 * n <= 2^53), np.argmax semantics -- ties to the lowest index, NaN above every number   [the maximum the
 * reference's callers take of PeriodSearch's powers; sharding.sharded_search(gather='best')]. best is a host
 * pointer; with CRIMP_FLAG_DEVICE_PTRS x is device memory (else host, staged). One stream sync. */
int crimp_best(const double* x, int64_t n, double* best, uint32_t flags, void* stream);

/* Many one-trial searches at once: for every set i, PeriodSearch(t[offsets[i]:offsets[i+1]], [freq[i]],
 * nbrHarm).htest() / .ztest()   [periodsearch.py:40-125 as measureToAs.py:210-212 calls it per ToA interval;
 * t0 = (first + last)/2 of each set, :54]. t in seconds; out[nset]. fp64 (the reference's precision). */
int crimp_search_sets(const double* t, const int64_t* offsets, int64_t nset, const double* freq, int32_t nharm,
                      int32_t stat, double* out, uint32_t flags, void* stream);

/* Fourier|WrappedCauchy|VonMises(theta, x).loglikelihood{FS,CA,VM}normalized(exposure) and its
 * (norm, phShift) derivatives at arbitrary points   [templatemodels.py:98-121, 201-226, 306-329].
 * x: folded phases of all intervals concatenated, interval i = x[offsets[i] : offsets[i+1]]
 * (cycles for fourier, radians otherwise). Point p is (pt_interval[p], pt_norm[p], pt_phi[p]).
 * out[p*8 + 0..7] = { sum ln(norm + h), sum q, sum h' q, -sum q^2, -sum h' q^2,
 *                     sum (h'' q - h'^2 q^2), min(norm + h), N }   with q = 1/(norm + h),
 * h = model - norm, primes = d/dphShift. fp64 throughout. Host assembles the reference LL. */
int crimp_toa_points(const double* x, const int64_t* offsets, int64_t nint, const crimp_template* tpl,
                     const int64_t* pt_interval, const double* pt_norm, const double* pt_phi, int64_t npts,
                     double* out, uint32_t flags, void* stream);

/* lmfit 'brute' grid of measureToA_* (measureToAs.py:292-295, defineinitialfitparam :698-806):
 * for every interval i, norm a, phShift b:
 *   lnsum[(i*nnorm + a)*nphi + b] = sum_photons ln(norm[i*nnorm+a] + h(x; phi[b]))
 *   hmin[i*nphi + b]              = min_photons h(x; phi[b])
 * fp32 model + logarithm, fp64 accumulation; a Fourier template's part on the f16 matrix cores with every fp32
 * factor split hi + lo (fp32-level products), the likelihood part on the VALU. */
int crimp_toa_grid(const double* x, const int64_t* offsets, int64_t nint, const crimp_template* tpl,
                   const double* norm, int64_t nnorm, const double* phi, int64_t nphi, double* lnsum,
                   double* hmin, uint32_t flags, void* stream);

#define CRIMP_TOA_BRUTE 1      /* crimp_toa_fit options: lmfit brute start (measureToAs.py:292-295, -bm) */
#define CRIMP_TOA_VARY_AMPS 2  /* ampShift free in [0.01, 100] after the first fit (measureToAs.py:305-312, -va) */

/* measureToA_fourier / _cauchy / _vonmises(tempModPP, phases, exposure, phShiftRes=res, brutemin=...,
 * varyAmps=...) for every interval at once, readvaryparam=False   [measureToAs.py:254-693, :698-806]:
 * optional lmfit brute start (20 norms in [norm0/100, 500] x phShift = k*0.05 - bound), the extended-LL
 * maximum in (norm, phShift) -- and ampShift with CRIMP_TOA_VARY_AMPS --, and the 1-sigma scan in steps of
 * 2pi/res with the other free parameters re-profiled at each step. One workgroup per interval runs the
 * whole fit on the device (csrc/toa_fit.h).
 * out[i*8 + 0..6] = { norm, phShift, LLmax, phShift_LL, phShift_UL, likelihood evaluations, ampShift }.
 * The reduced chi2 (:385-393) is crimp_toa_redchi2 on these records (or crimp_toa_fit_redchi2: both at once). */
int crimp_toa_fit(const double* x, const int64_t* offsets, int64_t nint, const crimp_template* tpl,
                  const double* exposure, double norm0, int32_t ph_shift_res, int32_t options, double* out,
                  uint32_t flags, void* stream);

/* Extended-LL sums with template-shape gradients, for fits that free template parameters
 * (readvaryparam, measureToAs.py:727-801 with the likelihoods of templatemodels.py:98-121, 201-226,
 * 306-329). Point p is interval pt_interval[p] with its own template tpls[p] (ampShift applied),
 * norm pt_norm[p] and phShift pt_phi[p]; aux[p*CRIMP_MAX_COMP + j] = I1(k)/I0(k), k = 1/wid_j^2
 * (vonmises; may be NULL otherwise). With m = norm + h the model at a photon:
 * out[p*CRIMP_SHAPE_SUMS + ...] = { sum ln m, min m, sum 1/m, sum (dh/dphShift)/m,
 *     then for j < CRIMP_MAX_COMP: sum (dh/damp_j)/m, sum (dh/dloc_j)/m, sum (dh/dwid_j)/m }
 * (loc = ph_j or cen_j; unused components and the Fourier wid terms are 0). fp64. */
#define CRIMP_SHAPE_SUMS (4 + 3 * CRIMP_MAX_COMP)
int crimp_toa_shape_points(const double* x, const int64_t* offsets, int64_t nint, const crimp_template* tpls,
                           const double* aux, const int64_t* pt_interval, const double* pt_norm,
                           const double* pt_phi, int64_t npts, double* out, uint32_t flags, void* stream);

/* redChi2 of every fitted interval   [measureToAs.py:385-393 (Fourier), :530-538, :675-683; binphases.py:9-39]:
 * the binned profile (np.histogram with edges[nbins+1] = numpy.linspace(0, upper, nbins+1), upper 1 (Fourier, cycles)
 * or 2 pi) against the template curve at centers[nbins] with the interval's fitted norm, phShift and ampShift from
 * records[i*8 + 0, 1, 6] (crimp_toa_fit's records): out[i] = sum_b (model_b - rate_b)^2 / err_b^2 / (nbins - nfree),
 * rate = cts / (E_i / nbins), err = sqrt(cts) / (E_i / nbins). fp64. */
int crimp_toa_redchi2(const double* x, const int64_t* offsets, int64_t nint, const crimp_template* tpl,
                      const double* exposure, const double* records, const double* edges, const double* centers,
                      int32_t nbins, int32_t nfree, double* out, uint32_t flags, void* stream);

/* crimp_toa_fit and crimp_toa_redchi2 in one call (the whole measureToA_* of every interval, :254-393): the same
 * records in out[i*8 + 0..6] and the same redchi2[i]. The histogram needs only the photons, so it runs on a second
 * stream beside the brute grid and the fits (with CRIMP_FLAG_TIME_KERNELS: after them). */
int crimp_toa_fit_redchi2(const double* x, const int64_t* offsets, int64_t nint, const crimp_template* tpl,
                          const double* exposure, double norm0, int32_t ph_shift_res, int32_t options,
                          const double* edges, const double* centers, int32_t nbins, int32_t nfree, double* out,
                          double* redchi2, uint32_t flags, void* stream);

/* binphases(phases, nbrBins) counts per interval   [binphases.py:9-39]:
 * np.histogram(x, bins=edges) semantics with edges[nbins+1] (numpy.linspace). counts[i*nbins+b]. */
int crimp_binphases(const double* x, const int64_t* offsets, int64_t nint, const double* edges, int32_t nbins,
                    int64_t* counts, uint32_t flags, void* stream);

/* Interval selection of measureToAs (measureToAs.py:168-182): TIME[(TIME >= start) & (TIME <= end)] per ToA interval
 * (:173-174) and its first / last photon (ToA_mid, :182).
 * crimp_is_sorted: *unsorted = 1 if some t[i+1] < t[i] (or a NaN), else 0 (host int; t host or device per flags).
 * crimp_select_intervals: on time-sorted t, lo[i] = np.searchsorted(t, starts[i], "left"), count[i] =
 *   max(np.searchsorted(t, ends[i], "right") - lo[i], 0) (0 for a NaN bound), first_last[2i], [2i+1] = the
 *   interval's first and last time (NaN if empty; may be NULL) -- the mask's photons on sorted times.
 * crimp_gather_ranges: out[offsets[i] + j] = t[lo[i] + j] for j < offsets[i+1] - offsets[i] (offsets[0] = 0; every
 *   range inside t[0, n)): the intervals' photons concatenated, as measureToAs.py's per-interval selections. */
int crimp_is_sorted(const double* t, int64_t n, int32_t* unsorted, uint32_t flags, void* stream);
int crimp_select_intervals(const double* t, int64_t n, const double* starts, const double* ends, int64_t nint,
                           int64_t* lo, int64_t* count, double* first_last, uint32_t flags, void* stream);
int crimp_gather_ranges(const double* t, int64_t n, const int64_t* lo, const int64_t* offsets, int64_t nint,
                        double* out, uint32_t flags, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* CRIMP_HIP_H */

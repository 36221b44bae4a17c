"""Benchmark: Z^2_2 photon x trial evaluations per second (BASELINE.json metric, config 3), plus the exact-path,
ToA-fit, calcphase, config-4 and config-2 legs.

One step = one complete Z^2_2 search of the config-3 workload per GPU: 1e7 synthetic pulsed photons (T = 1e6 s,
p = 0.1, f0 = 7.123456789 Hz, seed 0, time-sorted as event files are) against 1e6 trial frequencies spaced 1/(10T),
inputs resident in HBM, followed by the search's one exchange step (every rank's best trial gathered so that all
ranks agree on the global best, ties -> lowest index). With N ranks each rank searches its own 1e6-trial slice of
an N*1e6 grid (weak scaling); ``value`` = all ranks' evaluations / max-over-ranks time. The step is the search call
without a precision keyword -- what the reference's own ``PeriodSearch(time, freq, 2).ztest()`` reaches: the
default NUFFT (csrc/search_nufft.h: Chebyshev-moment non-uniform FFT in fp64, every trial within 1e-6 of the
reference by its truncation-bound certificate + fp64 fix-up, tests/test_gpu_nufft.py, test_gpu_fullsize.py);
``--precision exact`` times the exact-integer MFMA path instead. The unit says "equivalent": evaluations are the
photon x trial pairs the reference evaluates directly, and the NUFFT returns the same per-trial powers without
evaluating every pair (``exact_path`` and ``cpu_baseline`` do evaluate every pair).

Also reported:
* ``roofline``: the NUFFT's dominant kernel class, its algorithmic work per launch (crimp_last_nufft_work) over the
  mean launch time (hipEvents on the library's stream); every class under ``nufft.kernels``;
* ``exact_path``: the default exact-integer path (k_search_exact) on the same inputs, ``--exact-steps`` steps, with
  its i8 matrix-core roofline: per 4 photons x 2048 trials x harmonic it issues 8 dense v_mfma_i32_32x32x32_i8
  (65536 ops each) and 4 2:4-sparse v_smfmac_i32_32x32x64_i8 (131072 nominal ops each) = 128 ops per
  photon*trial*harmonic, against the 6.67 POP/s peak of that 2:1 mix; ``traffic`` from the tree's rocprofv3 PMC pass
  (profiles/r04/pmc_traffic.json) when it was taken on this workload;
* ``cpu_baseline``: the oracle (oracle/liborc.so, fp64 direct sums, OpenMP over trials) on a bounded sample;
* ToA (config 5 per GPU): the device fit of 1250 intervals x 1e5 photons, and the end-to-end ``measure_intervals``
  (interval selection, calcphase, fits, per-interval H-test) from host MJD arrays, with the oracle's fits on all
  allowed host cores as its CPU baseline (a sample, extrapolated) and the fits' VALU roofline;
* ``config4``: 1e8 photons, 2-D H_20 on a sub-grid of the 1e7-trial grid (131072 trials per GPU), sharded_search;
  ``config4.nufft``: the WHOLE 1e7-trial grid by the default search (the NUFFT; each rank its 1e7/N slice);
* ``config2``: ``measureToAs`` on the bundled events, ToAs 35-41, FITS -> table (the reference's published rate).
The multi-GPU paths are the tested ones (tests/test_distributed_*.py): the search step and the config-4 leg run
``sharding.sharded_search(gather="best")``, the ToA leg ``sharding.sharded_toa_fit`` (records all_gathered).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# MI355X_MICROARCH.md: I8 MFMA dense = 2x BF16 (2.5 PF) = 5.0 POP/s, 2:4 sparse 2x that; the exact kernel issues
# 2 dense : 1 sparse instructions at 32 cycles each, so its mix peaks at (2 x 5.0 + 1 x 10.0) / 3 POP/s
PEAK_I8_TOPS = (2 * 5000.0 + 10000.0) / 3
OPS_PER_EVAL_HARM = 128.0       # (8 x 65536 dense + 4 x 131072 sparse ops) per 4 photons x 2048 trials x harmonic
PEAK_HBM_GBS = 8000.0           # MI355X_MICROARCH.md: HBM3E ~8 TB/s
PEAK_VALU_SLOTS = 256 * 4 * 32 * 2.4e9   # fp32 lane-ops/s: 256 CUs x 4 SIMD-32 x 2.4 GHz
PEAK_F64_OPS = 256 * 64 * 2.4e9          # fp64 FMA-rate lane-ops/s: half the fp32 rate (78.6 TFLOP/s fp64 vector)
PEAK_F16_TFLOPS = 2500.0                 # MI355X_MICROARCH.md: dense F16/BF16 MFMA ~2.5 PFLOP/s
PMC_FILE = os.path.join(ROOT, "profiles", "r04", "pmc_traffic.json")
PMC_NUFFT_FILE = os.path.join(ROOT, "profiles", "r06", "pmc_nufft_traffic.json")
# the kernel behind each NUFFT class on the config-3 plan (cell gather, n1 = 256 columns, 4096-element rows)
NUFFT_CLASS_KERNEL = {"cellstart": "k_nu_cellstart", "spread": "k_nu_gather", "pass1": "k_nu_cols256",
                      "pass2": "k_nu_rows_iw", "finalize": "k_nu_finalize"}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--settle", type=float, default=0.3,
                   help="seconds of untimed steps before the warmup steps (GPU clocks back at steady state)")
    p.add_argument("--photons", type=int, default=10_000_000)
    p.add_argument("--trials", type=int, default=1_000_000, help="trial frequencies per GPU")
    p.add_argument("--nharm", type=int, default=2)
    p.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline legs")
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--precision", default="default", choices=["default", "nufft", "exact"],
                   help="the search path of `value`: default = no precision keyword (the NUFFT where it applies); "
                        "the exact path is timed beside it")
    p.add_argument("--exact-steps", type=int, default=3, help="timed steps of the exact-path leg (~0.8 s each)")
    p.add_argument("--no-exact", action="store_true", help="skip the exact-path leg (when value is nufft)")
    p.add_argument("--toa-intervals", type=int, default=1250, help="ToA intervals per GPU (config 5: 1e4 over 8)")
    p.add_argument("--toa-photons", type=int, default=100_000)
    p.add_argument("--no-toa", action="store_true", help="skip the ToA legs")
    p.add_argument("--full-c5", type=int, default=10_000, help="N=1: intervals of the whole-config-5 fit (0: skip)")
    p.add_argument("--calcphase-photons", type=int, default=100_000_000)
    p.add_argument("--no-calcphase", action="store_true", help="skip the calcphase (HBM-bound) leg")
    p.add_argument("--no-config2", action="store_true", help="skip the config-2 measureToAs leg")
    p.add_argument("--no-config4", action="store_true", help="skip the config-4 (1e8 photons, H_20) leg")
    p.add_argument("--c4-photons", type=int, default=100_000_000)
    p.add_argument("--c4-trials", type=int, default=131072, help="config-4 trials timed per GPU (even)")
    p.add_argument("--no-nufft-c4", action="store_true", help="skip the whole-grid config-4 NUFFT search")
    return p.parse_args()


def host_cores():
    """CPU threads this process may use: its affinity set, capped by OMP_NUM_THREADS when the host sets it (the
    GPU box gives each GPU 16 of the machine's CPUs), and the machine's count for the record."""
    try:
        allowed = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        allowed = os.cpu_count() or 1
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return (min(allowed, omp) if omp > 0 else allowed), os.cpu_count()


# 1E 2259+586 Fourier template (data/1e2259_template.txt), config 5 draws intervals from it
T2259 = {"model": "fourier", "norm": {"value": 17.060771467236613},
         "amp": [1.508994969593123, 4.055594828231136, 1.4384785819368275, 0.3505348524380939,
                 0.19725727340744187, 0.3483402644535841],
         "ph": [-0.4071967961461897, -0.8051383329477251, 0.5157949575544241, 1.9295783704947946,
                -0.1917798112304259, 0.8297144204463391]}


def _tmpl():
    tm = {"model": "fourier", "norm": T2259["norm"]}
    for j, (am, ph) in enumerate(zip(T2259["amp"], T2259["ph"]), start=1):
        tm["amp_%d" % j] = {"value": am}
        tm["ph_%d" % j] = {"value": ph}
    return tm


def toa_leg(a, dev, world, rank):
    """Config 5 (per GPU): intervals x photons drawn from the 1e2259 template with random true shifts,
    brute grid + exact MLE + 1-sigma scan + redChi2 per interval (measureToA_fourier -bm).
    (1) device fit of phases resident in HBM: ``warmup`` untimed fits, then the mean of up to 3 timed fits;
    (2) end to end from host MJD arrays: measure_intervals (the upload of the times in blocks beside the device work
        of the previous block, interval selection, calcphase, the fits, the per-interval H_5), one untimed call, then
        the mean of up to 3 timed calls."""
    import torch
    import torch.distributed as dist
    from crimp_amd.synth import template_intervals_torch
    from crimp_amd.toafit import ToAFitter
    from crimp_amd import _native as N
    from crimp_amd.measureToAs import measure_intervals
    from crimp_amd.sharding import interval_shard, sharded_toa_fit
    tm = _tmpl()
    # one global interval set of world x toa_intervals intervals (weak scaling); rank r's block [r n, (r+1) n) is
    # drawn with seed 2 + r, so every rank generates only the photons it fits (sharding.interval_shard)
    nint_g = a.toa_intervals * world
    off_g = np.arange(nint_g + 1, dtype=np.int64) * a.toa_photons
    E_g = np.full(nint_g, a.toa_photons / T2259["norm"]["value"])
    x, off, E, shifts = template_intervals_torch(a.toa_intervals, a.toa_photons, T2259["norm"]["value"],
                                                 T2259["amp"], T2259["ph"], seed=2 + rank, device=dev)
    first, count, pa, pb = interval_shard(off_g, world, rank)
    assert (first, count) == (rank * a.toa_intervals, a.toa_intervals)

    def rank_photons(lo, hi):  # sharded_toa_fit's loader: this rank's block only
        assert (lo, hi) == (pa, pb)
        return x

    for _ in range(max(a.warmup, 0)):  # untimed: code-object load, scratch-pool growth
        res = ToAFitter(x, off, E, tm).fit(brutemin=True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    reps = max(1, min(a.steps, 3))
    t1 = time.perf_counter()
    for _ in range(reps):  # the tested multi-GPU path: each rank fits its block, one all_gather of the records
        allrec = sharded_toa_fit(rank_photons, off_g, E_g, tm, brutemin=True)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t1) / reps
    assert allrec["phShi"].size == nint_g and np.array_equal(allrec["phShi"][first:first + count], res["phShi"])
    # kernel split of one fit (hipEvents around the brute-grid and the fit kernels inside crimp_toa_fit)
    from crimp_amd import ops
    f = ToAFitter(x, off, E, tm)
    edges, pp = f._bins()
    ops.toa_fit_redchi2(f.x, f.offsets, f.tpl, f._arr(f.E, np.float64), f.norm0, f.res, True, False,
                        f._arr(edges, np.float64), f._arr(pp, np.float64), 2, flags=N.FLAG_TIME_KERNELS)
    grid_ms, fit_ms = N.last_kernel_times()[:2]
    elt = torch.tensor([el], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(elt, op=dist.ReduceOp.MAX)
    d = np.angle(np.exp(1j * (res["phShi"] - shifts)))  # recovered vs true shift, wrapped
    out = {"toa_fits_per_s": a.toa_intervals * world / float(elt.item()),
           "toa_config": "config5: %d intervals/GPU x %d photons, Fourier K=6 (1e2259), brute+MLE+1-sigma scan+redChi2; "
                         "sharding.sharded_toa_fit over %d ranks (all_gather of the records in the timed region)"
                         % (a.toa_intervals, a.toa_photons, world),
           "toa_seconds": float(elt.item()),
           "toa_mean_likelihood_evaluations": float(np.mean(res["evaluations"])),
           "toa_shift_recovery_rms_cycles": float(np.sqrt(np.mean(d ** 2)) / (2 * np.pi)),
           "toa_median_sigma_cycles": float(np.median(res["phShi_LL"]) / (2 * np.pi)),
           "toa_kernel_ms": {"k_toa_grid": grid_ms, "k_toa_fit": fit_ms}}
    # Algorithmic work (SURVEY.md section 8d's lane-slot model). Brute grid (k_toa_grid_mf): the
    # template part h of every photon x phShift point is a (photons x 2K) . (2K x phShifts) product on the f16 matrix
    # cores (each fp32 factor as hi + lo f16, four products per term: 8K f16 MACs per point, padded to 16 per pair of
    # harmonics); the VALU does the likelihood part, one min and per evaluated norm an add, 3/4 of a multiply, 1/4 of a
    # quarter-rate v_log_f32 (4 slots) and 1/4 of an add: S_grid = 1 + 3 NN fp32 lane-op slots per point, NN = norms
    # evaluated per phShift (the pruned candidates, crimp_last_toa_grid_norms); fp32 peak = 256 CUs x 4 SIMDs x 32
    # lanes x 2.4 GHz = 7.86e13 lane-ops/s. Fit: per photon and likelihood pass, in fp64
    # operations (FMA rate, half the fp32 rate: 3.93e13/s): table sin/cos 14, per harmonic the Chebyshev step (2)
    # and h, h', h'' (7) = 9K, the model add 1, the reciprocal 5 (v_rcp_f64 + two Newton steps), ln as 1/8 of a fp64
    # log (~29) + a multiply = 4.6, 6 sums and fmin 9 -> S_full = 33 + 9K (the Newton ascent's passes); the first
    # pass of each 1-sigma-scan norm profile forms h alone (5 per harmonic, 3 sums): S_store = 27 + 5K; a pass that
    # reads the cached template part: S_cached = 13 (the add, reciprocal, ln, two sums and fmin). Passes per interval
    # from the fit's own counters: cached ones in out[7]; one store pass per scan step, kk - 1 per side where the
    # side's sigma is kk step + step / 2.
    K = len(T2259["amp"])
    nn = int(N.load().crimp_last_toa_grid_norms())
    gmode = int(N.load().crimp_last_toa_grid_fast())   # bits: 1 no min h, 2 log2 per eight model values, 4 certificate
    nphi = 126
    nph_tot = float(a.toa_intervals) * a.toa_photons
    # per point: the min (1, unless bit 0) and per norm an add, (P-1)/P multiply, 1/P of a 4-slot v_log_f32 and 1/P add;
    # with one evaluated norm on the eight-factor kernel the add is done by the MFMA (accumulators start at the norm)
    P = 8 if gmode & 2 else 4
    cin = bool(gmode & 2) and nn == 1
    s_grid = (0 if gmode & 5 else 1) + nn * ((0 if cin else 1) + (P - 1) / P + 5.0 / P)
    g_slots = nph_tot * nphi * s_grid
    g_ach = g_slots / (grid_ms * 1e-3)
    g_mf = nph_tot * nphi * 2 * 16 * ((K + 1) // 2) / (grid_ms * 1e-3)   # f16 matrix FLOP/s issued
    valu = {"achieved": g_ach / 1e12, "peak": PEAK_VALU_SLOTS / 1e12, "unit": "Tlane-op/s (fp32)",
            "frac": g_ach / PEAK_VALU_SLOTS}
    matrix = {"achieved": g_mf / 1e12, "peak": PEAK_F16_TFLOPS, "unit": "TFLOP/s (f16 dense)",
              "frac": g_mf / 1e12 / PEAK_F16_TFLOPS}
    # the headline is the unit nearer its peak: the VALU likelihood part until round 4, the matrix-core template since
    # the eight-factor kernel, the norm-initialised accumulators and the lazy-norm certificate took the VALU's share
    head, other = (matrix, ("valu", valu)) if matrix["frac"] >= valu["frac"] else (valu, ("matrix", matrix))
    out["toa_roofline"] = dict({"kernel": "k_toa_grid_mf", "bound": "mfma" if head is matrix else "valu"}, **head)
    out["toa_roofline"].update({"norms_evaluated": nn, "slots_per_photon_phshift": s_grid, "grid_mode": gmode,
                                other[0]: other[1],
                                "note": "S_grid = [min] + NN ([1] + (P-1)/P + 5/P) fp32 lane-op slots per photon x phShift "
                                   "(log2 of products of P = 4 or 8 model values, v_log_f32 at 4; the add of the norm "
                                   "not counted where the MFMA accumulators start at it: P = 8, NN = 1) beside "
                                   "the template on v_mfma_f32_32x32x16_f16 (hi/lo f16 split, 16 MACs per pair of "
                                   "harmonics), x 1250 x 1e5 photons x 126 phShifts / brute-grid hipEvent time "
                                   "(k_toa_grid_mf + k_toa_grid_best); peaks 256 CU x 4 SIMD x 32 lanes x 2.4 GHz, "
                                   "f16 dense 2.5 PFLOP/s"})
    fev = np.asarray(res["evaluations"], dtype=np.float64)
    fca = np.asarray(res["cached_evaluations"], dtype=np.float64)
    step = 2 * np.pi / f.res
    kl = np.rint((res["phShi_LL"] - step / 2) / step) - 1  # scan profiles per side
    ku = np.rint((res["phShi_UL"] - step / 2) / step) - 1
    fst = kl + ku
    fjo = 2 * np.minimum(kl, ku)  # profiles evaluated two per joint pass (both sides active)
    fnw = fev - fca - fst
    # a scan profile's first pass: the moment pass (S_1..S_5, no cached passes) or, in the CRIMP_FIT_MOMENTS=0
    # build, the pass that stores h for the cached passes
    # (CRIMP_FIT_MOMENTS=0 build) or, for a step of both sides in one joint pass, the shared sin/cos and recurrence
    # (14 + 2K) once and each side's template and moment work (3K + 19) per profile: 26 + 4K per profile
    if np.any(fca > 0):
        s_scan, fjo = 27 + 5 * K, 0 * fjo
    else:
        s_scan = 33 + 5 * K
    f_ops = float(np.sum(fnw * (33 + 9 * K) + (fst - fjo) * s_scan + fjo * (26 + 4 * K) + fca * 13) * a.toa_photons)
    f_ach = f_ops / (fit_ms * 1e-3)
    out["toa_fit_roofline"] = {"kernel": "k_toa_fit", "bound": "valu", "achieved": f_ach / 1e12,
                               "peak": PEAK_F64_OPS / 1e12, "unit": "Tlane-op/s (fp64)", "frac": f_ach / PEAK_F64_OPS,
                               "newton_passes_per_interval": float(np.mean(fnw)),
                               "scan_profiles_per_interval": float(np.mean(fst)),
                               "joint_pass_profiles_per_interval": float(np.mean(fjo)),
                               "cached_passes_per_interval": float(np.mean(fca)),
                               "scan_pass_ops": s_scan,
                               "note": "S_full = 33 + 9K fp64 ops per photon and Newton pass, S_scan = 33 + 5K for a "
                                       "scan profile's moment pass, 26 + 4K per profile of a joint two-side moment pass "
                                       "(27 + 5K for the h-storing pass of the iterative profile), S_cached = 13 for a pass over its cached template part; passes from the fit's own counters / "
                                       "k_toa_fit hipEvent time; peak fp64 FMA rate 256 CU x 64 lanes x 2.4 GHz"}
    # end to end from host arrays: photon times t = (cycle + phase) / F0 around PEPOCH, intervals bracketing them
    F0, pep = 0.5, 58000.0
    cyc = torch.arange(x.numel(), device=dev, dtype=torch.float64)
    tsec = (cyc + x) / F0
    mjd = (pep + tsec / 86400.0).cpu().numpy()
    offh = off.cpu().numpy()
    starts = mjd[offh[:-1]] - 1e-9
    ends = mjd[offh[1:] - 1] + 1e-9
    del cyc, tsec
    par = {"PEPOCH": pep, "F0": F0}
    for k in range(1, 13):
        par["F%d" % k] = 0.0
    measure_intervals(mjd, par, tm, starts, ends, E, brutemin=True)   # untimed: allocation / code objects
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(reps):
        r2 = measure_intervals(mjd, par, tm, starts, ends, E, brutemin=True)
    torch.cuda.synchronize()
    e2e = (time.perf_counter() - t1) / reps
    out["toa_e2e_fits_per_s"] = a.toa_intervals / e2e
    out["toa_e2e_seconds"] = e2e
    out["toa_e2e_note"] = ("measure_intervals from a host MJD array (%d photons, pageable numpy; toa_e2e_pinned_*: "
                           "from a page-locked torch tensor): upload, interval selection, calcphase, brute+MLE+1-sigma "
                           "fits, redChi2, per-interval H_5 (measureToAs.py:168-226 minus file I/O)" % mjd.size)
    out["toa_e2e_max_shift_diff_vs_device_fit_cycles"] = float(np.max(np.abs(
        np.angle(np.exp(1j * (r2["phShi"] - res["phShi"]))))) / (2 * np.pi))
    # the same from a page-locked host tensor (an event reader's pinned staging buffer): the upload is one DMA
    pin = torch.from_numpy(mjd).pin_memory()
    measure_intervals(pin, par, tm, starts, ends, E, brutemin=True)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(reps):
        r3 = measure_intervals(pin, par, tm, starts, ends, E, brutemin=True)
    torch.cuda.synchronize()
    e2p = (time.perf_counter() - t1) / reps
    assert np.array_equal(r3["phShi"], r2["phShi"])
    out["toa_e2e_pinned_fits_per_s"] = a.toa_intervals / e2p
    out["toa_e2e_pinned_seconds"] = e2p
    del pin, r3
    if not a.no_cpu and rank == 0 and world == 1:  # CPU baselines: rank 0 at N=1 only
        out["toa_cpu_baseline"] = toa_cpu_baseline(x, off, E, tm, a.cpu_seconds)
    if world == 1 and a.full_c5 > 0:  # the whole of config 5 (1e4 intervals x 1e5 photons, 8 GB) on one GPU
        del x, off, r2, mjd, allrec
        torch.cuda.empty_cache()
        t1 = time.perf_counter()
        xf, offf, Ef, _ = template_intervals_torch(a.full_c5, a.toa_photons, T2259["norm"]["value"], T2259["amp"],
                                                   T2259["ph"], seed=12, device=dev)
        torch.cuda.synchronize()
        gen = time.perf_counter() - t1
        ToAFitter(xf, offf, Ef, tm).fit(brutemin=True)   # untimed: scratch-pool growth to the larger sizes
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        rf = ToAFitter(xf, offf, Ef, tm).fit(brutemin=True)
        torch.cuda.synchronize()
        elf = time.perf_counter() - t1
        out["toa_full_config5"] = {"fits_per_s": a.full_c5 / elf, "seconds": elf, "intervals": a.full_c5,
                                   "photons_per_interval": a.toa_photons, "generation_s": gen,
                                   "median_sigma_cycles": float(np.median(rf["phShi_LL"]) / (2 * np.pi)),
                                   "note": "BASELINE config 5 whole (not per GPU) on one GPU: brute+MLE+1-sigma "
                                           "scan+redChi2, phases resident in HBM"}
        del xf, offf, rf
        torch.cuda.empty_cache()
    return out


def toa_cpu_baseline(x, off, E, tm, budget_s):
    """The oracle's measureToA_fourier restatement (fp64 C likelihoods, OpenMP) on every allowed host core over
    the first config-5 intervals until ``budget_s`` has passed; extrapolated as fits/s."""
    from oracle import oracle as O
    cores, visible = host_cores()
    O.set_threads(cores)
    xs = x[: int(off[min(8, off.numel() - 1)])].cpu().numpy()
    oh = off[:9].cpu().numpy()
    t1 = time.perf_counter()
    done = 0
    for i in range(min(8, oh.size - 1)):
        O.fit_toa(xs[oh[i]:oh[i + 1]], E[i], tm, brutemin=True)
        done += 1
        if time.perf_counter() - t1 > budget_s:
            break
    el = time.perf_counter() - t1
    return {"value": done / el, "unit": "ToA fits/s", "cores": cores, "host_cpus_visible": visible, "kind": "port",
            "sample": "%d config-5 intervals (1e5 photons, brute+MLE+1-sigma scan), oracle fit_toa, %.1f s; "
                      "reference log: 0.42 fits/s at 1e4 photons (BASELINE.md)" % (done, el)}


def config2_leg(a):
    """BASELINE config 2, the reference's one published rate: ``measureToAs`` (measureToAs.py:64-251) on the bundled
    1e2259 events (a FITS file written from tests/golden/events_1e2259.npz, the EVENTS rows of
    data/1e2259_ni1020600110.fits), .par, template and interval file, ``-el 1 -eh 5 -bm -ts 35 -te 41``: FITS read,
    energy filter, interval selection, calcphase, 7 brute+MLE+1-sigma fits, H_5, the table, .txt and the residual
    PDF. One untimed call, then the median of 3. The reference's log quotes 84 ToAs in 202 s = 0.42 fits/s
    (data/ToAs_2259.log:1,23); the oracle's fit_toa (fp64 C + SciPy) on the same 7 intervals and host cores sits
    beside it."""
    import tempfile
    import pandas as pd
    from crimp_amd.eventfile import write_events_fits
    from crimp_amd.measureToAs import measureToAs
    from crimp_amd.readPPtemplate import readPPtemplate
    G = os.path.join(ROOT, "tests", "golden")
    ev = np.load(os.path.join(G, "events_1e2259.npz"))
    ref = pd.read_csv(os.path.join(G, "ToAs_2259.txt"), sep=r"\s+", comment="#")
    ref = ref[(ref["ToA"] >= 35) & (ref["ToA"] <= 41)].reset_index(drop=True)
    times = []
    with tempfile.TemporaryDirectory() as d:
        fits = os.path.join(d, "ev.fits")
        write_events_fits(fits, ev["TIME"], ev["PI"], int(ev["MJDREFI"]), float(ev["MJDREFF"]))
        args = (fits, os.path.join(G, "1e2259.par"), os.path.join(G, "1e2259_template.txt"),
                os.path.join(G, "timIntToAs_1e2259.txt"))
        kw = dict(eneLow=1, eneHigh=5, toaStart=35, toaEnd=41, brutemin=True, toaFile=os.path.join(d, "ToAs"))
        tab = measureToAs(*args, **kw)   # untimed: code objects, scratch pool, matplotlib import
        for _ in range(3):
            t1 = time.perf_counter()
            tab = measureToAs(*args, **kw)
            times.append(time.perf_counter() - t1)
    el = float(np.median(times))
    nfit = len(tab)
    dphi = float(np.max(np.abs(tab["phShift"].to_numpy() - ref["phShift"].to_numpy())) / (2 * np.pi))
    out = {"fits_per_s": nfit / el, "seconds": el, "toas": nfit,
           "max_phShift_diff_vs_reference_table_cycles": dphi,
           "phShift_LL_UL_identical_to_reference_table": bool(
               np.array_equal(tab["phShift_LL"].to_numpy(), ref["phShift_LL"].to_numpy()) and
               np.array_equal(tab["phShift_UL"].to_numpy(), ref["phShift_UL"].to_numpy())),
           "reference_log_fits_per_s": 84 / 202.0,
           "note": "measureToAs FITS -> table incl. .txt and residual PDF, ToAs 35-41 of the worked example "
                   "(data/ToAs_2259.txt); reference: 84 ToAs in 202 s (data/ToAs_2259.log:1,23), author's machine"}
    if not a.no_cpu:
        from oracle import oracle as O
        cores, visible = host_cores()
        O.set_threads(cores)
        g = np.load(os.path.join(G, "toa_1e2259.npz"))
        iv = pd.read_csv(os.path.join(G, "timIntToAs_1e2259.txt"), sep=r"\s+", comment="#")
        E = iv["ToA_exposure"].to_numpy()[g["ids"]]
        tm = readPPtemplate(os.path.join(G, "1e2259_template.txt"))
        t1 = time.perf_counter()
        for i in range(len(g["ids"])):
            O.fit_toa(g["folded"][g["offsets"][i]:g["offsets"][i + 1]], E[i], tm, brutemin=True)
        el = time.perf_counter() - t1
        out["cpu_baseline"] = {"value": len(g["ids"]) / el, "unit": "ToA fits/s", "cores": cores,
                               "host_cpus_visible": visible, "kind": "port",
                               "sample": "the same 7 intervals (folded phases of tests/golden/toa_1e2259.npz), oracle "
                                         "fit_toa with brute start, %.1f s" % el}
    return out


def config4_leg(a, dev, world, rank):
    """BASELINE config 4, sharded: 1e8 photons (T = 1e7 s, p = 0.05, fdot = -1e-12, seed 1), 2-D H_20 on the grid of 1e5
    f (step 1/(10 T)) x 100 log10|fdot| rows linspace(-13.5, -11.5, 100) = 1e7 trials. The whole grid takes ~107 s per
    GPU at N = 8 (~14 min at N = 1), so the timed search is its sub-grid of the first ``c4_trials`` / 2 frequencies x
    the first 2 N fdot rows -- ``c4_trials`` trials per GPU -- through sharding.sharded_search(gather="best"), the
    tested multi-GPU path (each rank its contiguous fd-outer slice, one all_gather of the per-rank best). Default
    (exact) path; one untimed search, then one timed; evals/s summed over ranks / max-over-ranks time."""
    import torch
    import torch.distributed as dist
    from crimp_amd import _native as N
    from crimp_amd.sharding import shard_range, sharded_search
    from crimp_amd.synth import pulsed_events
    n, span, f0, fdot, M = a.c4_photons, 1.0e7, 7.123456789, -1.0e-12, 100_000
    nf = a.c4_trials // 2
    t1 = time.perf_counter()
    t_h = pulsed_events(n, span, f0, pulsed_frac=0.05, fdot=fdot, seed=1)
    gen_s = time.perf_counter() - t1
    t = torch.as_tensor(t_h, device=dev)
    del t_h
    f = torch.as_tensor((f0 + (np.arange(M) - M // 2) / (10.0 * span))[:nf], device=dev)
    fd = torch.as_tensor(np.linspace(-13.5, -11.5, 100)[:2 * world], device=dev)
    first, count = shard_range(2 * world * nf, world, rank)
    sharded_search(t, f, 20, 1, freq_dot=fd, gather="best")   # untimed
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    best_pow, best_idx = sharded_search(t, f, 20, 1, freq_dot=fd, gather="best", flags=N.FLAG_TIME_KERNELS)
    torch.cuda.synchronize()
    el = time.perf_counter() - t1
    kms = N.load().crimp_last_kernel_ms()
    nfix = N.load().crimp_last_fixups()
    elt = torch.tensor([el], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(elt, op=dist.ReduceOp.MAX)
    el = float(elt.item())
    ops_launch = OPS_PER_EVAL_HARM * 20 * float(n) * count
    ach = ops_launch / (kms * 1e-3) / 1e12
    nu = None
    if not a.no_nufft_c4:
        # the WHOLE config-4 grid (1e5 f x 100 fdot rows = 1e7 trials, N ranks each its 1e7/N slice) by
        # the default search (the NUFFT): the per-GPU workload of BASELINE config 4, timed end to end
        f_all = torch.as_tensor(f0 + (np.arange(M) - M // 2) / (10.0 * span), device=dev)
        fd_all = torch.as_tensor(np.linspace(-13.5, -11.5, 100), device=dev)
        nu_first, nu_count = shard_range(100 * M, world, rank)
        sharded_search(t, f_all, 20, 1, freq_dot=fd_all, gather="best")  # untimed
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t1 = time.perf_counter()
        nb_pow, nb_idx = sharded_search(t, f_all, 20, 1, freq_dot=fd_all, gather="best")
        torch.cuda.synchronize()
        nel = time.perf_counter() - t1
        elt = torch.tensor([nel], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(elt, op=dist.ReduceOp.MAX)
        nel = float(elt.item())
        nplan = N.last_nufft_plan()
        nrow_, ncol_ = divmod(nb_idx, M)
        nu = {"evals_per_s": float(n) * 100 * M / nel, "unit": "equivalent photon*trial evals/s (H_20)",
              "seconds": nel, "trials_total": 100 * M, "trials_per_gpu": nu_count,
              "search_path": N.load().crimp_last_search_path(), "fp64_fixup_trials": N.load().crimp_last_fixups(),
              "plan": {"fft_length": nplan[0], "moments": nplan[1], "spread": nplan[2]},
              "best_power": nb_pow, "best_trial": {"fdot_row": nrow_, "f_index": ncol_},
              "workload": "config4 WHOLE grid: %.3g photons, H_20, 1e5 f x 100 fdot rows (%d trials per GPU), "
                          "default precision (NUFFT), sharding.sharded_search(gather='best') over %d rank(s)"
                          % (n, nu_count, world)}
        del f_all, fd_all
    del t, f, fd
    torch.cuda.empty_cache()
    row, col = divmod(best_idx, nf)
    return {"evals_per_s": float(n) * count * world / el, "unit": "photon*trial evals/s (H_20)", "seconds": el, "nufft": nu,
            "kernel_ms": kms, "trials_per_gpu_timed": count, "photons": n, "first_flat_trial": first,
            "fp64_fixup_trials": nfix, "best_power": best_pow, "best_trial": {"fdot_row": row, "f_index": col},
            "photon_generation_s": gen_s,
            "roofline": {"bound": "mfma", "achieved": ach, "peak": PEAK_I8_TOPS, "unit": "TFLOP/s",
                         "frac": ach / PEAK_I8_TOPS,
                         "note": "128 int8 matrix ops per photon*trial*harmonic x 20 harmonics / k_search_exact "
                                 "hipEvent time (the harmonic launches of the search)"},
            "workload": "config4 sub-grid: %.3g photons, H_20, first %d f x first %d fdot rows of the 1e5 x 100 grid "
                        "(%d trials per GPU), sharding.sharded_search(gather='best') over %d rank(s)"
                        % (n, nf, 2 * world, count, world)}


def calcphase_leg(a, dev):
    """calcphase (calcphase.py:152-176) over 1e8 photons resident in HBM: 8 B read + 16 B written per photon
    (SURVEY.md section 8d), HBM-bound; hipEvents on the stream the library launches on (torch's current stream)."""
    import torch
    from crimp_amd import ops
    from crimp_amd import _native as N
    n = a.calcphase_photons
    tm = {"PEPOCH": 58000.0, "F0": 7.123456789, "F1": -1.0e-12, "F2": 1.0e-22}
    t = torch.rand(n, dtype=torch.float64, device=dev) * 120.0 + 57940.0   # +-60 d around PEPOCH (MJD)
    tot = torch.empty_like(t)
    fol = torch.empty_like(t)
    for _ in range(2):
        ops.calcphase(t, tm, total=tot, folded=fol)
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    reps = 5
    ev[0].record(stream)
    for _ in range(reps):
        ops.calcphase(t, tm, total=tot, folded=fol)
    ev[1].record(stream)
    torch.cuda.synchronize()
    ms = ev[0].elapsed_time(ev[1]) / reps
    kms = []
    for _ in range(reps):   # the kernel alone: hipEvents around the launch inside libcrimp_hip, on its stream
        ops.calcphase(t, tm, total=tot, folded=fol, flags=N.FLAG_TIME_KERNELS)
        kms.append(N.load().crimp_last_kernel_ms())
    kernel_ms = sum(kms) / len(kms)
    gbs = 24.0 * n / (kernel_ms * 1e-3) / 1e9
    del t, tot, fol
    torch.cuda.empty_cache()
    return {"photons": n, "ms": ms, "photons_per_s": n / (ms * 1e-3),
            "roofline": {"bound": "hbm", "achieved": gbs, "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": gbs / PEAK_HBM_GBS,
                         "kernel_ms": kernel_ms, "call_GBps": 24.0 * n / (ms * 1e-3) / 1e9,
                         "note": "24 algorithmic bytes per photon (8 in, 16 out) / mean k_calcphase_vec duration "
                                 "(hipEvents in libcrimp_hip); call_GBps over the whole C-ABI call"}}


def cpu_baseline(t, f0, df, nharm, budget_s):
    """Oracle (fp64 C restatement of periodsearch.py:57-71, OpenMP over trials) on a bounded sample, on every host
    core this process may use."""
    from oracle import oracle as O
    cores, visible = host_cores()
    O.set_threads(cores)
    n = min(t.size, 1_000_000)
    ts = np.ascontiguousarray(t[:n])
    m = 64
    while True:
        f = f0 + (np.arange(m) - m // 2) * df
        t1 = time.perf_counter()
        O.search(ts, f, nharm)
        el = time.perf_counter() - t1
        if el >= budget_s or m >= 1 << 20:
            break
        m = int(m * min(16.0, max(2.0, 1.2 * budget_s / max(el, 1e-3))))
    rate = n * m / el
    return {"value": rate, "unit": "photon*trial evals/s", "cores": cores, "host_cpus_visible": visible, "kind": "port",
            "sample": "%d photons x %d trials of the same workload, Z^2_%d, oracle/liborc.so fp64, %.1f s" % (
                n, m, nharm, el)}


PEAK_F64_TFLOPS = 78.6  # MI355X spec fp64 (vector and matrix); mb_f64 measures 58 TF VALU FMA, 33.5 TF f64 MFMA


def nufft_leg(a, t, t_h, f, rank, M, steps):
    """The rank's trial slice by the default search (the NUFFT): one untimed search, then ``steps`` timed ones (wall time with the
    stream drained, and the library's hipEvent spans: the whole pipeline and each kernel class's time and launches).
    Each class is priced by the algorithmic work the library counted for the plan it chose (crimp_last_nufft_work;
    DESIGN.md section 5.3):
      spread   fp64 flops: the cell gather's ~40 + 5 P per photon, row and harmonic (k_nu_gather), or the MFMA form's
               issued 512 per photon-harmonic (k_nu_spread), against the fp64 peak;
      merge    HBM: MFMA slots read + the FFT input written (absent for the cell gather, which writes W directly);
      pass1    HBM: the FFT's column pass reading the occupied rows and writing all (k_nu_cols256 / k_nu_fft_cols);
      pass2    HBM: the row pass fused with the Horner sum over moments, reading all and writing one complex sum per
               trial and harmonic (k_nu_rows4096_combine / k_nu_fft_rows_combine);
      finalize HBM: the harmonic sums read, the powers written (k_nu_finalize; absent when the last harmonic's
               pass 2 finalizes, the default, whose extra bytes pass2 then counts).
    The cell starts (k_nu_cellstart) are timed but not priced."""
    import torch
    from crimp_amd import ops
    from crimp_amd import _native as N
    t0 = (t_h[0] + t_h[-1]) / 2
    out = torch.empty(M, dtype=torch.float64, device=t.device)
    ops.search(t, t0, f, a.nharm, 0, first=rank * M, count=M, out=out)
    torch.cuda.synchronize()
    walls, spans = [], []
    for _ in range(steps):
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        ops.search(t, t0, f, a.nharm, 0, first=rank * M, count=M, out=out,
                   flags=N.FLAG_TIME_KERNELS)
        torch.cuda.synchronize()
        walls.append(time.perf_counter() - t2)
        spans.append(N.last_kernel_times()[:15])
    path = N.load().crimp_last_search_path()
    nfix = N.load().crimp_last_fixups()
    wall = float(np.mean(walls))
    sp = np.mean(np.array(spans), axis=0)  # total, then 7 class sums (ms), then 7 launch counts
    n, P, form = N.last_nufft_plan()  # search_nufft.h nu_plan: least n P with 2.4 (x/2)^P/P! <= 5e-14, x = pi (M/2) / n
    w = N.last_nufft_work()
    m = a.nharm
    work = {"spread": (w["spread_flops"], "fp64"), "merge": (w["merge_bytes"], "hbm"), "pass1": (w["pass1_bytes"], "hbm"),
            "pass2": (w["pass2_bytes"], "hbm"), "combine": (w["combine_bytes"], "hbm"),
            "finalize": (w["finalize_bytes"], "hbm")}
    legs = {}
    for c, name in enumerate(N.NUFFT_CLASSES):
        ms, launches = float(sp[1 + c]), int(round(sp[8 + c]))
        if ms <= 0.0 or launches == 0:
            continue  # no such kernel in this plan (the cell gather has no merge)
        leg = {"ms": ms, "launches": launches, "ms_per_launch": ms / launches}
        if name in work and work[name][0] > 0:
            wk, bound = work[name]
            per_launch = wk / launches
            if bound == "fp64":
                leg.update({"bound": bound, "achieved": per_launch / (leg["ms_per_launch"] * 1e-3) / 1e12,
                            "peak": PEAK_F64_TFLOPS, "unit": "TFLOP/s", "work_per_launch": per_launch})
            else:
                leg.update({"bound": bound, "achieved": per_launch / (leg["ms_per_launch"] * 1e-3) / 1e9,
                            "peak": PEAK_HBM_GBS, "unit": "GB/s", "work_per_launch": per_launch})
            leg["frac"] = leg["achieved"] / leg["peak"]
        legs[name] = leg
    # HBM bytes per launch from the tree's PMC pass on this workload (tools/pmc_nufft.sh -> pmc_nufft_traffic.json)
    try:
        pm = json.load(open(PMC_NUFFT_FILE))
        if (pm.get("photons"), pm.get("trials"), pm.get("nharm")) == (a.photons, M, m) and form == "gather":
            for name, leg in legs.items():
                kn = pm["kernels"].get(NUFFT_CLASS_KERNEL.get(name, ""), {})
                if "bytes_per_launch" in kn:
                    leg["traffic"] = kn["bytes_per_launch"]
    except (OSError, ValueError, KeyError):
        pass
    dom = max((k for k in legs if "frac" in legs[k]), key=lambda k: legs[k]["ms"])
    return {"evals_per_s": float(a.photons) * M / wall, "unit": "equivalent photon*trial evals/s (Z^2_%d)" % m,
            "ms_per_search": wall * 1e3, "pipeline_ms": float(sp[0]), "search_path": path, "fp64_fixup_trials": nfix,
            "plan": {"fft_length": n, "moments": P, "spread": form}, "kernels": legs, "dominant": dom,
            "roofline": dict({"kernel": dom}, **legs[dom]),
            "precision": "fp64 moments (%s), fp64 FFT, per-trial 1e-6 certificate + fp64 fix-up"
                         % ("VALU cell gather" if form == "gather" else "v_mfma_f64_16x16x4_f64 slots")}


def pmc_traffic(photons, trials, nharm):
    """HBM bytes per search of this workload from the tree's own rocprofv3 PMC pass (tools/pmc_exact.sh ->
    profiles/r04/pmc_traffic.json), or None if that pass was not taken on this workload."""
    try:
        rec = json.load(open(PMC_FILE))
    except (OSError, ValueError):
        return None, None
    if (rec.get("photons"), rec.get("trials"), rec.get("nharm")) != (photons, trials, nharm):
        return None, None
    return rec.get("bytes_per_search"), rec.get("source")


def pmc_clock():
    """The search kernel's clock and clock-normalised matrix-pipe occupancy from the tree's SQ counter pass
    (tools/pmc_round.sh -> profiles/r04/pmc_search/): clock = GRBM_GUI_ACTIVE / 8 XCDs / the launch's duration in
    the same session's kernel trace; busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x those cycles)."""
    d = os.path.join(ROOT, "profiles", "r04", "pmc_search")
    try:
        cnt = {}
        for line in open(os.path.join(d, "summary_k_search_exact.txt")):
            f = line.split()
            if len(f) >= 2 and f[0].endswith("/disp"):
                cnt[f[0][:-5]] = float(f[1])
        ns = None
        for line in open(os.path.join(d, "trace_kernel_stats.csv")):
            if line.startswith('"void k_search_exact<false>'):
                ns = float(line.rsplit('",', 1)[1].split(",")[2])
        cyc = cnt["GRBM_GUI_ACTIVE"] / 8.0
        return {"clock_ghz": cyc / ns, "matrix_pipe_busy_at_clock": cnt["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024.0 * cyc),
                "source": "profiles/r04/pmc_search (rocprofv3 --pmc over tools/run_search.py, config 3, the same kernel)"}
    except (OSError, KeyError, ValueError, IndexError, TypeError, ZeroDivisionError):
        return None


def main():
    a = parse()
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # CRIMP_BENCH_REHEARSE=1: every rank on cuda:0 over gloo, to run the N > 1 code path (sharded search, gathers,
    # max-over-ranks timing) on a one-GPU box; the numbers of such a run are not a scaling measurement
    rehearse = os.environ.get("CRIMP_BENCH_REHEARSE") == "1"
    if rehearse:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)
    from crimp_amd import ops
    from crimp_amd import _native as N
    from crimp_amd.synth import pulsed_events

    span, f0 = 1.0e6, 7.123456789
    t_h = pulsed_events(a.photons, span, f0, pulsed_frac=0.1, seed=0)
    df = 1.0 / (10.0 * span)
    M = a.trials
    # the whole N*M grid centred on f0; sharding.sharded_search gives this rank trials [rank*M, (rank+1)*M)
    f_h = f0 + (np.arange(world * M) - (world * M) // 2) * df
    t = torch.as_tensor(t_h, device=dev)
    f = torch.as_tensor(f_h, device=dev)
    t0_h = (t_h[0] + t_h[-1]) / 2  # periodsearch.py:54 on the host copy (the device tensor holds the same values)
    from crimp_amd.sharding import sharded_search, shard_range
    assert shard_range(world * M, world, rank) == (rank * M, M)

    def timed_steps(precision, steps, warmup, flags=0):
        """warmup untimed steps, then `steps` timed between barriers: (max-over-ranks seconds, kernel ms, fix-ups,
        last best, per-step hipEvent ms). A step is this rank's slice through crimp_search and one all_gather of
        every rank's (best power, flat index), ties -> lowest index (the tested path, tests/test_distributed_*)."""
        def step():
            return sharded_search(t, f, a.nharm, 0, gather="best", flags=flags, precision=precision, t0=t0_h)

        # clock settle (untimed): the step repeated for a.settle seconds before the W warmup steps -- after the
        # seconds of host-side setup the GPU's clocks have dropped, and a short timed window would measure the
        # ramp, not the steady state a search service runs at (20 steps after 3 warmups: 0.49 vs 0.43-0.44 ms per
        # step in a loop that had run for a while, profiles/r06/clock_settle.log)
        t_s = time.perf_counter()
        while time.perf_counter() - t_s < a.settle:
            step()
            torch.cuda.synchronize()
        for _ in range(warmup):
            step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        # the timed loop holds the steps only: the library's measurement hooks (kernel ms, fix-ups) are read after
        # it, from the last step (every step searches the same inputs), and one pair of events brackets the loop
        stream = torch.cuda.current_stream()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t1 = time.perf_counter()
        ev0.record(stream)
        for k in range(steps):
            b = step()
        ev1.record(stream)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        el = time.perf_counter() - t1
        elt = torch.tensor([el], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(elt, op=dist.ReduceOp.MAX)
        return (float(elt.item()), N.load().crimp_last_kernel_ms(), float(N.load().crimp_last_fixups()), b,
                ev0.elapsed_time(ev1) / steps, N.load().crimp_last_search_path())

    def exact_record(el, kern_ms, nfix, steps):
        ops_per_launch = OPS_PER_EVAL_HARM * a.nharm * float(a.photons) * M
        achieved = ops_per_launch / (kern_ms * 1e-3) / 1e12
        traffic, tsrc = pmc_traffic(a.photons, M, a.nharm)
        return {"value": float(a.photons) * M * world * steps / el, "unit": "photon*trial evals/s", "steps": steps,
                "ms_per_step": el / steps * 1e3, "fp64_fixup_trials_per_step": nfix,
                "dtype": "int8 digits on i8 MFMA, exact int32/int64 sums (fp64 phase, 2^30 fixed-point cos/sin)",
                "roofline": {"kernel": "k_search_exact", "bound": "mfma", "achieved": achieved, "peak": PEAK_I8_TOPS,
                             "unit": "TFLOP/s", "frac": achieved / PEAK_I8_TOPS, "traffic": traffic, "kernel_ms": kern_ms,
                             "pmc": pmc_clock(),
                             "note": "int8 matrix ops issued: 128 per photon*trial*harmonic (8 v_mfma_i32_32x32x32_i8 + "
                                     "4 2:4-sparse v_smfmac_i32_32x32x64_i8 per 4 photons x 2048 trials) / mean "
                                     "duration of the harmonic-sum kernels (hipEvents in libcrimp_hip on their stream); "
                                     "peak = that 2:1 dense:sparse instruction mix at 32 cycles each (I8 dense 5.0 "
                                     "POP/s, sparse 10.0): frac = matrix-pipe occupancy at 2.4 GHz; traffic: %s" % (
                                         tsrc or "no PMC pass on this workload")}}

    prec = None if a.precision == "default" else a.precision
    el, kern_ms, nfix, (best_pow, best_idx), step_ms, path = timed_steps(
        prec, a.steps, a.warmup, flags=N.FLAG_TIME_KERNELS if a.precision == "exact" else 0)
    value = float(a.photons) * M * world * a.steps / el
    exact = None
    if a.precision != "exact" and not a.no_exact:
        e_el, e_kms, e_nfix, e_best, _, _ = timed_steps("exact", a.exact_steps, 1, flags=N.FLAG_TIME_KERNELS)
        exact = exact_record(e_el, e_kms, e_nfix, a.exact_steps)
        exact["best_trial_index"], exact["best_power"] = e_best[1], float(e_best[0])
    rec = None
    if rank == 0:
        rec = {
            "metric": "Z^2_2 photon*trial evals/sec (node)",
            "value": value,
            "unit": "photon*trial evals/s" if a.precision == "exact" else "equivalent photon*trial evals/s",
            "value_kind": ("direct: every photon x trial pair evaluated" if a.precision == "exact" else
                           "equivalent: photons x trials / wall time of the NUFFT search, which returns every "
                           "trial's power (certified within 1e-6 of the reference) without evaluating each pair; "
                           "exact_path and cpu_baseline evaluate every pair"),
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": el / a.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64" if a.precision != "exact" else
                     "int8 digits on i8 MFMA, exact int32/int64 sums (fp64 phase, 2^30 fixed-point cos/sin)",
            "data": "synthetic (seeded Poisson pulsed events, crimp_amd/synth.py)",
            "config": {"workload": "config3: synthetic %d photons x %d trials/GPU, Z^2_%d" % (a.photons, M, a.nharm),
                       "photons": a.photons, "trials_per_gpu": M, "nharm": a.nharm, "span_s": span, "f0": f0,
                       "trial_step_hz": df,
                       "parallelism": "trial-sharded dp%d: sharding.sharded_search + all_gather(best)" % world,
                       "best_trial_index": best_idx, "best_power": float(best_pow),
                       "search_path": {0: "fp64", 1: "exact", 2: "nufft"}.get(path, path),
                       "precision": a.precision, "fp64_fixup_trials_per_step": nfix},
        }
        if a.precision == "exact":
            ex = exact_record(el, kern_ms, nfix, a.steps)
            rec["roofline"] = dict(ex["roofline"], step_ms=step_ms)
        else:
            # the NUFFT's per-kernel rooflines from separately timed searches (hipEvent spans per kernel class)
            nu = nufft_leg(a, t, t_h, f, rank, M, max(3, a.steps))
            rec["roofline"] = dict(nu["roofline"], step_ms=step_ms,
                                   note="dominant kernel class of the NUFFT search (DESIGN.md 5.3): algorithmic "
                                        "work per launch (crimp_last_nufft_work) / mean launch duration (hipEvents "
                                        "on the library's stream); all classes under `nufft.kernels`; traffic: HBM "
                                        "bytes per launch, rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (x2 FETCH gfx950 "
                                        "correction) of the same kernel, profiles/r06/pmc_nufft_traffic.json")
            rec["roofline"].setdefault("traffic", None)
            rec["nufft"] = nu
            if exact is not None:
                rec["exact_path"] = exact
                rec["exact_path"]["same_best_trial"] = (exact["best_trial_index"] == best_idx)
        if not a.no_cpu and world == 1:  # rank 0 at N=1 only
            rec["cpu_baseline"] = cpu_baseline(t_h, f0, df, a.nharm, a.cpu_seconds)
    del t, f
    torch.cuda.empty_cache()
    if not a.no_calcphase and rank == 0:
        rec["calcphase"] = calcphase_leg(a, dev)
    if not a.no_toa:
        toa = toa_leg(a, dev, world, rank)
        if rank == 0:
            rec.update(toa)
    if not a.no_config4:
        c4 = config4_leg(a, dev, world, rank)
        if rank == 0:
            rec["config4"] = c4
    if not a.no_config2 and rank == 0:
        rec["config2"] = config2_leg(a)
    if rank == 0:
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

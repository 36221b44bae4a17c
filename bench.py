"""Benchmark: Z^2_2 photon x trial evaluations per second (BASELINE.json metric, config 3).

One step = one complete Z^2_2 search of the config-3 workload per GPU: 1e7 synthetic pulsed
photons (T = 1e6 s, p = 0.1, f0 = 7.123456789 Hz, seed 0) against 1e6 trial frequencies
spaced 1/(10T), inputs resident in HBM, followed by the search's one exchange step (every
rank's best trial gathered so that all ranks agree on the global best, ties -> lowest index).
With N ranks each rank searches its own 1e6-trial slice of an N*1e6 grid (weak scaling);
``value`` = all ranks' evaluations / max-over-ranks time.

Also reported: the dominant kernel's roofline (algorithmic FLOP per launch / measured launch
time: 8 real FLOP per photon x trial x harmonic, the complex multiply-accumulate of the
factorised search), and the CPU oracle (oracle/liborc.so, OpenMP over trials) on
a bounded sample of the same workload.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_F32_TFLOPS = 157.3         # MI355X_MICROARCH.md: FP32-input MFMA = FP32 vector peak
PEAK_F16_DENSE_TFLOPS = 2500.0  # MI355X_MICROARCH.md: BF16/F16 dense (no 2:1 sparsity)
SPLIT_PRODUCTS = 4              # f16 hi/lo split: one fp32-exact product = four f16 products
# HBM bytes per harmonic-sum launch of this workload from rocprofv3 PMC passes (profiles/): (2 x FETCH_SIZE
# + WRITE_SIZE) KB x 1024, FETCH_SIZE doubled per the gfx950 correction in MI355X_MICROARCH.md (HBM section).
PMC_TRAFFIC_BYTES = {"f16": (2 * 659900.0 + 2019000.0) * 1024,  # profiles/r1_final2/pmc_s64/pmc_summary.txt (64 splits)
                     "f32": (2 * 588447.5625 + 153453.875) * 1024}  # profiles/r1/search_mfma_pmc_summary.json
FLOP_PER_EVAL_HARM = 8.0
PEAK_HBM_GBS = 8000.0           # MI355X_MICROARCH.md: HBM3E ~8 TB/s


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--photons", type=int, default=10_000_000)
    p.add_argument("--trials", type=int, default=1_000_000, help="trial frequencies per GPU")
    p.add_argument("--nharm", type=int, default=2)
    p.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--toa-intervals", type=int, default=1250, help="ToA intervals per GPU (config 5: 1e4 over 8)")
    p.add_argument("--toa-photons", type=int, default=100_000)
    p.add_argument("--no-toa", action="store_true", help="skip the ToA-fit throughput leg")
    p.add_argument("--calcphase-photons", type=int, default=100_000_000)
    p.add_argument("--no-calcphase", action="store_true", help="skip the calcphase (HBM-bound) leg")
    return p.parse_args()


# 1E 2259+586 Fourier template (data/1e2259_template.txt), config 5 draws intervals from it
T2259 = {"model": "fourier", "norm": {"value": 17.060771467236613},
         "amp": [1.508994969593123, 4.055594828231136, 1.4384785819368275, 0.3505348524380939,
                 0.19725727340744187, 0.3483402644535841],
         "ph": [-0.4071967961461897, -0.8051383329477251, 0.5157949575544241, 1.9295783704947946,
                -0.1917798112304259, 0.8297144204463391]}


def toa_leg(a, dev, world, rank):
    """Config 5 (per GPU): intervals x photons drawn from the 1e2259 template with random true shifts,
    brute grid + exact MLE + 1-sigma scan + redChi2 per interval (measureToA_fourier -bm); ``warmup``
    untimed fits, then the mean over up to 3 timed fits of all intervals (max over ranks)."""
    import torch
    import torch.distributed as dist
    from crimp_amd.synth import template_intervals_torch
    from crimp_amd.toafit import ToAFitter
    tm = {"model": "fourier", "norm": T2259["norm"]}
    for j, (am, ph) in enumerate(zip(T2259["amp"], T2259["ph"]), start=1):
        tm["amp_%d" % j] = {"value": am}
        tm["ph_%d" % j] = {"value": ph}
    x, off, E, shifts = template_intervals_torch(a.toa_intervals, a.toa_photons, T2259["norm"]["value"],
                                                 T2259["amp"], T2259["ph"], seed=2 + rank, device=dev)
    for _ in range(max(a.warmup, 0)):  # untimed: code-object load, scratch-pool growth
        ToAFitter(x, off, E, tm).fit(brutemin=True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    reps = max(1, min(a.steps, 3))
    t1 = time.perf_counter()
    for _ in range(reps):
        res = ToAFitter(x, off, E, tm).fit(brutemin=True)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t1) / reps
    elt = torch.tensor([el], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(elt, op=dist.ReduceOp.MAX)
    d = np.angle(np.exp(1j * (res["phShi"] - shifts)))  # recovered vs true shift, wrapped
    return {"toa_fits_per_s": a.toa_intervals * world / float(elt.item()),
            "toa_config": "config5: %d intervals/GPU x %d photons, Fourier K=6 (1e2259), brute+MLE+1-sigma scan"
                          % (a.toa_intervals, a.toa_photons),
            "toa_seconds": float(elt.item()),
            "toa_mean_likelihood_evaluations": float(np.mean(res["evaluations"])),
            "toa_shift_recovery_rms_cycles": float(np.sqrt(np.mean(d ** 2)) / (2 * np.pi)),
            "toa_median_sigma_cycles": float(np.median(res["phShi_LL"]) / (2 * np.pi)),
            "toa_cpu_reference_fits_per_s": 0.42}


def calcphase_leg(a, dev):
    """calcphase (calcphase.py:152-176) over 1e8 photons resident in HBM: 8 B read + 16 B written per photon
    (SURVEY.md §8d), HBM-bound; hipEvents on the stream the library launches on (torch's current stream)."""
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
    """Oracle (fp64 C restatement of periodsearch.py:57-71, OpenMP over trials) on a bounded sample."""
    from oracle import oracle as O
    threads = min(16, os.cpu_count() or 1)
    O.set_threads(threads)
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
    return {"value": rate, "unit": "photon*trial evals/s", "cores": threads, "kind": "port",
            "sample": "%d photons x %d trials of the same workload, Z^2_%d, oracle/liborc.so fp64, %.1f s" % (
                n, m, nharm, el)}


def main():
    a = parse()
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    from crimp_amd import ops
    from crimp_amd import _native as N
    from crimp_amd.synth import pulsed_events

    span, f0 = 1.0e6, 7.123456789
    t_h = pulsed_events(a.photons, span, f0, pulsed_frac=0.1, seed=0)
    df = 1.0 / (10.0 * span)
    M = a.trials
    g0 = rank * M - (world * M) // 2          # this rank's slice of the N*M grid centred on f0
    f_h = f0 + (np.arange(M) + g0) * df
    t = torch.as_tensor(t_h, device=dev)
    f = torch.as_tensor(f_h, device=dev)
    out = torch.empty(M, dtype=torch.float64, device=dev)
    t0 = (t_h[0] + t_h[-1]) / 2
    best = torch.zeros(2, dtype=torch.float64, device=dev)
    gathered = torch.zeros(world, 2, dtype=torch.float64, device=dev)

    kms = []

    def step():
        ops.search(t, t0, f, a.nharm, 0, out=out, flags=N.FLAG_TIME_KERNELS)
        kms.append(N.load().crimp_last_kernel_ms())
        i = torch.argmax(out)
        best[0] = out[i]
        best[1] = (i + (g0 + (world * M) // 2)).to(torch.float64)  # global trial index
        if world > 1:
            dist.all_gather_into_tensor(gathered, best)
        else:
            gathered[0] = best
        return gathered

    for _ in range(a.warmup):
        step()
    kms.clear()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]
    t1 = time.perf_counter()
    for k in range(a.steps):
        evs[k][0].record(stream)
        g = step()
        evs[k][1].record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t1
    elt = torch.tensor([el], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(elt, op=dist.ReduceOp.MAX)
    el = float(elt.item())
    step_ms = float(np.mean([s.elapsed_time(e) for s, e in evs]))
    kern_ms = float(np.mean(kms))  # hipEvents around the harmonic-sum kernels, on the stream they run on
    gb = g.cpu().numpy()
    order = np.lexsort((gb[:, 1], -gb[:, 0]))
    best_idx = int(gb[order[0], 1])

    evals = float(a.photons) * M * world * a.steps
    value = evals / el
    if rank == 0:
        flop = FLOP_PER_EVAL_HARM * a.nharm * float(a.photons) * M
        achieved = flop / (kern_ms * 1e-3) / 1e12
        variant = "f32" if os.environ.get("CRIMP_MFMA", "").lower() == "f32" else "f16"
        peak = PEAK_F32_TFLOPS if variant == "f32" else PEAK_F16_DENSE_TFLOPS / SPLIT_PRODUCTS
        rec = {
            "metric": "Z^2_2 photon*trial evals/sec (node)",
            "value": value,
            "unit": "photon*trial evals/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": el / a.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": ("f32-input MFMA" if variant == "f32" else "f16 hi/lo-split MFMA (fp32-exact products)")
                     + ", f32 sin/cos, f64 phase + sums",
            "data": "synthetic (seeded Poisson pulsed events, crimp_amd/synth.py)",
            "config": {"workload": "config3: synthetic %d photons x %d trials/GPU, Z^2_%d" % (a.photons, M, a.nharm),
                       "photons": a.photons, "trials_per_gpu": M, "nharm": a.nharm, "span_s": span, "f0": f0,
                       "trial_step_hz": df, "parallelism": "trial-sharded dp%d + all_gather(best)" % world,
                       "best_trial_index": best_idx, "best_power": float(gb[order[0], 0]),
                       "search_path": os.environ.get("CRIMP_SEARCH", "auto")},
            "roofline": {"bound": "mfma", "achieved": achieved, "peak": peak, "unit": "TFLOP/s",
                         "frac": achieved / peak,
                         "traffic": PMC_TRAFFIC_BYTES[variant]
                         if (a.photons, M, a.nharm) == (10_000_000, 1_000_000, 2) else None,
                         "kernel_ms": kern_ms, "step_ms": step_ms,
                         "note": "achieved = 8 FLOP (one complex MAC) per photon*trial*harmonic / mean duration of the "
                                 "harmonic-sum kernels (hipEvents in libcrimp_hip on their stream); peak = "
                                 + ("FP32-input MFMA" if variant == "f32" else
                                    "F16 dense MFMA / 4 (four f16 products per fp32-exact product)")},
        }
        if not a.no_cpu:
            rec["cpu_baseline"] = cpu_baseline(t_h, f0, df, a.nharm, a.cpu_seconds)
    del t, f, out
    torch.cuda.empty_cache()
    if not a.no_calcphase and rank == 0:
        rec["calcphase"] = calcphase_leg(a, dev)
    if not a.no_toa:
        toa = toa_leg(a, dev, world, rank)
        if rank == 0:
            rec.update(toa)
    if rank == 0:
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

"""GPU check of the exact-integer search kernel: plain per-trial relative error against the reference's
goldens and the oracle, bit-identity of trial partitions, and config-3 timing next to the NUFFT path."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def rel(got, ref):
    got, ref = np.asarray(got), np.asarray(ref)
    e = np.abs(got - ref) / np.abs(ref)
    return float(e.max()), int(e.argmax()), float(np.percentile(e, 50)), float(np.percentile(e, 99))


def main():
    import torch
    from conftest import gold
    from crimp_amd.periodsearch import PeriodSearch
    from crimp_amd import ops
    from crimp_amd import _native as N
    from crimp_amd.synth import pulsed_events
    from oracle import oracle as O
    L = N.load()
    g = gold("periodsearch_1e2259.npz")
    for prec in (None, "nufft"):
        z = PeriodSearch(g["time"], g["freq"], 2, precision=prec).ztest()
        print("config1 Z2_2 %s: argmax %d  rel(max, at, p50, p99) %s  fixups %d" % (
            prec, int(np.argmax(z)), rel(z, g["z2_m2"]), L.crimp_last_fixups()), flush=True)
        h = PeriodSearch(g["time"], g["freq"], 20, precision=prec).htest()
        print("config1 H20 %s: argmax %d  rel %s  fixups %d" % (prec, int(np.argmax(h)), rel(h, g["h_m20"]),
                                                                 L.crimp_last_fixups()), flush=True)
        a, _ = PeriodSearch(g["time"], g["fsub"], 2, precision=prec).twod_ztest(g["fd"])
        print("config1 2-D Z2 %s: rel %s" % (prec, rel(a[:, 2], g["z2d_m2"][:, 2])), flush=True)
    s = gold("periodsearch_synth.npz")
    for m in (1, 2, 3, 5):
        print("synth Z2_%d rel %s" % (m, rel(PeriodSearch(s["time"], s["freq"], m).ztest(), s["z_m%d" % m])), flush=True)
    for m in (1, 5, 20):
        print("synth H_%d rel %s" % (m, rel(PeriodSearch(s["time"], s["freq"], m).htest(), s["h_m%d" % m])), flush=True)
    t = pulsed_events(200000, 2.0e5, 7.123456789, pulsed_frac=0.05, seed=4)
    f = 7.123456789 + (np.arange(-1024, 1024) / (10 * 2.0e5))
    zr = O.search(t, f, 2)
    for prec in (None, "nufft"):
        z = PeriodSearch(t, f, 2, precision=prec).ztest()
        print("2e5x2048 Z2 %s: rel %s fixups %d  min power %.3g" % (prec, rel(z, zr), L.crimp_last_fixups(), zr.min()),
              flush=True)
    fd = np.array([-13.0, -12.0, -11.5])
    ar = O.search(t, f[512:1536], 3, freq_dot=fd, stat="h")
    a = PeriodSearch(t, f[512:1536], 3).twod_htest(fd)[0][:, 2]
    print("2e5 2-D H3 rel %s argmax %d vs %d" % (rel(a, ar), int(np.argmax(a)), int(np.argmax(ar))), flush=True)
    # config 3
    n, M, span, f0 = 10_000_000, 1_000_000, 1.0e6, 7.123456789
    t_h = pulsed_events(n, span, f0, pulsed_frac=0.1, seed=0)
    f_h = f0 + (np.arange(M) - M // 2) / (10.0 * span)
    tt = torch.as_tensor(t_h, device="cuda")
    ff = torch.as_tensor(f_h, device="cuda")
    t0 = (t_h[0] + t_h[-1]) / 2
    res = {}
    for prec in (None, "nufft"):
        z = ops.search(tt, t0, ff, 2, 0, precision=prec)
        torch.cuda.synchronize()
        ts = []
        for _ in range(3):
            t1 = time.perf_counter()
            z = ops.search(tt, t0, ff, 2, 0, precision=prec, flags=N.FLAG_TIME_KERNELS)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t1)
        km = L.crimp_last_kernel_ms()
        res[prec] = z.cpu().numpy()
        print("config3 %s: %.1f ms/call (kernels %.1f ms) = %.3e evals/s  argmax %d fixups %d" % (
            prec, 1e3 * min(ts), km, n * M / min(ts), int(np.argmax(res[prec])), L.crimp_last_fixups()), flush=True)
    rng = np.random.default_rng(1)
    idx = np.unique(np.concatenate([[M // 2, M // 2 - 1, M // 2 + 1, 0, M - 1], rng.integers(0, M, 11)]))
    zr = O.search(t_h, f_h[idx], 2)
    print("config3 sampled rel exact %s   nufft %s" % (rel(res[None][idx], zr), rel(res["nufft"][idx], zr)), flush=True)
    a = ops.search(tt, t0, ff, 2, 0, first=0, count=M // 2 + 123).cpu().numpy()
    b = ops.search(tt, t0, ff, 2, 0, first=M // 2 + 123, count=M - (M // 2 + 123)).cpu().numpy()
    print("config3 partition bit-identical:", bool(np.array_equal(np.concatenate([a, b]), res[None])), flush=True)
    print("exact vs nufft scaled diff: %.3g" % float((np.abs(res[None] - res["nufft"]) / np.mean(res[None])).max()))


if __name__ == "__main__":
    main()

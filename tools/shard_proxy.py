"""Single-GPU proxy of the two ways to strong-scale ONE trial row (config 3: 1e7 photons x 1e6 trials, Z^2_2) over W
ranks: (a) trial slices -- each rank searches M/W trials of the row (its own plan, nseg = M/W)
over all N photons; (b) photon slices -- each rank searches all M trials over N/W photons, then one all-reduce of the
per-trial complex harmonic sums (2 m x 16 B x M). Prints the per-rank device time of each (REPS timed searches after
a warm-up) and the all-reduce volume of (b)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from crimp_amd import ops, _native as N  # noqa: E402
from crimp_amd.synth import pulsed_events  # noqa: E402

n, M, m, span, f0 = 10_000_000, 1_000_000, 2, 1.0e6, 7.123456789
t_h = pulsed_events(n, span, f0, pulsed_frac=0.1, seed=0)
dev = torch.device("cuda", 0)
t = torch.as_tensor(t_h, device=dev)
f = torch.as_tensor(f0 + (np.arange(M) - M // 2) / (10 * span), device=dev)
t0 = (t_h[0] + t_h[-1]) / 2
reps = int(os.environ.get("REPS", 20))


def tm(fn):
    for _ in range(30):  # clock settle + warm-up
        fn()
    torch.cuda.synchronize()
    a = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - a) / reps * 1e3


full = tm(lambda: ops.search(t, t0, f, m, 0))
print("W=1 whole row: %.3f ms (plan %s)" % (full, N.last_nufft_plan()), flush=True)
for W in (2, 4, 8):
    a = tm(lambda: ops.search(t, t0, f, m, 0, first=0, count=M // W))
    pa = N.last_nufft_plan()
    ts = t[: n // W]
    b = tm(lambda: ops.search(ts, t0, f, m, 0))
    print("W=%d (a) trial slice %d trials x %d photons: %.3f ms (plan %s) | (b) photon slice %d photons x %d trials: "
          "%.3f ms + all-reduce of %.1f MB per search" % (W, M // W, n, a, pa, n // W, M, b, 2 * m * 16 * M / 1e6),
          flush=True)

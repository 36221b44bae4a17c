"""Config-4 throughput on one GPU, the workload of bench.py's config4 leg: 1e8 photons
(T = 1e7 s, p = 0.05, fdot = -1e-12, seed 1), 2-D H-test m = 20 on the default (exact) path over the first NTR
trials (default 131072) of the flat fd-outer grid 1e5 f (step 1/(10 T)) x 100 rows linspace(-13.5, -11.5, 100)
(rank 0's shard of the 1e7-trial grid starts there). One untimed search, then one timed.
usage: python tools/run_config4.py   (NTR, FIRST override the trial range)"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from crimp_amd import ops, _native as N  # noqa: E402
from crimp_amd.synth import pulsed_events  # noqa: E402

n, span, f0, fdot, M = 100_000_000, 1.0e7, 7.123456789, -1.0e-12, 100_000
NTR, FIRST = int(os.environ.get("NTR", 131072)), int(os.environ.get("FIRST", 0))
t_h = pulsed_events(n, span, f0, pulsed_frac=0.05, fdot=fdot, seed=1)
dev = torch.device("cuda", 0)
t = torch.as_tensor(t_h, device=dev)
f = torch.as_tensor(f0 + (np.arange(M) - M // 2) / (10.0 * span), device=dev)
fd = torch.as_tensor(np.linspace(-13.5, -11.5, 100), device=dev)
t0 = (t_h[0] + t_h[-1]) / 2
h = ops.search(t, t0, f, 20, 1, log10_negfdot=fd, first=FIRST, count=NTR)  # warm-up
torch.cuda.synchronize()
t1 = time.perf_counter()
h = ops.search(t, t0, f, 20, 1, log10_negfdot=fd, first=FIRST, count=NTR, flags=N.FLAG_TIME_KERNELS)
torch.cuda.synchronize()
el = time.perf_counter() - t1
kms = N.load().crimp_last_kernel_ms()
ev = float(n) * NTR
print("config4: %d photons x trials [%d, %d), H_20: %.2f s (kernels %.2f s), %.3e evals/s, %.3e harmonic sums/s, "
      "fixups %d, best flat index %d H %.3f" % (n, FIRST, FIRST + NTR, el, kms / 1e3, ev / el, 20 * ev / el,
                                                N.load().crimp_last_fixups(), FIRST + int(torch.argmax(h)),
                                                float(h.max())), flush=True)

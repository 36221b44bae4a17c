"""Config 4 (1e8 photons, T = 1e7 s, H_20, 1e5 f x 100 log10|fdot| rows) by precision="nufft" on one GPU: whole grid
or ROWS rows, REPS timed searches with the per-kernel-class hipEvent spans (crimp_last_kernel_times)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from crimp_amd import ops, _native as N  # noqa: E402
from crimp_amd.synth import pulsed_events  # noqa: E402

n, span, f0, fdot, M = int(os.environ.get("NPH", 100_000_000)), 1.0e7, 7.123456789, -1.0e-12, 100_000
rows = int(os.environ.get("ROWS", 100))
t_h = pulsed_events(n, span, f0, pulsed_frac=0.05, fdot=fdot, seed=1)
dev = torch.device("cuda", 0)
t = torch.as_tensor(t_h, device=dev)
t0 = (t_h[0] + t_h[-1]) / 2
f = torch.as_tensor(f0 + (np.arange(M) - M // 2) / (10.0 * span), device=dev)
fd = torch.as_tensor(np.linspace(-13.5, -11.5, 100)[:rows], device=dev)
for rep in range(int(os.environ.get("REPS", 2)) + 1):
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    z = ops.search(t, t0, f, 20, 1, log10_negfdot=fd, precision="nufft",
                   flags=N.FLAG_TIME_KERNELS if os.environ.get("TIMED", "1") == "1" else 0)
    torch.cuda.synchronize()
    el = time.perf_counter() - t1
    sp = N.last_kernel_times()[:15]
    i = int(torch.argmax(z))
    print("rep %d: %.3f s, %.3e evals/s, plan %s, fixups %d, best row %d f %d power %.6g | spans ms %s" % (
        rep, el, n * M * rows / el, N.last_nufft_plan(), N.load().crimp_last_fixups(), i // M, i % M, float(z[i]),
        " ".join("%s=%.1f/%d" % (c, sp[1 + k], sp[8 + k]) for k, c in enumerate(N.NUFFT_CLASSES)) if sp else "-"),
          flush=True)

"""One config-3 Z^2_2 search (1e7 photons x 1e6 trials) for profiling; precision from CRIMP_PRECISION."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from crimp_amd import ops  # noqa: E402
from crimp_amd.synth import pulsed_events  # noqa: E402

n = int(os.environ.get("NPH", 10_000_000))
M = int(os.environ.get("NTR", 1_000_000))
m = int(os.environ.get("NHARM", 2))
span, f0 = 1.0e6, 7.123456789
t_h = pulsed_events(n, span, f0, pulsed_frac=0.1, seed=0)
dev = torch.device("cuda", 0)
t = torch.as_tensor(t_h, device=dev)
f = torch.as_tensor(f0 + (np.arange(M) - M // 2) / (10 * span), device=dev)
t0 = (t_h[0] + t_h[-1]) / 2
for rep in range(int(os.environ.get("REPS", 1))):
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    z = ops.search(t, t0, f, m, 0)
    torch.cuda.synchronize()
    el = time.perf_counter() - t1
    print("precision %s: %.1f ms %.3e evals/s argmax %d" % (
        os.environ.get("CRIMP_PRECISION", "exact"), el * 1e3, n * M / el, int(torch.argmax(z))), flush=True)

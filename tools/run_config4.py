"""Config-4 throughput on one GPU: 1e8 photons (T = 1e7 s, p = 0.05, fdot = -1e-12,
seed 1), 2-D H-test m = 20 over fd rows x f trials on the default (exact) path. The full config-4 grid is
1e5 f x 100 fd = 1e7 trials sharded over 8 GPUs (1.25e6 per GPU, ~2.5 min per GPU at this rate); this times a
ROWS x NF sub-grid and reports photon*trial evals/s and harmonic-sums/s. usage: python tools/run_config4.py"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from crimp_amd import ops, _native as N  # noqa: E402
from crimp_amd.synth import pulsed_events  # noqa: E402

n, span, f0, fdot = 100_000_000, 1.0e7, 7.123456789, -1.0e-12
NF, ROWS = int(os.environ.get("NF", 32768)), int(os.environ.get("ROWS", 4))
t_h = pulsed_events(n, span, f0, pulsed_frac=0.05, fdot=fdot, seed=1)
dev = torch.device("cuda", 0)
t = torch.as_tensor(t_h, device=dev)
f = torch.as_tensor(f0 + (np.arange(NF) - NF // 2) / (10.0 * span), device=dev)
fd = torch.as_tensor(np.linspace(-12.75, -11.25, ROWS), device=dev)
t0 = (t_h[0] + t_h[-1]) / 2
h = ops.search(t, t0, f, 20, 1, log10_negfdot=fd)  # warm-up
torch.cuda.synchronize()
t1 = time.perf_counter()
h = ops.search(t, t0, f, 20, 1, log10_negfdot=fd, flags=N.FLAG_TIME_KERNELS)
torch.cuda.synchronize()
el = time.perf_counter() - t1
kms = N.load().crimp_last_kernel_ms()
hb = h.cpu().numpy().reshape(ROWS, NF)
r, j = np.unravel_index(int(np.argmax(hb)), hb.shape)
ev = float(n) * NF * ROWS
print("config4 slice: %d photons x %d x %d trials, H_20: %.2f s (kernels %.2f s), %.3e evals/s, %.3e harmonic "
      "sums/s, fixups %d, best row %d idx %d H %.3f" % (n, ROWS, NF, el, kms / 1e3, ev / el, 20 * ev / el,
                                                      N.load().crimp_last_fixups(), r, j, hb[r, j]), flush=True)

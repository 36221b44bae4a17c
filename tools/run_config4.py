"""Config 4 on one GPU: the 2-D H-test (m = 20) over one GPU's eighth of the
1e5 f x 100 freq_dot grid (1.25e6 flat trials, fd-outer) for N = 1e8 photons spanning 1e7 s.
The slice is searched in CHUNKS calls (progress line after each); the photon split count depends
on N only, so the chunked values equal one call's. Prints one JSON line at the end: photon x trial
evals/s of this GPU (wall, resident inputs) and the harmonic-sum kernel time (hipEvents)."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from crimp_amd import ops  # noqa: E402
from crimp_amd import _native as N  # noqa: E402
from crimp_amd.synth import pulsed_events  # noqa: E402

n = int(os.environ.get("NPH", 100_000_000))
chunks = int(os.environ.get("CHUNKS", 2))
nf, nfd, ngpu = 100_000, 100, 8
span, f0 = 1.0e7, 7.123456789
t1 = time.perf_counter()
t_h = pulsed_events(n, span, f0, pulsed_frac=0.05, fdot=-1e-12, seed=1)
print("generated %d photons in %.1f s" % (t_h.size, time.perf_counter() - t1), flush=True)
n = int(t_h.size)
dev = torch.device("cuda", 0)
t = torch.as_tensor(t_h, device=dev)
f = torch.as_tensor(f0 + (np.arange(nf) - nf // 2) / (10 * span), device=dev)
fd = torch.as_tensor(np.linspace(-13.5, -11.5, nfd), device=dev)
t0 = float((t_h[0] + t_h[-1]) / 2)
del t_h
count = nf * nfd // ngpu
out = torch.empty(count, dtype=torch.float64, device=dev)
L = N.load()
# warm-up: one small call (code-object load, scratch allocation)
ops.search(t, t0, f, 20, 1, log10_negfdot=fd, first=0, count=4096, out=out[:4096])
torch.cuda.synchronize()
bounds = np.linspace(0, count, chunks + 1).astype(np.int64)
el = km = 0.0
for c in range(chunks):
    a, b = int(bounds[c]), int(bounds[c + 1])
    torch.cuda.synchronize()
    s = time.perf_counter()
    ops.search(t, t0, f, 20, 1, log10_negfdot=fd, first=a, count=b - a, out=out[a:b], flags=N.FLAG_TIME_KERNELS)
    torch.cuda.synchronize()
    el += time.perf_counter() - s
    km += L.crimp_last_kernel_ms()
    print("chunk %d/%d trials [%d, %d): %.1f s so far, %.3e evals/s" % (c + 1, chunks, a, b, el, n * b / el),
          flush=True)
i = int(torch.argmax(out))
print(json.dumps({"workload": "config4 one-GPU slice: 2-D H_20, %d photons x %d trials (flat [0, %d) of %d)"
                  % (n, count, count, nf * nfd),
                  "seconds": el, "kernel_ms": km, "evals_per_s": n * count / el,
                  "harmonic_evals_per_s": 20 * n * count / el,
                  "kernel_evals_per_s": n * count / (km * 1e-3),
                  "node_estimate_8gpu_evals_per_s": 8 * n * count / el,
                  "best_flat_index": i, "best_H": float(out[i])}), flush=True)

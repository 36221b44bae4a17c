"""A/B of NUFFT search variants on config 3 (1e7 photons x 1e6 trials, Z^2_2) through the library's env hooks:
VARIANTS="NAME=VAL[,NAME=VAL...];..." (e.g. "CRIMP_NUFFT_LANES=4;CRIMP_NUFFT_LANES=8"), REPS timed searches each
(interleaved rounds), per-class hipEvent spans (cellstart, spread, merge, pass1, pass2, combine, finalize) and
a digest of the powers."""
import hashlib
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from crimp_amd import ops, _native as N  # noqa: E402
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
variants = [v for v in os.environ.get("VARIANTS", "").split(";")]
keys = sorted({kv.split("=")[0] for v in variants for kv in v.split(",") if kv})
res = {v: [] for v in variants}
dig = {}
zs = {}
for rnd in range(int(os.environ.get("REPS", 5)) + 1):
    for v in variants:
        for k in keys:
            os.environ.pop(k, None)
        for kv in v.split(","):
            if kv:
                a, b = kv.split("=")
                os.environ[a] = b
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        z = ops.search(t, t0, f, m, 0, precision="nufft", flags=N.FLAG_TIME_KERNELS)
        torch.cuda.synchronize()
        el = time.perf_counter() - t1
        sp = N.last_kernel_times()[:15]
        if rnd > 0:
            res[v].append([el * 1e3] + sp[:8])
        zs[v] = z.cpu().numpy()
        dig[v] = hashlib.sha1(zs[v].tobytes()).hexdigest()[:12]
print("%-32s %8s %8s | %s | digest  max-rel-vs-first" % ("variant", "wall", "pipe",
                                                          " ".join("%8s" % c for c in N.NUFFT_CLASSES)))
z0 = zs[variants[0]]
for v in variants:
    a = np.mean(np.array(res[v]), axis=0)
    print("%-32s %8.3f %8.3f | %s | %s %.2e" % (v or "(default)", a[0], a[1], " ".join("%8.4f" % x for x in a[2:9]),
                                                dig[v], float(np.max(np.abs(zs[v] - z0) / np.abs(z0)))))

"""Compare the f32-input and f16-split factorised search kernels: accuracy vs the oracle and speed."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from crimp_amd import ops, _native as N  # noqa: E402
from crimp_amd.synth import pulsed_events  # noqa: E402
from oracle import oracle as O  # noqa: E402

dev = torch.device("cuda", 0)
VARIANTS = {"f32": N.FLAG_MFMA_F32, "t1": 0, "t2": N.FLAG_MFMA_T2}


def scaled(got, ref):
    return float((np.abs(got - ref) / np.maximum(np.abs(ref), np.mean(np.abs(ref)))).max())


# accuracy: full oracle on moderate sizes, several harmonics / stats / 2-D
cases = [(300000, 3.0e5, 5.0, 0.02, 2048, 2, 0, None), (300000, 3.0e5, 5.0, 0.3, 2048, 2, 0, None),
         (200000, 2.0e5, 7.1, 0.05, 2048, 5, 1, None), (100000, 1.0e5, 3.3, 0.1, 1024, 20, 1, None),
         (100000, 1.0e5, 3.3, 0.1, 1024, 3, 0, np.array([-13.0, -11.5]))]
for (n, span, f0, p, M, m, stat, fd) in cases:
    t = pulsed_events(n, span, f0, pulsed_frac=p, seed=7)
    f = f0 + (np.arange(M) - M // 2) / (10 * span)
    t0 = (t[0] + t[-1]) / 2
    ref = O.search(t, f, m, freq_dot=fd, stat="h" if stat else "z2")
    line = "n=%d p=%.2f M=%d m=%d stat=%d 2d=%s:" % (n, p, M, m, stat, fd is not None)
    for name, fl in VARIANTS.items():
        got = ops.search(t, t0, f, m, stat, log10_negfdot=fd, flags=fl | N.FLAG_FORCE_MFMA)
        line += "  %s err %.3g argmax %s" % (name, scaled(got, ref), int(np.argmax(got)) == int(np.argmax(ref)))
    print(line, flush=True)

# speed + agreement at config-3 size
n, M, span, f0 = 10_000_000, 1_000_000, 1.0e6, 7.123456789
t_h = pulsed_events(n, span, f0, pulsed_frac=0.1, seed=0)
f_h = f0 + (np.arange(M) - M // 2) / (10 * span)
t = torch.as_tensor(t_h, device=dev)
f = torch.as_tensor(f_h, device=dev)
t0 = (t_h[0] + t_h[-1]) / 2
res = {}
for name, fl in VARIANTS.items():
    ops.search(t, t0, f[:65536].contiguous(), 2, 0, flags=fl)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    z = ops.search(t, t0, f, 2, 0, flags=fl)
    torch.cuda.synchronize()
    el = time.perf_counter() - t1
    res[name] = z.cpu().numpy()
    print("%s: %.1f ms  %.3e evals/s  argmax %d" % (name, el * 1e3, n * M / el, int(np.argmax(res[name]))), flush=True)
idx = np.unique(np.concatenate([[M // 2 - 1, M // 2, M // 2 + 1], np.random.default_rng(1).integers(0, M, 5)]))
zr = O.search(t_h, f_h[idx], 2)
for name in VARIANTS:
    print("%s vs oracle on %d sampled trials: %.3g" % (name, idx.size, scaled(res[name][idx], zr)))
for name in ("t1", "t2"):
    print("%s vs f32 over all trials: %.3g" % (name, scaled(res[name], res["f32"])))

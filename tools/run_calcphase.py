"""calcphase over 1e8 photons resident in HBM (24 B/photon), hipEvent-timed."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from crimp_amd import ops  # noqa: E402

n = int(os.environ.get("NPH", 100_000_000))
dev = torch.device("cuda", 0)
tm = {"PEPOCH": 58000.0, "F0": 7.123456789, "F1": -1.0e-12, "F2": 1.0e-22}
t = torch.rand(n, dtype=torch.float64, device=dev) * 120.0 + 57940.0
tot, fol = torch.empty_like(t), torch.empty_like(t)
for _ in range(3):
    ops.calcphase(t, tm, total=tot, folded=fol)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
torch.cuda.synchronize()
e0.record()
for _ in range(20):
    ops.calcphase(t, tm, total=tot, folded=fol)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 20
print("lib %s: %.3f ms  %.0f GB/s" % ("libcrimp_hip", ms, 24.0 * n / ms / 1e6), flush=True)

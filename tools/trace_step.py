"""bench.py's search step (sharded_search(gather="best") of config 3, default precision) repeated, for a rocprofv3
kernel + HIP API + copy trace of the gaps between kernels (tools/trace_timeline.py reads it)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from crimp_amd.sharding import sharded_search  # noqa: E402
from crimp_amd.synth import pulsed_events  # noqa: E402

span, f0 = 1.0e6, 7.123456789
t_h = pulsed_events(10_000_000, span, f0, pulsed_frac=0.1, seed=0)
dev = torch.device("cuda", 0)
t = torch.as_tensor(t_h, device=dev)
f = torch.as_tensor(f0 + (np.arange(1_000_000) - 500_000) / (10 * span), device=dev)
t0 = (t_h[0] + t_h[-1]) / 2
for _ in range(int(os.environ.get("STEPS", 30))):
    b = sharded_search(t, f, 2, 0, gather="best", t0=t0)
torch.cuda.synchronize()
print("best", b)

"""Host-side time of the bench's ToA leg (config 5 per GPU): the sharded_toa_fit wall, ToAFitter construction and
fit, and -- CRIMP_TOA_HOST_TRACE=1 -- crimp_toa_fit_redchi2's own host phases (stderr), against its kernels.
usage: python tools/toa_host_trace.py"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from crimp_amd.sharding import sharded_toa_fit  # noqa: E402
from crimp_amd.synth import template_intervals_torch  # noqa: E402
from crimp_amd.toafit import ToAFitter  # noqa: E402

tm = bench._tmpl()
x, off, E, _ = template_intervals_torch(1250, 100000, bench.T2259["norm"]["value"], bench.T2259["amp"],
                                        bench.T2259["ph"], seed=2, device="cuda")
offh = off.cpu().numpy()
for _ in range(2):
    ToAFitter(x, off, E, tm).fit(brutemin=True)
torch.cuda.synchronize()
for rep in range(3):
    t0 = time.perf_counter()
    f = ToAFitter(x, off, E, tm)
    t1 = time.perf_counter()
    f.fit(brutemin=True)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    sharded_toa_fit(x, offh, E, tm, brutemin=True)
    torch.cuda.synchronize()
    t3 = time.perf_counter()
    print("construct %.3f ms, fit %.3f ms, sharded_toa_fit %.3f ms" % ((t1 - t0) * 1e3, (t2 - t1) * 1e3,
                                                                       (t3 - t2) * 1e3), flush=True)
os.environ["CRIMP_TOA_HOST_TRACE"] = "1"
for rep in range(3):
    ToAFitter(x, off, E, tm).fit(brutemin=True)
    torch.cuda.synchronize()

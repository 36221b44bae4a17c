"""Where the bench's ToA leg spends its time (config 5 per GPU: 1250 intervals x 1e5 photons, brute + MLE + 1-sigma
scan + redChi2): ToAFitter construction, the crimp_toa_fit call, and the device redChi2 step (crimp_toa_redchi2),
each bracketed by torch.cuda.synchronize(), mean of REPS after one warm-up.
usage: python tools/toa_leg_breakdown.py"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from crimp_amd import ops  # noqa: E402
from crimp_amd.synth import template_intervals_torch  # noqa: E402
from crimp_amd.toafit import ToAFitter  # noqa: E402

nint, nper, reps = 1250, 100000, int(os.environ.get("REPS", 5))
tm = bench._tmpl()
x, off, E, _ = template_intervals_torch(nint, nper, bench.T2259["norm"]["value"], bench.T2259["amp"],
                                        bench.T2259["ph"], seed=2, device="cuda")
ToAFitter(x, off, E, tm).fit(brutemin=True)
torch.cuda.synchronize()
t = {"construct": [], "toa_fit": [], "redchi2": [], "whole_fit": []}
for _ in range(reps):
    t0 = time.perf_counter()
    f = ToAFitter(x, off, E, tm)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    r = ops.toa_fit(f.x, f.offsets, f.tpl, f._arr(f.E, np.float64), f.norm0, f.res, True, False)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    t3 = time.perf_counter()
    f.reduced_chi2(None, None, records=r)
    torch.cuda.synchronize()
    t4 = time.perf_counter()
    ToAFitter(x, off, E, tm).fit(brutemin=True)
    torch.cuda.synchronize()
    t5 = time.perf_counter()
    for k, v in zip(t, (t1 - t0, t2 - t1, t4 - t3, t5 - t4)):
        t[k].append(v * 1e3)
for k, v in t.items():
    print("%-10s %8.3f ms (min %.3f)" % (k, np.mean(v), np.min(v)), flush=True)

"""Host-side phases of crimp_toa_fit_redchi2 calls (CRIMP_TOA_HOST_TRACE=1 lines on stderr) and the wall time of
ToAFitter.fit and sharding.sharded_toa_fit on the bench's config-5 share (1250 intervals x 1e5 photons, one GPU).
usage: CRIMP_TOA_HOST_TRACE=1 python tools/toa_host_trace.py"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from crimp_amd.synth import template_intervals_torch  # noqa: E402
from crimp_amd.toafit import ToAFitter  # noqa: E402
from crimp_amd.sharding import sharded_toa_fit  # noqa: E402

dev = torch.device("cuda", 0)
tm = bench._tmpl()
T = bench.T2259
nint, nph = 1250, 100000
x, off, E, shifts = template_intervals_torch(nint, nph, T["norm"]["value"], T["amp"], T["ph"], seed=2, device=dev)
off_g = np.arange(nint + 1, dtype=np.int64) * nph
E_g = np.full(nint, nph / T["norm"]["value"])
for _ in range(3):
    ToAFitter(x, off, E, tm).fit(brutemin=True)
torch.cuda.synchronize()
for name, fn in (("ToAFitter.fit", lambda: ToAFitter(x, off, E, tm).fit(brutemin=True)),
                 ("sharded_toa_fit", lambda: sharded_toa_fit(lambda a, b: x, off_g, E_g, tm, brutemin=True))):
    ts = []
    for _ in range(5):
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t1)
    print("%s: %.3f ms (min %.3f)" % (name, 1e3 * np.mean(ts), 1e3 * np.min(ts)), flush=True)
    sys.stderr.flush()

"""Config-5 ToA fits on one GPU (brute + MLE + 1-sigma scan), timed after a warm-up, with the brute-grid and fit
kernel times (hipEvents inside crimp_toa_fit). CRIMP_LIB selects a library build (A/B of kernel variants);
NINT / NPH override the interval count and photons per interval."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import T2259  # noqa: E402
from crimp_amd.synth import template_intervals_torch  # noqa: E402
from crimp_amd.toafit import ToAFitter  # noqa: E402
from crimp_amd import ops, _native as N  # noqa: E402
import numpy as np  # noqa: E402

nint, nph = int(os.environ.get("NINT", 1250)), int(os.environ.get("NPH", 100_000))
dev = torch.device("cuda", 0)
tm = {"model": "fourier", "norm": T2259["norm"]}
for j, (am, ph) in enumerate(zip(T2259["amp"], T2259["ph"]), start=1):
    tm["amp_%d" % j], tm["ph_%d" % j] = {"value": am}, {"value": ph}
x, off, E, shifts = template_intervals_torch(nint, nph, T2259["norm"]["value"], T2259["amp"], T2259["ph"], seed=2,
                                             device=dev)
ToAFitter(x, off, E, tm).fit(brutemin=True)
for rep in range(3):
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    r = ToAFitter(x, off, E, tm).fit(brutemin=True)
    torch.cuda.synchronize()
    el = time.perf_counter() - t1
    f = ToAFitter(x, off, E, tm)
    ops.toa_fit_redchi2(f.x, f.offsets, f.tpl, f._arr(f.E, np.float64), f.norm0, f.res, True, False, f._arr(f._bins()[0], np.float64), f._arr(f._bins()[1], np.float64), 2, flags=N.FLAG_TIME_KERNELS)
    g_ms, f_ms = N.last_kernel_times()[:2]
    print("lib %s: %d x %d photons: %.1f ms (grid %.2f ms, fit %.2f ms), %.4g fits/s, phShi[0:3] %s" % (
        os.path.basename(N.LIB_PATH), nint, nph, el * 1e3, g_ms, f_ms, nint / el, r["phShi"][:3]), flush=True)

"""Repeatability diagnostic: the same search repeated must give identical results."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from crimp_amd import ops  # noqa: E402
from crimp_amd import _native as N  # noqa: E402
from crimp_amd.synth import pulsed_events  # noqa: E402
from oracle import oracle as O  # noqa: E402

ev = pulsed_events(300000, 3.0e5, 5.0, pulsed_frac=0.02, seed=12)
ff = 5.0 + np.arange(-1024, 1024) / 3.0e6
t0 = (ev[0] + ev[-1]) / 2
zr = O.search(ev, ff, 2)
for name, fl in (("poly", N.FLAG_FORCE_DIRECT), ("hw", N.FLAG_FORCE_DIRECT | N.FLAG_HW_SINCOS),
                 ("mfma", N.FLAG_FORCE_MFMA)):
    res = [ops.search(ev, t0, ff, 2, 0, flags=fl) for _ in range(4)]
    errs = ["%.3g" % (np.abs(r - zr) / np.maximum(zr, zr.mean())).max() for r in res]
    same = all(np.array_equal(res[0], r) for r in res[1:])
    print(name, "repeat-identical", same, "errs", errs, "nan", [int(np.isnan(r).sum()) for r in res], flush=True)

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
zr = O.search(ev, ff, 4)
for name, fl in (("direct-poly", N.FLAG_FORCE_DIRECT), ("mfma", N.FLAG_FORCE_MFMA)):
    z = ops.search(ev, t0, ff, 4, 0, flags=fl)
    e = np.abs(z - zr) / np.maximum(zr, zr.mean())
    order = np.argsort(e)[-6:]
    print(name, [(int(j), float(z[j]), float(zr[j]), float(e[j])) for j in order], flush=True)

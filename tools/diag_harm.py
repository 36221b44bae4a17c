"""Per-harmonic error diagnostic for the search kernels."""
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
zr = [O.search(ev, ff, m) for m in range(1, 10)]
for name, fl in (("direct-poly", N.FLAG_FORCE_DIRECT), ("direct-hw", N.FLAG_FORCE_DIRECT | N.FLAG_HW_SINCOS),
                 ("mfma", N.FLAG_FORCE_MFMA)):
    zs = [ops.search(ev, t0, ff, m, 0, flags=fl) for m in range(1, 10)]
    out = []
    for m in range(9):
        sc = np.maximum(zr[m], zr[m].mean())
        out.append("m%d:%.2g" % (m + 1, (np.abs(zs[m] - zr[m]) / sc).max()))
    # per-harmonic contributions
    ph = []
    for m in range(9):
        gk = zs[m] - (zs[m - 1] if m else 0)
        rk = zr[m] - (zr[m - 1] if m else 0)
        ph.append("k%d:%.2g" % (m + 1, (np.abs(gk - rk) / np.maximum(rk, rk.mean())).max()))
    print(name, " ".join(out), "|", " ".join(ph), flush=True)
# small N check of single harmonics k with tiny photon count
t2 = np.array([5.0e9, 5.0e9 + 12345.678901, 5.0e9 + 22222.2])
f2 = 5.0 + np.arange(300) * 1e-3
for m in (1, 2, 3, 4, 5, 8):
    g = ops.search(t2, (t2[0] + t2[-1]) / 2, f2, m, 0, flags=N.FLAG_FORCE_DIRECT)
    r = O.search(t2, f2, m)
    print("3 photons m=%d direct max abs err %.3g" % (m, np.abs(g - r).max()), flush=True)

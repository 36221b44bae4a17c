"""Where does the f16-split kernel lose accuracy? Error vs the oracle by photon count and harmonic count."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from crimp_amd import ops, _native as N  # noqa: E402
from crimp_amd.synth import pulsed_events  # noqa: E402
from oracle import oracle as O  # noqa: E402


def scaled(got, ref):
    return float((np.abs(got - ref) / np.maximum(np.abs(ref), np.mean(np.abs(ref)))).max())


for n in (32, 64, 2048, 65536, 300000):
    t = pulsed_events(n, 3.0e5, 5.0, pulsed_frac=0.02, seed=7)
    f = 5.0 + (np.arange(1024) - 512) / 3.0e6
    t0 = (t[0] + t[-1]) / 2
    for m in (1, 2, 3):
        ref = O.search(t, f, m)
        line = "n=%6d m=%d:" % (n, m)
        for name, fl in (("f32", N.FLAG_MFMA_F32), ("f16", 0)):
            got = ops.search(t, t0, f, m, 0, flags=fl | N.FLAG_FORCE_MFMA)
            e = np.abs(got - ref) / np.maximum(np.abs(ref), np.mean(np.abs(ref)))
            line += "  %s max %.3g (at %d) median %.3g" % (name, e.max(), int(e.argmax()), np.median(e))
        print(line, flush=True)

"""GPU diagnostic: precision of the search kernels (direct poly / direct hw / mfma) vs the oracle."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from crimp_amd import ops  # noqa: E402
from crimp_amd import _native as N  # noqa: E402
from crimp_amd.synth import pulsed_events  # noqa: E402
from oracle import oracle as O  # noqa: E402


def err(z, zr):
    sc = np.maximum(np.abs(zr), zr.mean())
    e = np.abs(z - zr) / sc
    return "max %.3g mean %.3g argmax_ok %s" % (e.max(), e.mean(), int(np.argmax(z)) == int(np.argmax(zr)))


def run(t, f, m, stat=0, fd=None, label=""):
    t0 = (t[0] + t[-1]) / 2
    zr = O.search(t, f, m, freq_dot=fd, stat="z2" if stat == 0 else "h")
    for name, fl in (("direct-poly", N.FLAG_FORCE_DIRECT), ("direct-hw", N.FLAG_FORCE_DIRECT | N.FLAG_HW_SINCOS),
                     ("mfma", N.FLAG_FORCE_MFMA)):
        try:
            z = ops.search(t, t0, f, m, stat, log10_negfdot=fd, flags=fl)
            print("%-28s %-12s %s" % (label, name, err(z, zr)), flush=True)
        except Exception as e:  # noqa: BLE001
            print("%-28s %-12s ERROR %s" % (label, name, e), flush=True)


g = np.load(os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "periodsearch_synth.npz"))
t, f = g["time"], g["freq"]
run(t, f, 1, label="synth6000 m1")
run(t, f, 2, label="synth6000 m2")
# f = 0 trial: every phase is 0, Z2 = 2N*m exactly
tt = pulsed_events(100000, 1e5, 1.0, seed=1)
t0 = (tt[0] + tt[-1]) / 2
for fl in (N.FLAG_FORCE_DIRECT, N.FLAG_FORCE_DIRECT | N.FLAG_HW_SINCOS):
    z = ops.search(tt, t0, np.zeros(4), 2, 0, flags=fl)
    print("f=0 Z2 (expect %g):" % (2 * 2 * 100000 / 100000 * 100000 / 1), z)
# two photons: Z2_1 = 2 + 2 cos(2 pi f (t1 - t2))
t2 = np.array([5.0e9, 5.0e9 + 12345.678901])
f2 = np.linspace(0.1, 10.0, 1000)
z = ops.search(t2, (t2[0] + t2[1]) / 2, f2, 1, 0, flags=N.FLAG_FORCE_DIRECT)
ex = 2 + 2 * np.cos(2 * np.pi * f2 * (t2[1] - t2[0]))
print("two photons max abs err", np.abs(z - ex).max())
ev = pulsed_events(300000, 3.0e5, 5.0, pulsed_frac=0.02, seed=12)
ff = 5.0 + np.arange(-1024, 1024) / 3.0e6
run(ev, ff, 2, label="300k x 2048 m2")
run(ev, ff, 5, stat=1, label="300k x 2048 H m5")
run(ev, ff[:1500], 2, fd=np.array([-12.0, -11.0]), label="300k 2D m2")

"""Raw exact-kernel powers (fix-up disabled: CRIMP_FIXUP_REL=1e30) of the 2-D search of
tests/test_gpu_parity.py::test_search_sharded_ranges_equal_full and a 1-D one, against the fp64 path."""
import os, sys, numpy as np
sys.path.insert(0, '/root/repo' if os.path.exists('/root/repo') else '.')
from crimp_amd import ops, _native as N
from crimp_amd.synth import pulsed_events
t = pulsed_events(50000, 1.0e5, 3.0, pulsed_frac=0.1, seed=9)
f = 3.0 + np.arange(-300, 300) / 1.0e6
t0 = (t[0] + t[-1]) / 2
for fd in (None, np.array([-12.0, -11.0])):
    ref = ops.search(t, t0, f, 2, 0, log10_negfdot=fd, precision="f64")
    z = ops.search(t, t0, f, 2, 0, log10_negfdot=fd)
    r = np.abs(z - ref) / np.abs(ref)
    bad = np.nonzero(r > 1e-6)[0]
    print("2-D" if fd is not None else "1-D", "fixups", N.load().crimp_last_fixups(), "max rel %.3g" % r.max(),
          "bad", bad.size, bad[:16], flush=True)
    for i in bad[:6]:
        print("   trial %d: exact %.9g f64 %.9g" % (i, z[i], ref[i]))

"""Which trials differ between a 2-D search and its trial partitions (tests/test_gpu_parity.py::
test_search_sharded_ranges_equal_full), against repeat runs and the fp64 path. CRIMP_LIB selects a build."""
import os, sys, numpy as np
sys.path.insert(0, '/root/repo' if os.path.exists('/root/repo') else '.')
from crimp_amd import ops, _native as N
from crimp_amd.synth import pulsed_events
t = pulsed_events(50000, 1.0e5, 3.0, pulsed_frac=0.1, seed=9)
f = 3.0 + np.arange(-300, 300) / 1.0e6
fd = np.array([-12.0, -11.0])
t0 = (t[0] + t[-1]) / 2
ref = ops.search(t, t0, f, 2, 0, log10_negfdot=fd, precision="f64")
fulls = []
for r in range(3):
    fulls.append(ops.search(t, t0, f, 2, 0, log10_negfdot=fd)); print("full fixups", N.load().crimp_last_fixups())
for r in range(1, 3):
    d = np.nonzero(fulls[r] != fulls[0])[0]
    print("repeat", r, "differs at", d[:20], d.size)
parts = []
for a, b in ((0, 333), (333, 901), (901, 1200)):
    parts.append(ops.search(t, t0, f, 2, 0, log10_negfdot=fd, first=a, count=b - a))
    print("part", a, b, "fixups", N.load().crimp_last_fixups())
pc = np.concatenate(parts)
d = np.nonzero(pc != fulls[0])[0]
print("partition differs at", d, d.size)
for i in d[:12]:
    print("  trial %4d row %d col %3d: full %.9g part %.9g f64 %.9g" % (i, i // 600, i % 600, fulls[0][i], pc[i], ref[i]))
rel = lambda z: np.max(np.abs(z - ref) / np.abs(ref))
print("max rel vs f64: full %.3g parts %.3g" % (rel(fulls[0]), rel(pc)))

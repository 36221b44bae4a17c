"""A/B timing of library builds (build/variants/*.so, or 'cur' = crimp_amd/lib) on the config-5 ToA fit (1250
intervals x 1e5 photons, 1e2259 template, brute grid + MLE + 1-sigma scan); each build in its own process.
Prints the brute-grid / fit kernel times and a digest of the fitted records (equal digests = identical fits).
usage: python tools/ab_toa.py name1 name2 ...  (NINT, NPER, REPS from the environment)"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import os, sys, hashlib, numpy as np, torch
sys.path.insert(0, %r)
import bench
from crimp_amd import ops, _native as N
from crimp_amd.synth import template_intervals_torch
from crimp_amd.toafit import ToAFitter
nint, nper = int(os.environ.get("NINT", 1250)), int(os.environ.get("NPER", 100000))
tm = bench._tmpl()
x, off, E, shifts = template_intervals_torch(nint, nper, bench.T2259["norm"]["value"], bench.T2259["amp"],
                                             bench.T2259["ph"], seed=2, device="cuda")
res = ToAFitter(x, off, E, tm).fit(brutemin=True); torch.cuda.synchronize()
g, k = [], []
for _ in range(int(os.environ.get("REPS", 3))):
    f = ToAFitter(x, off, E, tm)
    ops.toa_fit_redchi2(f.x, f.offsets, f.tpl, f._arr(f.E, np.float64), f.norm0, f.res, True, False, f._arr(f._bins()[0], np.float64), f._arr(f._bins()[1], np.float64), 2, flags=N.FLAG_TIME_KERNELS)
    gm, km = N.last_kernel_times()[:2]; g.append(gm); k.append(km)
h = hashlib.sha1()
for key in sorted(res):
    v = np.asarray(res[key])
    if v.dtype.kind in "fiu": h.update(np.ascontiguousarray(v).tobytes())
print("%%-12s k_toa_grid %%.2f ms (min %%.2f)  k_toa_fit %%.2f ms  fits digest %%s" %% (sys.argv[1], np.mean(g), min(g),
      np.mean(k), h.hexdigest()[:16]), flush=True)
''' % ROOT

for name in sys.argv[1:]:
    lib = os.path.join(ROOT, "crimp_amd", "lib", "libcrimp_hip.so") if name == "cur" else \
        os.path.join(ROOT, "build", "variants", name + ".so")
    r = subprocess.run([sys.executable, "-c", CHILD, name], env=dict(os.environ, CRIMP_LIB=lib), timeout=300)
    if r.returncode != 0:
        print("variant %s failed rc=%d" % (name, r.returncode), flush=True)
        sys.exit(r.returncode)

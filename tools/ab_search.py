"""A/B timing of library builds (build/variants/*.so) on one search workload; each build in its own process.
usage: python tools/ab_search.py name1 name2 ...  (NPH, NTR, NHARM, PREC, REPS, NFD, DUMP from the environment)"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import os, sys, time, hashlib, numpy as np, torch
sys.path.insert(0, %r)
from crimp_amd import ops, _native as N
from crimp_amd.synth import pulsed_events
n, M, m = int(os.environ.get("NPH", 10_000_000)), int(os.environ.get("NTR", 1_000_000)), int(os.environ.get("NHARM", 2))
prec = os.environ.get("PREC") or None
span, f0 = 1.0e6, 7.123456789
t_h = pulsed_events(n, span, f0, pulsed_frac=0.1, seed=0)
t = torch.as_tensor(t_h, device="cuda"); f = torch.as_tensor(f0 + (np.arange(M) - M // 2) / (10 * span), device="cuda")
t0 = (t_h[0] + t_h[-1]) / 2
nfd = int(os.environ.get("NFD", 0))  # > 0: the 2-D grid, nfd fd rows of M trials
fd = torch.as_tensor(np.linspace(-14.0, -12.0, nfd), device="cuda") if nfd else None
M = M * max(nfd, 1)
z = ops.search(t, t0, f, m, 0, fd, precision=prec); torch.cuda.synchronize()
ks = []
for _ in range(int(os.environ.get("REPS", 3))):
    z = ops.search(t, t0, f, m, 0, fd, precision=prec, flags=N.FLAG_TIME_KERNELS); ks.append(N.load().crimp_last_kernel_ms())
zz = z.cpu().numpy()
if os.environ.get("DUMP"):  # the per-trial powers, for a trial-by-trial comparison of builds
    np.save(os.path.join(os.environ["DUMP"], sys.argv[1] + ".npy"), zz)
print("%%-12s kernels %%.1f ms (min %%.1f)  %%.3e evals/s  argmax %%d  sum %%.17g  digest %%s" %% (sys.argv[1], np.mean(ks),
      min(ks), n * M / (min(ks) * 1e-3), int(np.argmax(zz)), float(zz.sum()), hashlib.sha1(zz.tobytes()).hexdigest()[:12]),
      flush=True)
''' % ROOT

for name in sys.argv[1:]:
    env = dict(os.environ, CRIMP_LIB=os.path.join(ROOT, "build", "variants", name + ".so"))
    r = subprocess.run([sys.executable, "-c", CHILD, name], env=env, timeout=300)
    if r.returncode != 0:
        print("variant %s failed rc=%d" % (name, r.returncode), flush=True)
        sys.exit(r.returncode)

import os, sys, time
import numpy as np, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from crimp_amd import ops, _native as N
from crimp_amd.sharding import sharded_search
from crimp_amd.synth import pulsed_events
span, f0 = 1.0e6, 7.123456789
t_h = pulsed_events(10_000_000, span, f0, pulsed_frac=0.1, seed=0)
dev = torch.device("cuda", 0)
t = torch.as_tensor(t_h, device=dev)
f = torch.as_tensor(f0 + (np.arange(1_000_000) - 500_000) / (10 * span), device=dev)
t0 = (t_h[0] + t_h[-1]) / 2
out = torch.empty(1_000_000, dtype=torch.float64, device=dev)
def tm(fn, k=20):
    for _ in range(3): fn()
    torch.cuda.synchronize(); a = time.perf_counter()
    for _ in range(k): fn()
    torch.cuda.synchronize(); return (time.perf_counter() - a) / k * 1e3
print("ops.search out=given   %.3f ms" % tm(lambda: ops.search(t, t0, f, 2, 0, out=out, precision="nufft")))
print("ops.search out=None    %.3f ms" % tm(lambda: ops.search(t, t0, f, 2, 0, precision="nufft")))
print("sharded best           %.3f ms" % tm(lambda: sharded_search(t, f, 2, 0, gather="best", precision="nufft", t0=t0)))
z = ops.search(t, t0, f, 2, 0, out=out, precision="nufft")
def best():
    v, i = torch.max(z, 0); return torch.stack([v, i.to(torch.float64)]).cpu().numpy()
print("max+stack+cpu          %.3f ms" % tm(best))
print("search+sync only       %.3f ms" % tm(lambda: (ops.search(t, t0, f, 2, 0, out=out, precision="nufft"), torch.cuda.synchronize())))
print("ops.best alone         %.3f ms" % tm(lambda: ops.best(z)))
def torch_best():
    v, i = torch.max(z, 0); return torch.stack([v, i.to(torch.float64)]).cpu().numpy()
print("search+ops.best        %.3f ms" % tm(lambda: (ops.search(t, t0, f, 2, 0, out=out, precision="nufft"), ops.best(out))))
print("search+torch best      %.3f ms" % tm(lambda: (ops.search(t, t0, f, 2, 0, out=out, precision="nufft"), torch_best())))
print("sharded best (again)   %.3f ms" % tm(lambda: sharded_search(t, f, 2, 0, gather="best", precision="nufft", t0=t0)))

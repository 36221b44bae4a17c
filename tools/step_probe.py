"""Where the time of one config-3 search step goes outside the kernels: the C-ABI call through ops.search, the raw
ctypes call with prepared pointers (no Python wrapper), search + best (two calls) against crimp_search_best (one),
sharded_search(gather='best') (bench.py's step), and the library's own pipeline span (first kernel to last).
usage: python tools/step_probe.py"""
import ctypes
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from crimp_amd import ops, _native as N  # noqa: E402
from crimp_amd.sharding import sharded_search  # noqa: E402
from crimp_amd.synth import pulsed_events  # noqa: E402

span, f0 = 1.0e6, 7.123456789
t_h = pulsed_events(10_000_000, span, f0, pulsed_frac=0.1, seed=0)
dev = torch.device("cuda", 0)
t = torch.as_tensor(t_h, device=dev)
f = torch.as_tensor(f0 + (np.arange(1_000_000) - 500_000) / (10 * span), device=dev)
t0 = (t_h[0] + t_h[-1]) / 2
out = torch.empty(1_000_000, dtype=torch.float64, device=dev)
L = N.load()


def tm(fn, k=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a = time.perf_counter()
    for _ in range(k):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - a) / k * 1e3


stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
res = np.zeros(2)


def raw():
    N.check(L.crimp_search(ctypes.c_void_p(t.data_ptr()), t.numel(), t0, ctypes.c_void_p(f.data_ptr()), f.numel(),
                           None, 0, 2, 0, 0, out.numel(), ctypes.c_void_p(out.data_ptr()), N.FLAG_DEVICE_PTRS, stream))


ARGS = (ctypes.c_void_p(t.data_ptr()), t.numel(), t0, ctypes.c_void_p(f.data_ptr()), f.numel(), None, 0, 2, 0, 0,
        out.numel(), ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(res.ctypes.data), N.FLAG_DEVICE_PTRS, stream)


def raw_best():
    N.check(L.crimp_search_best(*ARGS))


rows = [("ops.search out=given", lambda: ops.search(t, t0, f, 2, 0, out=out)),
        ("ops.search out=None", lambda: ops.search(t, t0, f, 2, 0)),
        ("raw ctypes crimp_search", raw),
        ("raw ctypes crimp_search_best", raw_best),
        ("ops.search + ops.best", lambda: (ops.search(t, t0, f, 2, 0, out=out), ops.best(out))),
        ("ops.search_best", lambda: ops.search_best(t, t0, f, 2, 0, out=out)),
        ("sharded_search best (bench step)", lambda: sharded_search(t, f, 2, 0, gather="best", t0=t0)),
        ("raw best, plan cache off", lambda: (os.environ.__setitem__("CRIMP_NUFFT_PLAN_CACHE", "0"), raw_best(),
                                              os.environ.pop("CRIMP_NUFFT_PLAN_CACHE"))),
        ("ops.best alone", lambda: ops.best(out))]
for name, fn in rows:
    print("%-34s %.3f ms" % (name, tm(fn)), flush=True)
spans = []
for _ in range(10):
    ops.search(t, t0, f, 2, 0, out=out, flags=N.FLAG_TIME_KERNELS)
    spans.append(N.last_kernel_times()[:15])
sp = np.mean(np.array(spans), axis=0)
print("pipeline span (first kernel mark to last) %.3f ms; classes %s" % (
    sp[0], ", ".join("%s %.3f" % (c, v) for c, v in zip(N.NUFFT_CLASSES, sp[1:8]))), flush=True)

"""Host overhead of one config-3 search step, layer by layer: bench's sharded_search(gather="best"), ops.search_best,
and crimp_search_best called straight through ctypes with prepared pointers (the C-ABI alone). The differences are
the Python layers' cost per step; the C-ABI line minus the kernels' sum is the library's own host + launch cost.
usage: python tools/step_overhead.py [steps]"""
import ctypes
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from crimp_amd import _native as N  # noqa: E402
from crimp_amd import ops  # noqa: E402
from crimp_amd.sharding import sharded_search  # noqa: E402
from crimp_amd.synth import pulsed_events  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    span, f0, M = 1.0e6, 7.123456789, 1_000_000
    t_h = pulsed_events(10_000_000, span, f0, pulsed_frac=0.1, seed=0)
    f_h = f0 + (np.arange(M) - M // 2) * (1.0 / (10.0 * span))
    t = torch.as_tensor(t_h, device=dev)
    f = torch.as_tensor(f_h, device=dev)
    t0 = (t_h[0] + t_h[-1]) / 2
    out = torch.empty(M, dtype=torch.float64, device=dev)
    res = np.zeros(2, dtype=np.float64)
    L = N.load()
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    tp, fp, op = ctypes.c_void_p(t.data_ptr()), ctypes.c_void_p(f.data_ptr()), ctypes.c_void_p(out.data_ptr())
    rp = ctypes.c_void_p(res.ctypes.data)
    flags = N.FLAG_DEVICE_PTRS

    def raw():
        N.check(L.crimp_search_best(tp, t.numel(), float(t0), fp, M, None, 0, 2, 0, 0, M, op, rp, flags, stream))

    variants = [
        ("sharded_search", lambda: sharded_search(t, f, 2, 0, gather="best", t0=t0)),
        ("ops.search_best", lambda: ops.search_best(t, t0, f, 2, 0, count=M)),
        ("ops.search_best(out=)", lambda: ops.search_best(t, t0, f, 2, 0, count=M, out=out)),
        ("crimp_search_best (ctypes)", raw),
    ]
    for rep in range(2):
        for name, fn in variants:
            ts = time.perf_counter()
            while time.perf_counter() - ts < 0.3:
                fn()
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            for _ in range(steps):
                fn()
            torch.cuda.synchronize()
            el = (time.perf_counter() - t1) / steps
            print("rep %d %-28s %8.1f us per step" % (rep, name, el * 1e6), flush=True)
    N.check(L.crimp_search_best(tp, t.numel(), float(t0), fp, M, None, 0, 2, 0, 0, M, op, rp,
                                flags | N.FLAG_TIME_KERNELS, stream))
    print("kernel pipeline ms (last, timed call):", L.crimp_last_kernel_ms(), "path", L.crimp_last_search_path(),
          flush=True)


if __name__ == "__main__":
    main()

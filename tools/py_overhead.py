"""Per-call host cost of the Python pieces around one search step (no kernels): what sharded_search(gather="best")
-> ops.search_best spends before and after the C-ABI call. usage: python tools/py_overhead.py [reps]"""
import ctypes
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from crimp_amd import _native as N  # noqa: E402
from crimp_amd import ops  # noqa: E402
from crimp_amd import sharding  # noqa: E402


def timeit(name, fn, reps):
    for _ in range(100):
        fn()
    t1 = time.perf_counter()
    for _ in range(reps):
        fn()
    print("%-40s %7.2f us" % (name, (time.perf_counter() - t1) / reps * 1e6), flush=True)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    M = 1_000_000
    t = torch.zeros(10_000_000, dtype=torch.float64, device=dev)
    f = torch.zeros(M, dtype=torch.float64, device=dev)
    out = torch.empty(M, dtype=torch.float64, device=dev)
    L = N.load()

    def bufs():
        b = N.Buffers()
        b.arg(t, np.float64)
        b.arg(f, np.float64)
        b.arg(None, np.float64, allow_none=True)
        b.arg(out, np.float64, writable=True)
        return b

    b = bufs()
    timeit("sharding._dist()", sharding._dist, reps)
    timeit("ops.search_flags()", ops.search_flags, reps)
    timeit("N.load()", N.load, reps)
    timeit("Buffers + 4 args", bufs, reps)
    timeit("torch.empty(1e6 f64, cuda)", lambda: torch.empty(M, dtype=torch.float64, device=dev), reps)

    def guard():
        with b.device_guard():
            pass
    timeit("device_guard enter/exit", guard, reps)
    timeit("Buffers.stream()", b.stream, reps)
    timeit("torch.cuda.current_device()", torch.cuda.current_device, reps)
    timeit("_as_comm(out, dev)", lambda: sharding._as_comm(out, dev), reps)
    timeit("shard_range", lambda: sharding.shard_range(M, 1, 0), reps)
    res = np.zeros(2)
    rp = ctypes.c_void_p(res.ctypes.data)
    timeit("res = np.zeros(2) + c_void_p", lambda: ctypes.c_void_p(np.zeros(2).ctypes.data), reps)
    # a ctypes call of crimp_search_best's arity that fails its argument check at once (nharm = 0): the FFI cost
    timeit("ctypes call, 15 args (rejected)", lambda: L.crimp_search_best(None, 0, 0.0, None, 0, None, 0, 0, 0, 0, 0,
                                                                         None, rp, 0, None), reps)


if __name__ == "__main__":
    main()

"""Host -> device upload of the e2e ToA leg's photon times (1.25e8 fp64 = 1 GB): pageable numpy through
torch.as_tensor, a page-locked torch tensor, a staged copy (numpy -> reusable pinned chunks -> device, the host copy of
chunk k+1 beside the DMA of chunk k), and hipHostRegister of the numpy buffer itself. Mean of REPS after one warm-up.
usage: python tools/upload_ab.py"""
import os
import time

import numpy as np
import torch

n, reps = int(os.environ.get("NPH", 125_000_000)), int(os.environ.get("REPS", 4))
h = np.random.default_rng(1).random(n) + 58000.0
dev = torch.device("cuda", 0)


def timed(fn):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return np.mean(ts), np.min(ts)


def pageable():
    return torch.as_tensor(h, device=dev)


pin = torch.from_numpy(h).pin_memory()


def pinned():
    return pin.to(dev, non_blocking=True)


CH = int(os.environ.get("CHUNK", 1 << 23))  # photons per staging chunk (64 MB)
stage = [torch.empty(CH, dtype=torch.float64).pin_memory() for _ in range(2)]
evs = [torch.cuda.Event() for _ in range(2)]
src = torch.from_numpy(h)


def staged():
    out = torch.empty(n, dtype=torch.float64, device=dev)
    for k, a in enumerate(range(0, n, CH)):
        b = min(n, a + CH)
        j = k & 1
        evs[j].synchronize()  # the DMA that last read this staging buffer is done
        stage[j][: b - a].copy_(src[a:b])
        out[a:b].copy_(stage[j][: b - a], non_blocking=True)
        evs[j].record()
    return out


print("photons %d (%.2f GB)" % (n, n * 8 / 1e9), flush=True)
for name, fn in (("pageable", pageable), ("pinned", pinned), ("staged", staged)):
    m, mn = timed(fn)
    print("%-9s %8.2f ms (min %.2f)  %.1f GB/s" % (name, m * 1e3, mn * 1e3, n * 8 / mn / 1e9), flush=True)
chk = staged()
assert torch.equal(chk.cpu(), src), "staged upload differs"
t0 = time.perf_counter()
pin2 = torch.from_numpy(h).pin_memory()
print("pin_memory() copy of the array: %.2f ms" % ((time.perf_counter() - t0) * 1e3), flush=True)

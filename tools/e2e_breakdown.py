"""Where the bench's end-to-end ToA leg (measure_intervals from host MJD arrays, config 5 per GPU: 1250 intervals x
1e5 photons) spends its time: the steps of crimp_amd.measureToAs.measure_intervals, each bracketed by
torch.cuda.synchronize(), mean of REPS after one warm-up; then the whole call from a pageable numpy array and from a
page-locked torch tensor.
usage: python tools/e2e_breakdown.py"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from crimp_amd import ops  # noqa: E402
from crimp_amd.calcphase import calcphase  # noqa: E402
from crimp_amd.ephemTmjd import ephemTmjd  # noqa: E402
from crimp_amd.measureToAs import measure_intervals  # noqa: E402
from crimp_amd.synth import template_intervals_torch  # noqa: E402
from crimp_amd.toafit import ToAFitter  # noqa: E402

nint, nper, reps = int(os.environ.get("NINT", 1250)), 100000, int(os.environ.get("REPS", 3))
tm = bench._tmpl()
dev = torch.device("cuda", 0)
x, off, E, _ = template_intervals_torch(nint, nper, bench.T2259["norm"]["value"], bench.T2259["amp"],
                                        bench.T2259["ph"], seed=2, device=dev)
F0, pep = 0.5, 58000.0
mjd = (pep + ((torch.arange(x.numel(), device=dev, dtype=torch.float64) + x) / F0) / 86400.0).cpu().numpy()
offh = off.cpu().numpy()
starts, ends = mjd[offh[:-1]] - 1e-9, mjd[offh[1:] - 1] + 1e-9
E = E.cpu().numpy() if hasattr(E, "cpu") else np.asarray(E)
par = {"PEPOCH": pep, "F0": F0}
del x
torch.cuda.empty_cache()


def steps():
    t = {}

    def mark(k, t0):
        torch.cuda.synchronize()
        t[k] = (time.perf_counter() - t0) * 1e3
        return time.perf_counter()

    t0 = time.perf_counter()
    T = torch.as_tensor(mjd, device=dev)
    t0 = mark("upload", t0)
    ok = bool((T[1:] >= T[:-1]).all())
    t0 = mark("sorted_check", t0)
    lo = torch.searchsorted(T, torch.as_tensor(starts, device=dev), right=False)
    hi = torch.maximum(torch.searchsorted(T, torch.as_tensor(ends, device=dev), right=True), lo)
    n = (hi - lo).cpu().numpy()
    offs = np.concatenate([[0], np.cumsum(n)]).astype(np.int64)
    t0 = mark("searchsorted", t0)
    rel = torch.arange(int(offs[-1]), device=dev, dtype=torch.int64)
    seg = torch.repeat_interleave(torch.arange(n.size, device=dev), torch.as_tensor(n, device=dev))
    offs_d = torch.as_tensor(offs, device=dev)
    allt = T[lo[seg] + (rel - offs_d[seg])]
    first, last = allt[offs_d[:-1]], allt[offs_d[1:] - 1]
    mids = (((last - first) / 2) + first).cpu().numpy()
    t0 = mark("gather", t0)
    _, folded = calcphase(allt, par)
    t0 = mark("calcphase", t0)
    res = ToAFitter(folded, offs, E, tm).fit(brutemin=True)
    t0 = mark("fit+redchi2", t0)
    freqs = np.atleast_1d(ephemTmjd(mids, par)["freqAtTmjd"])
    hp = ops.search_sets(allt * 86400, torch.as_tensor(offs, device=dev),
                         torch.as_tensor(freqs, dtype=torch.float64, device=dev), 5, 1).cpu().numpy()
    t0 = mark("htest", t0)
    assert ok and hp.size == nint and res["phShi"].size == nint
    return t


steps()
acc = {}
for _ in range(reps):
    for k, v in steps().items():
        acc.setdefault(k, []).append(v)
tot = 0.0
for k, v in acc.items():
    tot += np.mean(v)
    print("%-13s %8.3f ms (min %.3f)" % (k, np.mean(v), np.min(v)), flush=True)
print("%-13s %8.3f ms" % ("sum", tot), flush=True)
pin = torch.from_numpy(mjd).pin_memory()
runs = [("numpy", mjd, b) for b in os.environ.get("BLOCKS", "1,4,d").split(",")] + [("pinned", pin, "d")]
for name, src, nbk in runs:  # nbk: "1" one shot, "n" n blocks of shares n : ... : 1, "un" n equal blocks, "wa/b/..." shares a : b : ..., "d" default
    os.environ.pop("CRIMP_E2E_BLOCKS", None)
    os.environ.pop("CRIMP_E2E_WEIGHTS", None)
    if nbk.startswith("w"):  # "w1/1/0.5": those shares
        os.environ.pop("CRIMP_E2E_MIN_PHOTONS", None)
        os.environ["CRIMP_E2E_WEIGHTS"] = nbk[1:].replace("/", ",")
    elif nbk.startswith("u"):
        os.environ.pop("CRIMP_E2E_MIN_PHOTONS", None)
        os.environ["CRIMP_E2E_WEIGHTS"] = ",".join(["1"] * int(nbk[1:]))
    elif nbk == "1":
        os.environ["CRIMP_E2E_MIN_PHOTONS"] = str(1 << 62)
    else:
        os.environ.pop("CRIMP_E2E_MIN_PHOTONS", None)
        if nbk != "d":
            os.environ["CRIMP_E2E_BLOCKS"] = nbk
    name = "%s/%s blocks" % (name, nbk)
    measure_intervals(src, par, tm, starts, ends, E, brutemin=True)
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        measure_intervals(src, par, tm, starts, ends, E, brutemin=True)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    print("measure_intervals from %-16s %8.3f ms (min %.3f), %.4g fits/s" % (name, np.mean(ts) * 1e3, np.min(ts) * 1e3,
                                                                          nint / np.mean(ts)), flush=True)
os.environ.pop("CRIMP_E2E_MIN_PHOTONS", None)
os.environ.pop("CRIMP_E2E_BLOCKS", None)
os.environ.pop("CRIMP_E2E_WEIGHTS", None)
if os.environ.get("TRACE_WEIGHTS"):
    os.environ["CRIMP_E2E_WEIGHTS"] = os.environ["TRACE_WEIGHTS"]
os.environ["CRIMP_E2E_TRACE"] = "1"
for _ in range(2):  # the pipeline's timeline: upload done / block start / block done per block
    measure_intervals(mjd, par, tm, starts, ends, E, brutemin=True)

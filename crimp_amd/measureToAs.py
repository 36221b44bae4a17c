"""Drop-in ``measureToAs`` / ``measureToA_*`` / ``measuretoas`` CLI on the MI355X.

Same signatures, return values, output text file and CLI flags as CRIMP v2.3.0
``measureToAs.py`` (:64-251 ToA loop, :254-693 per-template fits, :698-806
initial parameters, :951-1003 CLI). The per-interval likelihood work runs in
batches on the device (crimp_amd/toafit.py); the loop body keeps the
reference's order of operations and its text formatting (``str()`` of each value,
tab-separated, 13 columns, :161-162, :222-226).

``varyAmps`` runs on the device (crimp_toa_fit); ``readvaryparam`` frees the template parameters
flagged ``vary True`` (crimp_amd/toafit_vary.py, photon sums on the device through
crimp_toa_shape_points); with both, ampShift is freed after the readvaryparam fit (:306-312).
"""
import argparse
import math
import sys
import time

import numpy as np

from .calcphase import Phases
from .ephemTmjd import ephemTmjd
from .eventfile import EvtFileOps
from .logging_utils import configure_logging, get_logger
from . import ops
from ._native import FLAG_TIME_DAYS, STAT_H
from .readPPtemplate import readPPtemplate
from .readtimingmodel import ReadTimingModel
from .timfile import phshiftTotimfile
from .toafit import ToAFitter, warn_capped
from .toafit_vary import VaryParamFitter

logger = get_logger(__name__)


class Param:
    """Minimal stand-in for an lmfit Parameter (value / min / max / vary / brute_step)."""

    def __init__(self, name, value, vary=True, min=-np.inf, max=np.inf, brute_step=None):  # noqa: A002
        self.name, self.value, self.vary, self.min, self.max, self.brute_step = name, value, vary, min, max, brute_step

    def __float__(self):
        return float(min(max(self.value, self.min), self.max))

    def __repr__(self):
        return "<Param %s=%r vary=%s bounds=[%r, %r]>" % (self.name, self.value, self.vary, self.min, self.max)


def defineinitialfitparam(tempModPP, readvaryparam=False):
    """Initial parameters and number of free parameters (measureToAs.py:698-806)."""
    model = tempModPP["model"]
    if readvaryparam:
        if model not in ("fourier", "vonmises", "cauchy"):
            raise ValueError("Unknown template model. Only fourier, cauchy, or vonmises are supported")
        K = len([k for k in tempModPP if k.startswith("amp_")])
        n0 = tempModPP["norm"]["value"]
        p = {"norm": Param("norm", n0, tempModPP["norm"]["vary"], n0 / 5, n0 * 5)}
        nfree = 1 if tempModPP["norm"]["vary"] else 0
        for k in range(1, K + 1):
            if model == "fourier":
                a, ph = tempModPP["amp_%d" % k], tempModPP["ph_%d" % k]
                p["amp_%d" % k] = Param("amp_%d" % k, a["value"], a["vary"], 0, 1000)
                p["ph_%d" % k] = Param("ph_%d" % k, ph["value"], ph["vary"], -np.pi, np.pi)
                nfree += int(bool(a["vary"])) + int(bool(ph["vary"]))
            else:
                a, c, w = (tempModPP["%s_%d" % (nm, k)] for nm in ("amp", "cen", "wid"))
                p["amp_%d" % k] = Param("amp_%d" % k, a["value"], a["vary"], 0, 5 * a["value"])
                p["cen_%d" % k] = Param("cen_%d" % k, c["value"], c["vary"], -0.6 + c["value"], 0.6 + c["value"], 0.05)
                p["wid_%d" % k] = Param("wid_%d" % k, w["value"], w["vary"], 0, 30 * np.pi)
                nfree += int(bool(a["vary"])) + int(bool(c["vary"])) + int(bool(w["vary"]))
        pb = np.pi if model == "fourier" else 1.5 * np.pi
        p["phShift"] = Param("phShift", 0, True, -pb, pb, 0.05)
        p["ampShift"] = Param("ampShift", 1, False, *((0, 100) if model == "fourier" else (-np.inf, np.inf)))
        return p, nfree
    K = len([k for k in tempModPP if k.startswith("amp_")])
    n0 = tempModPP["norm"]["value"]
    p = {"norm": Param("norm", n0, True, n0 / 100, 500)}
    if model == "fourier":
        for k in range(1, K + 1):
            p["amp_%d" % k] = Param("amp_%d" % k, tempModPP["amp_%d" % k]["value"], False)
            p["ph_%d" % k] = Param("ph_%d" % k, tempModPP["ph_%d" % k]["value"], False)
        p["phShift"] = Param("phShift", 0, True, -np.pi, np.pi, 0.05)
        p["ampShift"] = Param("ampShift", 1, False, 0, 100)
    elif model in ("vonmises", "cauchy"):
        for k in range(1, K + 1):
            for nm in ("amp", "cen", "wid"):
                key = "%s_%d" % (nm, k)
                p[key] = Param(key, tempModPP[key]["value"], False)
        p["phShift"] = Param("phShift", 0, True, -1.5 * np.pi, 1.5 * np.pi, 0.05)
        p["ampShift"] = Param("ampShift", 1, False, -np.pi, np.pi)
    else:
        raise ValueError("Unknown template model. Only fourier, cauchy, or vonmises are supported")
    return p, 2


def _single(model, tempModPP, phases, exposureInt, phShiftRes, nbrBins, varyAmps, brutemin, readvaryparam,
            plotLLs, plotPPs, outFile=''):
    if str(tempModPP["model"]).lower() != model:
        raise ValueError("template model %s used with measureToA_%s" % (tempModPP["model"], model))
    x = np.ascontiguousarray(np.ravel(phases), dtype=np.float64)
    if readvaryparam:
        r = VaryParamFitter(x, np.array([0, x.size]), np.array([float(exposureInt)]), tempModPP, phShiftRes,
                            nbrBins, vary_amps=bool(varyAmps)).fit(brutemin=brutemin)
    else:
        fit = ToAFitter(x, np.array([0, x.size]), np.array([float(exposureInt)]), tempModPP, phShiftRes, nbrBins)
        r = fit.fit(brutemin=brutemin, vary_amps=bool(varyAmps))
    warn_capped(r, phShiftRes, [outFile], logger)                 # measureToAs.py:348-350, :373-375
    if plotLLs or plotPPs:
        logger.warning("plotPPs/plotLLs are diagnostic plots and are not produced by this build")
    return {"phShi": float(r["phShi"][0]), "phShi_LL": float(r["phShi_LL"][0]), "phShi_UL": float(r["phShi_UL"][0]),
            "reducedChi2": float(r["reducedChi2"][0])}


def measureToA_fourier(tempModPP, cycleFoldedPhases, exposureInt, outFile='', phShiftRes=1000, nbrBins=15,
                       varyAmps=False, brutemin=False, plotPPs=False, plotLLs=False, readvaryparam=False):
    """Fourier-template ToA (measureToAs.py:254-403); phases in cycles [0,1)."""
    return _single("fourier", tempModPP, cycleFoldedPhases, exposureInt, phShiftRes, nbrBins, varyAmps, brutemin,
                   readvaryparam, plotLLs, plotPPs, outFile)


def measureToA_cauchy(tempModPP, cycleFoldedPhases, exposureInt, outFile='', phShiftRes=1000, nbrBins=15,
                      varyAmps=False, brutemin=False, plotPPs=False, plotLLs=False, readvaryparam=False):
    """Wrapped-Cauchy ToA (measureToAs.py:406-548); phases in radians [0,2pi)."""
    return _single("cauchy", tempModPP, cycleFoldedPhases, exposureInt, phShiftRes, nbrBins, varyAmps, brutemin,
                   readvaryparam, plotLLs, plotPPs, outFile)


def measureToA_vonmises(tempModPP, cycleFoldedPhases, exposureInt, outFile='', phShiftRes=1000, nbrBins=15,
                        varyAmps=False, brutemin=False, plotPPs=False, plotLLs=False, readvaryparam=False):
    """von Mises ToA (measureToAs.py:551-693); phases in radians [0,2pi)."""
    return _single("vonmises", tempModPP, cycleFoldedPhases, exposureInt, phShiftRes, nbrBins, varyAmps, brutemin,
                   readvaryparam, plotLLs, plotPPs, outFile)


HEADER = ('ToA \t ToA_mid \t ToA_start \t ToA_end \t ToA_lenInt \t ToA_exp \t nbr_events \t count_rate \t phShift'
          ' \t phShift_LL \t phShift_UL \t Hpower \t redChi2\n')


def select_intervals(TIMEMJD, starts, ends):
    """Concatenated photons of every interval [start, end] (inclusive, measureToAs.py:173-174) and the offsets.
    Time-sorted input (event files are): two binary searches per interval; otherwise the reference's mask."""
    T = np.asarray(TIMEMJD, dtype=np.float64)
    starts, ends = np.asarray(starts, dtype=np.float64), np.asarray(ends, dtype=np.float64)
    if T.size < 2 or np.all(T[1:] >= T[:-1]):
        lo = np.searchsorted(T, starts, side="left")
        hi = np.maximum(np.searchsorted(T, ends, side="right"), lo)
        offs = np.concatenate([[0], np.cumsum(hi - lo)]).astype(np.int64)
        idx = np.concatenate([np.arange(a, b) for a, b in zip(lo, hi)]) if len(lo) else np.zeros(0, np.int64)
        return T[idx.astype(np.int64)], offs
    sel = [T[(T >= a) & (T <= b)] for a, b in zip(starts, ends)]
    return (np.concatenate(sel) if sel else np.zeros(0)), np.concatenate([[0], np.cumsum([x.size for x in sel])]).astype(
        np.int64)


def _device_times(TIMEMJD):
    """The photon times as one fp64 CUDA tensor (uploaded once), or None without a GPU. A host torch tensor in
    page-locked memory (``pin_memory()``, e.g. an event reader's staging buffer) goes up by DMA straight from it."""
    from ._native import _is_torch
    import torch
    if _is_torch(TIMEMJD):
        if TIMEMJD.is_cuda:
            return TIMEMJD.reshape(-1).to(torch.float64).contiguous()
        if not torch.cuda.is_available():
            return None
        src = TIMEMJD.reshape(-1).to(torch.float64).contiguous()
        return src.to("cuda", non_blocking=src.is_pinned())
    if not torch.cuda.is_available():
        return None
    return torch.as_tensor(np.ascontiguousarray(TIMEMJD, dtype=np.float64), device="cuda")


def measure_intervals(TIMEMJD, timMod, tempModPP, starts, ends, exposures, phShiftRes=1000, nbrBins=15, varyAmps=False,
                      brutemin=False, readvaryparam=False):
    """Batched core of measureToAs on in-memory arrays: per interval ToA_mid, fit dict entries, H power.
    The timing model is parsed once; the photon times go to the device once, where the intervals are selected
    (binary search on the time-sorted photons, measureToAs.py:173-174), folded in one calcphase call, fitted in
    one device fit and H-tested (:210-212) in one crimp_search_sets launch. Unsorted times take the reference's
    mask on the host."""
    import torch
    tmpl = readPPtemplate(tempModPP) if isinstance(tempModPP, str) else tempModPP
    model = str(tmpl["model"]).lower()
    tm = timMod if isinstance(timMod, dict) else ReadTimingModel(str(timMod)).readfulltimingmodel()[0]
    starts = np.asarray(starts, dtype=np.float64)
    ends = np.asarray(ends, dtype=np.float64)
    if not readvaryparam:
        res = _measure_pipelined(TIMEMJD, tm, tmpl, model, starts, ends, exposures, phShiftRes, nbrBins, varyAmps,
                                 brutemin)
        if res is not None:
            return res
    T = _device_times(TIMEMJD)
    if T is not None and ops.is_sorted(T):
        # time-sorted photons on the device: two binary searches per interval (crimp_select_intervals), the
        # intervals' photons gathered by crimp_gather_ranges -- torch holds the buffers only
        lo, n, first, last = ops.select_intervals(T, starts, ends)
        offs = np.concatenate([[0], np.cumsum(n)]).astype(np.int64)
        if np.any(n <= 0):  # measureToAs.py:182 reads TIME_toa[-1] of every interval
            raise IndexError("index -1 is out of bounds for axis 0 with size 0 (a ToA interval holds no photons)")
        if n.size == 1 or np.all(lo[1:] == lo[:-1] + n[:-1]):
            # consecutive intervals with no photon between them (ToA intervals tiling an observation): their
            # concatenation is a slice of the time array, no copy
            allt = T[int(lo[0]):int(lo[0]) + int(offs[-1])]
        else:
            allt = ops.gather_ranges(T, lo, offs)
    else:
        allt, offs = select_intervals(TIMEMJD if T is None else T.cpu().numpy(), starts, ends)
        if np.any(np.diff(offs) <= 0):
            raise IndexError("index -1 is out of bounds for axis 0 with size 0 (a ToA interval holds no photons)")
        first, last = allt[offs[:-1]], allt[offs[1:] - 1]
        if T is not None:
            allt = torch.as_tensor(allt, device=T.device)
    mids = ((last - first) / 2) + first                 # measureToAs.py:182 (host NumPy)
    folded = _folded(allt, tm, model)
    E = np.asarray(exposures, dtype=np.float64)
    if readvaryparam:
        res = VaryParamFitter(folded, offs, E, tmpl, phShiftRes, nbrBins, vary_amps=bool(varyAmps)).fit(
            brutemin=brutemin)
    else:
        res = ToAFitter(folded, offs, E, tmpl, phShiftRes, nbrBins).fit(brutemin=brutemin, vary_amps=bool(varyAmps))
    freqs = np.atleast_1d(ephemTmjd(mids, tm)["freqAtTmjd"])          # :210
    # :211-212, one trial per interval; TIME_toa * 86400 formed in the kernel (CRIMP_FLAG_TIME_DAYS)
    if hasattr(allt, "device"):
        hp = ops.search_sets(allt, torch.as_tensor(offs, device=allt.device),
                             torch.as_tensor(freqs, dtype=torch.float64, device=allt.device), 5, STAT_H,
                             flags=FLAG_TIME_DAYS).cpu().numpy()
    else:
        hp = ops.search_sets(allt, offs, freqs, 5, STAT_H, flags=FLAG_TIME_DAYS)
    res["ToA_mid"] = mids
    res["htestPow"] = np.asarray(hp)
    return res


_HTEST_STREAMS = {}


def _folded(allt, tm, model):
    """The folded phases of the selected photons (measureToAs.py:186-200): calcphase's cycle fold, in radians for the
    Cauchy and von Mises templates -- the host's `folded * (2 * np.pi)` formed in the kernel (CRIMP_FLAG_FOLD_RADIANS,
    the same fp64 multiply)."""
    from ._native import FLAG_FOLD_RADIANS
    ph = Phases(allt, tm)
    _, folded = ops.calcphase(ph.timeMJD, ph.timModParam,
                              flags=FLAG_FOLD_RADIANS if model in ("cauchy", "vonmises") else 0)
    return folded


def _fit_block(allt, offs, mids, tm, tmpl, model, E, phShiftRes, nbrBins, varyAmps, brutemin):
    """Fold, fit and H-test one block of intervals whose photons (device tensor ``allt``, days MJD) are concatenated
    at ``offs`` (measureToAs.py:186-226 for every interval of the block). The per-interval H-test does not depend on
    the fit: it is queued first on a second stream (crimp_search_sets with CRIMP_FLAG_ASYNC) and runs beside the
    folding and the fits."""
    import torch
    from ._native import FLAG_ASYNC
    dev = allt.device
    freqs = np.atleast_1d(ephemTmjd(mids, tm)["freqAtTmjd"])          # :210
    offs_d = torch.as_tensor(offs, device=dev)
    freqs_d = torch.as_tensor(freqs, dtype=torch.float64, device=dev)
    side = _HTEST_STREAMS.get(dev.index)
    if side is None:
        side = _HTEST_STREAMS[dev.index] = torch.cuda.Stream(device=dev)
    cur = torch.cuda.current_stream(dev)
    side.wait_stream(cur)
    with torch.cuda.stream(side):  # :211-212, one trial per interval, TIME_toa * 86400 in the kernel
        hp_d = ops.search_sets(allt, offs_d, freqs_d, 5, STAT_H, flags=FLAG_ASYNC | FLAG_TIME_DAYS)
    for t_ in (allt, offs_d, freqs_d, hp_d):
        t_.record_stream(side)
    folded = _folded(allt, tm, model)
    res = ToAFitter(folded, offs, E, tmpl, phShiftRes, nbrBins).fit(brutemin=brutemin, vary_amps=bool(varyAmps))
    cur.wait_stream(side)
    res["ToA_mid"] = mids
    res["htestPow"] = hp_d.cpu().numpy()
    return res


_UPLOAD_STREAMS = {}


def _measure_pipelined(TIMEMJD, tm, tmpl, model, starts, ends, exposures, phShiftRes, nbrBins, varyAmps, brutemin):
    """measure_intervals for host photon times of at least CRIMP_E2E_MIN_PHOTONS (default 2^24): the intervals are cut
    into consecutive blocks of shrinking size (_E2E_WEIGHTS; CRIMP_E2E_BLOCKS = n: n blocks of shares n : ... : 1;
    CRIMP_E2E_WEIGHTS = "a,b,...": those shares); a second host thread
    uploads block k + 1
    on its own stream (a pageable copy blocks only that thread; torch releases the GIL) while this thread folds, fits
    and H-tests block k on the device, so the PCIe upload hides the device work. Interval selection is the host's
    binary search on the times (measureToAs.py:173-174 for sorted times); every block is checked on the device to be
    sorted (and to continue the previous one), and the whole call is redone by the one-shot path below when one is
    not, or when an interval is empty (its IndexError). Every interval's fit and H test are independent of its block
    (the brute grid's kernel choice is per call: records within the fast-vs-full grid tolerance of the one-shot
    path's, test_measure_intervals_blocks_equal_one_shot). Returns None where it does not apply."""
    import os
    import queue
    import threading
    import torch
    from ._native import _is_torch
    if not torch.cuda.is_available() or (_is_torch(TIMEMJD) and TIMEMJD.is_cuda):
        return None
    src = TIMEMJD.reshape(-1).to(torch.float64).contiguous() if _is_torch(TIMEMJD) else \
        torch.from_numpy(np.ascontiguousarray(TIMEMJD, dtype=np.float64).reshape(-1))
    if src.numel() < int(os.environ.get("CRIMP_E2E_MIN_PHOTONS", 1 << 24)) or starts.size < 2:
        return None
    t = src.numpy()
    lo = np.searchsorted(t, starts, side="left")
    hi = np.maximum(np.searchsorted(t, ends, side="right"), lo)
    n = hi - lo
    if np.any(n <= 0):
        return None
    wenv = os.environ.get("CRIMP_E2E_WEIGHTS")
    nbk = os.environ.get("CRIMP_E2E_BLOCKS")
    weights = [float(v) for v in wenv.split(",")] if wenv else (None if nbk else _E2E_WEIGHTS)
    blocks = _shrinking_blocks(n, len(weights) if weights is not None else int(nbk), weights)
    if len(blocks) < 2:
        return None
    # uploaded photon range of every block: [min lo, max hi) of its intervals (intervals need not be in start order)
    spans = [(int(np.min(lo[b0:b1])), int(np.max(hi[b0:b1]))) for b0, b1 in blocks]
    if not _gaps_sorted(t, spans):
        return None
    E = np.asarray(exposures, dtype=np.float64)
    dev = torch.device("cuda", torch.cuda.current_device())
    up = _UPLOAD_STREAMS.get(dev.index)
    if up is None:  # one per device for the process: the caching allocator pools blocks per stream
        up = _UPLOAD_STREAMS[dev.index] = torch.cuda.Stream(device=dev)
    pinned = src.is_pinned()
    q = queue.Queue(maxsize=2)

    trace = [] if os.environ.get("CRIMP_E2E_TRACE") else None  # (event, block, seconds): tools/e2e_breakdown.py
    t_start = time.perf_counter()

    def uploader():
        try:
            for k, (a, b) in enumerate(spans):
                with torch.cuda.stream(up):
                    d = src[a:b].to(dev, non_blocking=pinned)
                    ev = torch.cuda.Event()
                    ev.record(up)
                if trace is not None:
                    trace.append(("uploaded", k, time.perf_counter() - t_start))
                q.put((d, ev, a))
        except BaseException as e:  # handed to the main thread
            q.put(e)

    th = threading.Thread(target=uploader, daemon=True)
    # this thread holds the GIL between its device calls; a short switch interval lets the uploader start its next
    # copy within ~0.1 ms instead of up to 5 ms (restored below)
    switch = sys.getswitchinterval()
    sys.setswitchinterval(1e-4)
    th.start()
    cur = torch.cuda.current_stream(dev)
    ok = True
    parts = []
    try:
        for b0, b1 in blocks:
            item = q.get()
            if isinstance(item, BaseException):
                raise item
            d, ev, a = item
            cur.wait_event(ev)
            d.record_stream(cur)
            # the block's photons in order on the device (crimp_is_sorted); the joins between blocks and the photons
            # no block uploads were checked on the host (_gaps_sorted)
            ok = ok and ops.is_sorted(d)
            nb = n[b0:b1]
            offs = np.concatenate([[0], np.cumsum(nb)]).astype(np.int64)
            rel_lo = lo[b0:b1] - a
            if np.all(rel_lo[1:] == rel_lo[:-1] + nb[:-1]):   # consecutive intervals: one slice, no copy
                allt = d[int(rel_lo[0]):int(rel_lo[0]) + int(offs[-1])]
            else:
                allt = ops.gather_ranges(d, rel_lo, offs)
            first = t[lo[b0:b1]]
            last = t[lo[b0:b1] + nb - 1]
            mids = ((last - first) / 2) + first                 # measureToAs.py:182
            if trace is not None:
                trace.append(("start", len(parts), time.perf_counter() - t_start))
            parts.append(_fit_block(allt, offs, mids, tm, tmpl, model, E[b0:b1], phShiftRes, nbrBins, varyAmps,
                                    brutemin))
            if trace is not None:
                trace.append(("done", len(parts) - 1, time.perf_counter() - t_start))
    finally:  # on an error here, keep taking the uploader's blocks until it has finished
        while th.is_alive():
            try:
                q.get(timeout=0.05)
            except queue.Empty:
                pass
        th.join()
        sys.setswitchinterval(switch)
    if not ok:
        return None
    out = {k: np.concatenate([np.atleast_1d(np.asarray(p[k])) for p in parts]) for k in parts[0]}
    if trace is not None:
        trace.append(("end", -1, time.perf_counter() - t_start))
        print("e2e trace: " + ", ".join("%s %d %.2f ms" % (e, k, t * 1e3) for e, k, t in sorted(trace, key=lambda r: r[2])),
              flush=True)
    return out


# Photon shares of the pipelined upload's blocks (CRIMP_E2E_WEIGHTS overrides). A block's device work costs ~1.2 ms of
# per-block latency (one round of fits, the H-test launch, the calls) + ~5.5 us per 1e5-photon interval on config 5,
# its upload ~14.6 us per interval at 56 GB/s: the pipeline is balanced near 140 intervals per block, where every
# block's work ends as the next block's upload does. Equal blocks, 8 of them (config 5 per GPU: 156 intervals each):
# 21.2 ms against 26.1 one-shot and 21.1-22.5 for 50/23/15/12 %; 12 equal blocks fall behind (24.9 ms)
# (profiles/r04/e2e_sched.log, e2e_trace_*.log).
_E2E_WEIGHTS = (1.0,) * 8


def _gaps_sorted(t, spans):
    """Host half of the pipelined path's sortedness check: the photons that no block uploads (before the first
    block, between blocks, after the last) are non-decreasing and join the uploaded ranges in order; the device
    checks every uploaded range and the joins between consecutive blocks. Together they cover every photon, as the
    reference's mask over the whole array (measureToAs.py:173) does. Blocks whose ranges overlap or run backwards
    are not pipelined (False)."""
    N = t.size
    edges = [0]
    for a, b in spans:
        if a < edges[-1]:
            return False
        edges += [a, b]
    edges.append(N)
    for g0, g1 in zip(edges[0::2], edges[1::2]):  # gaps [g0, g1), each with one neighbour on either side
        s = t[max(g0 - 1, 0):min(g1 + 1, N)]
        if s.size > 1 and not np.all(s[1:] >= s[:-1]):
            return False
    return True


def _shrinking_blocks(counts, nblocks, weights=None):
    """Consecutive runs of intervals for the pipelined upload: photon shares by ``weights`` (default: nblocks,
    nblocks - 1, ..., 1), non-increasing, so that the last block -- whose device work follows the whole upload -- is
    among the smallest."""
    w = np.asarray(weights, dtype=np.float64) if weights is not None else np.arange(nblocks, 0, -1, dtype=np.float64)
    cuts = np.cumsum(w)[:-1] / w.sum() * float(np.sum(counts))
    at = np.searchsorted(np.cumsum(counts), cuts, side="left") + 1
    edges = np.unique(np.concatenate([[0], np.clip(at, 1, len(counts) - 1), [len(counts)]]))
    return [(int(a), int(b)) for a, b in zip(edges[:-1], edges[1:])]


def _interval_counts(T, starts, ends):
    """Photons of every interval [start, end] (inclusive, measureToAs.py:173-174) without selecting them."""
    T = np.asarray(T, dtype=np.float64)
    if T.size < 2 or np.all(T[1:] >= T[:-1]):
        return np.maximum(np.searchsorted(T, ends, side="right") - np.searchsorted(T, starts, side="left"), 0)
    return np.array([np.count_nonzero((T >= a) & (T <= b)) for a, b in zip(starts, ends)], dtype=np.int64)


def _batches(counts, budget):
    """Consecutive runs of intervals holding at most ``budget`` photons each (at least one interval per run)."""
    out, lo, acc = [], 0, 0
    for i, c in enumerate(counts):
        if i > lo and acc + c > budget:
            out.append((lo, i))
            lo, acc = i, 0
        acc += int(c)
    if lo < len(counts):
        out.append((lo, len(counts)))
    return out


def measureToAs(evtFile, timMod, tempModPP, toagtifile, eneLow=0.5, eneHigh=10., toaStart=0, toaEnd=None,
                phShiftRes=1000, nbrBins=15, varyAmps=False, readvaryparam=False, brutemin=False, plotPPs=False,
                plotLLs=False, toaFile='ToAs', timFile=None):
    """ToAs of every interval of ``toagtifile`` (measureToAs.py:64-251).

    The reference writes each ToA's row as soon as it is measured (:160-162, :222-226). Here the intervals are
    fitted in batches of at most CRIMP_TOA_BATCH_PHOTONS photons (default 2^27) and each batch's rows are written
    and flushed when the batch finishes. An interval without photons ends the reference's loop with an IndexError
    at :182 after the rows before it were written; the same happens here: the intervals before it are measured and
    written, then the IndexError is raised."""
    import os
    import pandas as pd
    logger.info("\n Running measureToAs with input parameters: evtFile: %s timMod: %s tempModPP: %s toagtifile: %s"
                " eneLow: %s eneHigh: %s toaStart: %s toaEnd: %s phShiftRes: %s brutemin: %s toaFile: %s",
                evtFile, timMod, tempModPP, toagtifile, eneLow, eneHigh, toaStart, toaEnd, phShiftRes, brutemin,
                toaFile)
    ef = EvtFileOps(evtFile).build_time_energy_df().filtenergy(eneLow=eneLow, eneHigh=eneHigh)
    TIMEMJD = ef.time_energy_df["TIME"].to_numpy()
    iv = pd.read_csv(toagtifile, sep=r'\s+', comment='#')
    st, en = iv['ToA_tstart'].to_numpy(), iv['ToA_tend'].to_numpy()
    lenInt, expo = iv['ToA_lenInt'].to_numpy(), iv['ToA_exposure'].to_numpy()
    events, rate = iv['Events'].to_numpy(), iv['ct_rate'].to_numpy()
    toaEnd = np.size(en) if toaEnd is None else toaEnd + 1  # :147-150 (inclusive end)
    rng = np.arange(toaStart, toaEnd)
    tmpl = readPPtemplate(tempModPP)
    tm = timMod if isinstance(timMod, dict) else ReadTimingModel(str(timMod)).readfulltimingmodel()[0]
    logger.info('\n Using best fit model of template {} to measure ToAs'.format(tmpl["model"]))
    counts = _interval_counts(TIMEMJD, st[rng], en[rng])
    empty = np.nonzero(counts <= 0)[0]
    nfit = int(empty[0]) if empty.size else rng.size      # the reference's loop ends at the first empty interval
    T = _device_times(TIMEMJD) if nfit else None
    T = TIMEMJD if T is None else T
    budget = int(os.environ.get("CRIMP_TOA_BATCH_PHOTONS", 1 << 27))
    allres = []
    with open(toaFile + '.txt', "w+") as f:
        f.write(HEADER)
        f.flush()
        for b0, b1 in _batches(counts[:nfit], budget):
            sel = rng[b0:b1]
            for ii in sel:
                print('ToA {}'.format(ii))
            res = measure_intervals(T, tm, tmpl, st[sel], en[sel], expo[sel], phShiftRes, nbrBins, varyAmps,
                                    brutemin, readvaryparam)
            warn_capped(res, phShiftRes, ['ToA' + str(ii) for ii in sel], logger)
            for k, ii in enumerate(sel):
                f.write(str(ii) + '\t' + str(res["ToA_mid"][k]) + '\t' + str(st[ii]) + '\t' + str(en[ii]) + '\t' +
                        str(lenInt[ii]) + '\t' + str(expo[ii]) + '\t' + str(events[ii]) + '\t' + str(rate[ii]) + '\t' +
                        str(res["phShi"][k]) + '\t' + str(res["phShi_LL"][k]) + '\t' + str(res["phShi_UL"][k]) + '\t' +
                        str(res["htestPow"][k]) + '\t' + str(res["reducedChi2"][k]) + '\n')
            f.flush()
            allres.append(res)
        if nfit < rng.size:
            print('ToA {}'.format(rng[nfit]))
            raise IndexError("index -1 is out of bounds for axis 0 with size 0 (ToA {} holds no photons, "
                             "measureToAs.py:182)".format(rng[nfit]))
    logger.info('\n Wrote ToA properties to {}.txt'.format(toaFile))
    if timFile is not None:  # measureToAs.py:238-240
        phshiftTotimfile(toaFile + '.txt', timMod, timFile, tempModPP=tempModPP)
        logger.info('\n Wrote timfile {}.tim'.format(timFile))
    if allres:
        _plot_residuals({k: np.concatenate([r[k] for r in allres]) for k in ("ToA_mid", "phShi", "phShi_LL", "phShi_UL")},
                        toaFile)
    return pd.read_csv(toaFile + '.txt', sep=r'\s+', comment='#')


def _plot_residuals(res, outFile):
    try:
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
    except Exception:  # pragma: no cover - plotting is optional
        return
    fig, ax = plt.subplots(1, figsize=(7, 5))
    ax.errorbar(res["ToA_mid"], res["phShi"] / (2 * math.pi),
                yerr=(res["phShi_LL"] / (2 * math.pi), res["phShi_UL"] / (2 * math.pi)), fmt='ok')
    ax.set_xlabel('Time (MJD)')
    ax.set_ylabel(r'$\Delta\phi$ (cycles)')
    fig.tight_layout()
    fig.savefig(str(outFile) + '_phaseResiduals.pdf', format='pdf')
    plt.close(fig)


def main(argv=None):
    p = argparse.ArgumentParser(description="Script to measure ToAs from event file")
    p.add_argument("evtFile", help="Name of a barycentered event file", type=str)
    p.add_argument("timMod", help="Timing model, Tempo2 .par file should work", type=str)
    p.add_argument("tempModPP", help="Parameters of template pulse profile", type=str)
    p.add_argument("toagtifile", help=".txt file with ToA interval information", type=str)
    p.add_argument("-el", "--enelow", type=float, default=0.5)
    p.add_argument("-eh", "--enehigh", type=float, default=10)
    p.add_argument("-ts", "--toaStart", type=int, default=0)
    p.add_argument("-te", "--toaEnd", type=int, default=None)
    p.add_argument("-pr", "--phShiftRes", type=int, default=1000)
    p.add_argument("-nb", "--nbrBins", type=int, default=15)
    p.add_argument("-va", "--varyAmps", default=False, action=argparse.BooleanOptionalAction)
    p.add_argument("-rv", "--readvaryparam", default=False, action=argparse.BooleanOptionalAction)
    p.add_argument("-bm", "--brutemin", default=False, action=argparse.BooleanOptionalAction)
    p.add_argument("-pp", "--plotPPs", default=False, action=argparse.BooleanOptionalAction)
    p.add_argument("-ll", "--plotLLs", default=False, action=argparse.BooleanOptionalAction)
    p.add_argument("-tf", "--toaFile", type=str, default='ToAs')
    p.add_argument("-mf", "--timFile", type=str, default=None)
    p.add_argument("-v", "--verbose", action="count", default=0)
    a = p.parse_args(argv)
    configure_logging(console_level=("WARNING", "INFO", "DEBUG")[min(a.verbose, 2)],
                      file_path=f"{a.toaFile}.log", file_level="INFO", force=True)
    measureToAs(a.evtFile, a.timMod, a.tempModPP, a.toagtifile, a.enelow, a.enehigh, a.toaStart, a.toaEnd,
                a.phShiftRes, a.nbrBins, a.varyAmps, a.readvaryparam, a.brutemin, a.plotPPs, a.plotLLs, a.toaFile,
                a.timFile)


if __name__ == '__main__':
    sys.exit(main())

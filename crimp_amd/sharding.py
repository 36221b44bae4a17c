"""Multi-GPU layer: one process per GPU, the trial grid (or the ToA intervals) sharded across
ranks, one collective per search.

* ``shard_range``      contiguous slice of a flat index range for one rank;
* ``sharded_search``   each rank computes its slice of the fd-outer trial grid through
                       ``crimp_search`` (first/count), then either one ``all_gather`` of the
                       per-trial powers (``gather='all'``, every rank gets the full array) or one
                       ``all_gather`` of each rank's best (power, index) (``gather='best'``);
                       ties resolve to the lowest flat index, as ``np.argmax`` does;
* ``sharded_toa_fit``  each rank fits a contiguous block of intervals, loading only their photons
                       (``interval_shard``: blocks cut at quantiles of the intervals' photon counts, a fit's cost
                       being photon-proportional, plus a fixed per-interval share); one ``all_gather`` of the
                       per-interval result records.
The search's photon arrays are replicated (every rank holds all photons; 8 B/photon). The collectives go
through ``torch.distributed`` (backend ``nccl`` = RCCL over xGMI on the GPU box; ``gloo`` in the
CPU tests). ``compute`` hooks let the CPU tests drive the same collective logic without a GPU.
"""
import numpy as np


def shard_range(total, world, rank):
    """[first, first+count) of ``total`` items for ``rank`` (sizes differ by at most one)."""
    base, extra = divmod(int(total), int(world))
    first = rank * base + min(rank, extra)
    return first, base + (1 if rank < extra else 0)


def _dist():
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return dist, dist.get_world_size(), dist.get_rank()
    return None, 1, 0


def _device_for_backend(dist):
    import torch
    if dist is not None and dist.get_backend() == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def _gpu_slice(time, t0, freq, nharm, stat, freq_dot, first, count, flags=0, precision=None, best=False):
    from . import ops
    import torch
    if isinstance(time, torch.Tensor) and freq_dot is not None and not isinstance(freq_dot, torch.Tensor):
        freq_dot = torch.as_tensor(np.asarray(freq_dot, dtype=np.float64), device=time.device)
    fn = ops.search_best if best else ops.search
    return fn(time, t0, freq, nharm, stat, log10_negfdot=freq_dot, first=first, count=count, flags=flags,
              precision=precision)


def _as_comm(local, dev):
    """The rank's result as a float64 tensor on the collective's device, without a host round trip when it is
    already a device tensor and the backend is nccl."""
    import torch
    if isinstance(local, torch.Tensor):
        return local.to(device=dev, dtype=torch.float64)
    return torch.as_tensor(np.asarray(local), dtype=torch.float64, device=dev)


def sharded_search(time, freq, nharm=2, stat=0, freq_dot=None, gather="all", compute=None, flags=0, precision=None,
                   t0=None):
    """Z^2 (stat=0) / H (stat=1) over the fd-outer grid, sharded across the process group.

    Returns the full power array (gather='all'; a tensor on the rank's device when ``time`` is a device
    tensor, else a numpy array) or ``(best_power, best_flat_index)`` (gather='best'), identical on every rank.
    With the nccl backend the gather runs on the device buffers the search wrote (no host staging).
    ``flags`` and ``precision`` (None | "exact" | "nufft" | "f64", as PeriodSearch) go to the rank's crimp_search
    call (e.g. FLAG_TIME_KERNELS for bench.py). ``t0`` (optional): the reference time (time[0] + time[-1]) / 2 when
    the caller already holds it, which spares a device read for a device tensor.
    """
    import functools
    import torch
    dist, world, rank = _dist()
    custom = compute is not None
    compute = compute or functools.partial(_gpu_slice, flags=flags, precision=precision)
    as_tensor = isinstance(time, torch.Tensor)
    if as_tensor:
        if t0 is None:
            t0 = float((time[0] + time[-1]).item()) / 2
        nf = int(freq.numel())
    else:
        if t0 is None:
            t0 = (time[0] + time[-1]) / 2  # periodsearch.py:54, shared by every shard
        nf = int(np.size(freq))
    nfd = 0 if freq_dot is None else int(freq_dot.numel() if isinstance(freq_dot, torch.Tensor) else np.size(freq_dot))
    total = (nfd if nfd else 1) * nf
    first, count = shard_range(total, world, rank)
    rank_best = None
    if gather == "best" and count and not custom and as_tensor and time.is_cuda:
        # the rank's search and its best trial in one call (crimp_search_best: a NUFFT search reads the best back
        # with its fix-up count)
        local, bv_, bi_ = _gpu_slice(time, t0, freq, nharm, stat, freq_dot, first, count, flags=flags,
                                     precision=precision, best=True)
        rank_best = (bv_, bi_)
    else:
        local = compute(time, t0, freq, nharm, stat, freq_dot, first, count)
    if rank_best is not None and dist is None:  # one process: the call's own best is the answer
        return rank_best[0], rank_best[1] + first
    dev = _device_for_backend(dist) if dist is not None else (
        local.device if isinstance(local, torch.Tensor) else torch.device("cpu"))
    loc = _as_comm(local, dev)
    if gather == "best":
        if count:
            if rank_best is not None or (isinstance(local, torch.Tensor) and local.is_cuda):
                # the rank's best on the device (crimp_search_best, or crimp_best: one reduction, one 16-byte
                # readback)
                from . import ops
                bv, bi = rank_best if rank_best is not None else ops.best(local)
                if dist is None:
                    return bv, bi + first
                mine = torch.tensor([bv, float(bi + first)], dtype=torch.float64, device=dev)
            else:
                v, i = torch.max(loc, 0)  # the first maximal index, as np.argmax
                if dist is None:
                    res = torch.stack([v, i.to(torch.float64)]).cpu().numpy()
                    return float(res[0]), int(res[1]) + first
                mine = torch.stack([v, (i + first).to(torch.float64)])
        else:
            mine = torch.tensor([-np.inf, float(total)], dtype=torch.float64, device=dev)
        if dist is None:
            allb = mine.reshape(1, 2)
        else:
            allb = torch.empty(world * 2, dtype=torch.float64, device=dev)
            dist.all_gather_into_tensor(allb, mine)
            allb = allb.reshape(world, 2)
        # highest power, ties to the lowest flat index (np.argmax over the whole grid)
        top = allb[:, 0].max()
        idx = torch.where(allb[:, 0] == top, allb[:, 1], torch.full_like(allb[:, 1], np.inf)).min()
        res = torch.stack([top, idx]).cpu().numpy()
        return float(res[0]), int(res[1])
    if dist is None:
        return loc if as_tensor else loc.cpu().numpy()
    width = shard_range(total, world, 0)[1]
    buf = torch.full((width,), np.nan, dtype=torch.float64, device=dev)
    buf[:count] = loc
    allp = torch.empty(world * width, dtype=torch.float64, device=dev)
    dist.all_gather_into_tensor(allp, buf)
    allp = allp.reshape(world, width)
    out = torch.cat([allp[r, :shard_range(total, world, r)[1]] for r in range(world)])
    if as_tensor:
        return out.to(time.device)
    return out.cpu().numpy()


# A fit's cost per interval in photon units beyond its photons: the workgroup's fixed passes and reductions (config 5:
# ~1e5 photons per interval, so balance is by photons; a block of tiny intervals still costs per interval)
INTERVAL_OVERHEAD_PHOTONS = 4096


def interval_blocks(offsets, world, overhead=INTERVAL_OVERHEAD_PHOTONS):
    """Block boundaries b_0 = 0 <= b_1 <= ... <= b_world = nint: rank r fits intervals [b_r, b_{r+1}). Each boundary
    is the interval edge nearest to r/world of the total cost (photons + ``overhead`` per interval), so ranks hold
    equal photon loads however ragged the intervals are (within one interval of the even share); N x k equal intervals
    give every rank k."""
    off = np.asarray(offsets, dtype=np.int64)
    nint = off.size - 1
    cum = np.concatenate([[0.0], np.cumsum(np.diff(off).astype(np.float64) + float(overhead))])
    b = [0]
    for r in range(1, world):
        target = cum[-1] * r / world
        i = int(np.searchsorted(cum, target, side="left"))
        i = min(max(i, 1), nint)
        if abs(cum[i - 1] - target) <= abs(cum[i] - target):
            i -= 1
        b.append(max(b[-1], i))
    b.append(nint)
    return b


def interval_shard(offsets, world, rank):
    """(first interval, interval count, first photon, photon end) of ``rank``'s contiguous block of intervals
    (``interval_blocks``): the photon range [a, b) is all that rank has to load."""
    off = np.asarray(offsets, dtype=np.int64)
    b = interval_blocks(off, world)
    first, count = b[rank], b[rank + 1] - b[rank]
    return first, count, int(off[first]), int(off[first + count])


def sharded_toa_fit(x, offsets, exposure, tmpl, brutemin=False, ph_shift_res=1000, nbr_bins=15, fitter=None):
    """Fit interval blocks per rank; one all_gather of (phShi, LL, UL, redChi2, norm, LLmax).

    ``offsets`` (nint + 1, global) and ``exposure`` (nint) describe every interval. ``x`` supplies the photons:
    the whole concatenated array (host or device; the rank slices out its own range and uploads only that), or a
    callable ``x(a, b)`` returning photons [a, b) -- e.g. a slice of a memory-mapped file -- so that a rank never
    holds more than its own intervals' photons (``interval_shard`` gives the range)."""
    import torch
    from .toafit import ToAFitter
    dist, world, rank = _dist()
    off = np.asarray(offsets.cpu() if isinstance(offsets, torch.Tensor) else offsets, dtype=np.int64)
    nint = off.size - 1
    first, count, pa, pb = interval_shard(off, world, rank)
    keys = ("phShi", "phShi_LL", "phShi_UL", "reducedChi2", "norm", "LLmax")
    blocks = interval_blocks(off, world)
    width = max(1, max(blocks[r + 1] - blocks[r] for r in range(world)))
    rec = np.full((width, len(keys)), np.nan)
    if count:
        sl = off[first:first + count + 1]
        if callable(x):
            xs = x(pa, pb)
        elif isinstance(x, torch.Tensor):
            xs = x[pa:pb]
        else:
            xs = np.asarray(x)[pa:pb]
        fit = (fitter or ToAFitter)(xs, sl - sl[0], np.asarray(exposure)[first:first + count], tmpl, ph_shift_res,
                                    nbr_bins)
        r = fit.fit(brutemin=brutemin)
        rec[:count] = np.stack([r[k] for k in keys], axis=1)
    if dist is None:
        out = rec[:count]
    else:
        dev = _device_for_backend(dist)
        t = torch.as_tensor(rec.ravel(), device=dev)
        allr = torch.empty(world * rec.size, dtype=torch.float64, device=dev)
        dist.all_gather_into_tensor(allr, t)
        allr = allr.cpu().numpy().reshape((world,) + rec.shape)
        out = np.concatenate([allr[r, :blocks[r + 1] - blocks[r]] for r in range(world)])
    return {k: out[:, i] for i, k in enumerate(keys)}

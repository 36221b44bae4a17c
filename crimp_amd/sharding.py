"""Multi-GPU layer: one process per GPU, the trial grid (or the ToA intervals) sharded across
ranks, one collective per search.

* ``shard_range``      contiguous slice of a flat index range for one rank;
* ``sharded_search``   each rank computes its slice of the fd-outer trial grid through
                       ``crimp_search`` (first/count), then either one ``all_gather`` of the
                       per-trial powers (``gather='all'``, every rank gets the full array) or one
                       ``all_gather`` of each rank's best (power, index) (``gather='best'``);
                       ties resolve to the lowest flat index, as ``np.argmax`` does;
* ``sharded_toa_fit``  each rank fits a contiguous block of intervals; one ``all_gather`` of the
                       per-interval result records.
Photon arrays are replicated (every rank holds all photons; 8 B/photon). The collectives go
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


def _gpu_slice(time, t0, freq, nharm, stat, freq_dot, first, count):
    from . import ops
    return ops.search(time, t0, freq, nharm, stat, log10_negfdot=freq_dot, first=first, count=count)


def sharded_search(time, freq, nharm=2, stat=0, freq_dot=None, gather="all", compute=None):
    """Z^2 (stat=0) / H (stat=1) over the fd-outer grid, sharded across the process group.

    Returns the full power array (gather='all') or ``(best_power, best_flat_index)``
    (gather='best'), identical on every rank.
    """
    import torch
    dist, world, rank = _dist()
    compute = compute or _gpu_slice
    if hasattr(time, "numel"):
        t0 = float((time[0] + time[-1]).item()) / 2
        nf = int(freq.numel())
    else:
        t0 = (time[0] + time[-1]) / 2  # periodsearch.py:54, shared by every shard
        nf = int(np.size(freq))
    nfd = 0 if freq_dot is None else int(np.size(freq_dot))
    total = (nfd if nfd else 1) * nf
    first, count = shard_range(total, world, rank)
    local = compute(time, t0, freq, nharm, stat, freq_dot, first, count)
    dev = _device_for_backend(dist)
    loc = torch.as_tensor(np.asarray(local.cpu() if hasattr(local, "cpu") else local), dtype=torch.float64).to(dev)
    if gather == "best":
        if count:
            i = int(torch.argmax(loc).item())
            mine = torch.tensor([loc[i].item(), float(first + i)], dtype=torch.float64, device=dev)
        else:
            mine = torch.tensor([-np.inf, float(total)], dtype=torch.float64, device=dev)
        if dist is None:
            allb = mine.reshape(1, 2)
        else:
            allb = torch.empty(world * 2, dtype=torch.float64, device=dev)
            dist.all_gather_into_tensor(allb, mine)
        b = allb.cpu().numpy().reshape(-1, 2)
        k = np.lexsort((b[:, 1], -b[:, 0]))[0]
        return float(b[k, 0]), int(b[k, 1])
    if dist is None:
        return loc.cpu().numpy()
    width = shard_range(total, world, 0)[1]
    buf = torch.full((width,), np.nan, dtype=torch.float64, device=dev)
    buf[:count] = loc
    allp = torch.empty(world * width, dtype=torch.float64, device=dev)
    dist.all_gather_into_tensor(allp, buf)
    allp = allp.cpu().numpy().reshape(world, width)
    return np.concatenate([allp[r, :shard_range(total, world, r)[1]] for r in range(world)])


def sharded_toa_fit(x, offsets, exposure, tmpl, brutemin=False, ph_shift_res=1000, nbr_bins=15, fitter=None):
    """Fit interval blocks per rank; one all_gather of (phShi, LL, UL, redChi2, norm, LLmax)."""
    import torch
    from .toafit import ToAFitter
    dist, world, rank = _dist()
    off = np.asarray(offsets, dtype=np.int64)
    nint = off.size - 1
    first, count = shard_range(nint, world, rank)
    keys = ("phShi", "phShi_LL", "phShi_UL", "reducedChi2", "norm", "LLmax")
    rec = np.full((shard_range(nint, world, 0)[1], len(keys)), np.nan)
    if count:
        sl = off[first:first + count + 1]
        xs = np.asarray(x)[sl[0]:sl[-1]]
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
        out = np.concatenate([allr[r, :shard_range(nint, world, r)[1]] for r in range(world)])
    return {k: out[:, i] for i, k in enumerate(keys)}

"""World-size-2 gloo run of the sharding layer on CPU: the sharded search and ToA fits must equal
the unsharded results (same powers, same best index). The per-rank compute is the oracle here
(the GPU ranks call crimp_search through the same code path)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _oracle_slice(time, t0, freq, nharm, stat, freq_dot, first, count):
    from oracle import oracle as O
    full = O.search(np.asarray(time), np.asarray(freq), nharm, freq_dot=freq_dot, stat="z2" if stat == 0 else "h")
    return full[first:first + count]


class _OracleFitter:
    def __init__(self, x, offsets, exposure, tmpl, res, nb):
        self.x, self.off, self.E, self.tmpl, self.res, self.nb = x, offsets, exposure, tmpl, res, nb

    def fit(self, brutemin=False):
        from oracle import oracle as O
        rows = [O.fit_toa(self.x[self.off[i]:self.off[i + 1]], self.E[i], self.tmpl, self.res, self.nb, brutemin)
                for i in range(len(self.off) - 1)]
        return {k: np.array([r[k] for r in rows]) for k in rows[0]}


def _worker(rank, world, port, out_path):
    import sys
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from crimp_amd.sharding import sharded_search, sharded_toa_fit
    from crimp_amd.synth import pulsed_events, template_intervals
    t = pulsed_events(4000, 2.0e4, 1.7, pulsed_frac=0.3, seed=5)
    f = 1.7 + np.arange(-51, 50) / 2.0e5
    fd = np.array([-12.0, -9.0, -8.5])
    full = sharded_search(t, f, 2, 0, freq_dot=fd, gather="all", compute=_oracle_slice)
    best = sharded_search(t, f, 3, 1, freq_dot=fd, gather="best", compute=_oracle_slice)
    import torch  # the same through tensors (bench.py's config-4 leg passes device tensors, freq_dot included)
    best_t = sharded_search(torch.as_tensor(t), torch.as_tensor(f), 3, 1, freq_dot=torch.as_tensor(fd), gather="best",
                            compute=_oracle_slice)
    assert best_t == best
    amps, phs = [2.0, 1.0], [0.3, -1.0]
    x, off, E, _ = template_intervals(5, 1500, 10.0, amps, phs, seed=3)
    tmpl = {"model": "fourier", "norm": {"value": 10.0}, "amp_1": {"value": 2.0}, "ph_1": {"value": 0.3},
            "amp_2": {"value": 1.0}, "ph_2": {"value": -1.0}}
    toa = sharded_toa_fit(x, off, E, tmpl, brutemin=True, fitter=_OracleFitter)
    # per-rank photon loading: the rank asks only for its own intervals' photon range
    asked = []

    def load(a, b):
        asked.append((a, b))
        return x[a:b].copy()
    toa2 = sharded_toa_fit(load, off, E, tmpl, brutemin=True, fitter=_OracleFitter)
    from crimp_amd.sharding import interval_shard
    _, _, pa, pb = interval_shard(off, world, rank)
    assert asked == [(pa, pb)] and pb - pa < x.size
    assert np.array_equal(toa2["phShi"], toa["phShi"])
    # ragged intervals (rows 35-41 of the worked example are 5,136-10,000 photons): blocks balanced by photons
    xr, offr, Er = _ragged_intervals()
    toar = sharded_toa_fit(xr, offr, Er, tmpl, brutemin=True, fitter=_OracleFitter)
    if rank == 0:
        np.savez(out_path, full=full, best=np.array(best), phShi=toa["phShi"], LL=toa["phShi_LL"],
                 rphShi=toar["phShi"], rLL=toar["phShi_LL"], rUL=toar["phShi_UL"])
    dist.barrier()
    dist.destroy_process_group()


def _ragged_intervals():
    """Seven intervals of 300..4000 photons (ragged as the worked example's rows 35-41) drawn from one template."""
    from crimp_amd.synth import template_intervals
    sizes = [4000, 300, 2500, 900, 3500, 600, 1800]
    xs, Es = [], []
    for i, n in enumerate(sizes):
        x, _, E, _ = template_intervals(1, n, 10.0, [2.0, 1.0], [0.3, -1.0], seed=20 + i)
        xs.append(np.asarray(x))
        Es.append(float(np.asarray(E)[0]))
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    return np.concatenate(xs), off, np.array(Es)


def test_interval_blocks_balance_photons():
    from crimp_amd.sharding import interval_blocks, interval_shard, shard_range
    rng = np.random.default_rng(0)
    for world in (1, 2, 3, 8):
        for sizes in (np.full(16, 1000), rng.integers(1000, 100000, 37), np.r_[np.full(20, 100), [10 ** 6]]):
            off = np.concatenate([[0], np.cumsum(sizes)])
            b = interval_blocks(off, world)
            assert b[0] == 0 and b[-1] == sizes.size and all(b[r] <= b[r + 1] for r in range(world))
            cost = np.array([np.sum(sizes[b[r]:b[r + 1]] + 4096.0) for r in range(world)])
            biggest = np.max(sizes + 4096.0)
            assert cost.max() - cost.sum() / world <= biggest  # within one interval of the even share
            for r in range(world):
                first, count, pa, pb = interval_shard(off, world, r)
                assert (first, count) == (b[r], b[r + 1] - b[r]) and (pa, pb) == (off[b[r]], off[b[r + 1]])
    off = np.arange(0, 8 * 1250 + 1) * 100  # config 5 on 8 ranks: 1250 equal intervals each, as before
    assert [interval_shard(off, 8, r)[:2] for r in range(8)] == [shard_range(8 * 1250, 8, r) for r in range(8)]


def test_two_rank_sharded_search_and_toas(tmp_path):
    from oracle import oracle as O
    from crimp_amd.synth import pulsed_events, template_intervals
    out = str(tmp_path / "r.npz")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    r = np.load(out)
    t = pulsed_events(4000, 2.0e4, 1.7, pulsed_frac=0.3, seed=5)
    f = 1.7 + np.arange(-51, 50) / 2.0e5
    fd = np.array([-12.0, -9.0, -8.5])
    ref = O.search(t, f, 2, freq_dot=fd)
    np.testing.assert_array_equal(r["full"], ref)
    h = O.search(t, f, 3, freq_dot=fd, stat="h")
    assert int(r["best"][1]) == int(np.argmax(h)) and r["best"][0] == h.max()
    x, off, E, _ = template_intervals(5, 1500, 10.0, [2.0, 1.0], [0.3, -1.0], seed=3)
    tmpl = {"model": "fourier", "norm": {"value": 10.0}, "amp_1": {"value": 2.0}, "ph_1": {"value": 0.3},
            "amp_2": {"value": 1.0}, "ph_2": {"value": -1.0}}
    for i in range(5):
        o = O.fit_toa(x[off[i]:off[i + 1]], E[i], tmpl, brutemin=True)
        assert r["phShi"][i] == o["phShi"] and r["LL"][i] == o["phShi_LL"]
    xr, offr, Er = _ragged_intervals()
    for i in range(offr.size - 1):
        o = O.fit_toa(xr[offr[i]:offr[i + 1]], Er[i], tmpl, brutemin=True)
        assert r["rphShi"][i] == o["phShi"] and r["rLL"][i] == o["phShi_LL"] and r["rUL"][i] == o["phShi_UL"]


def test_shard_range_partitions():
    from crimp_amd.sharding import shard_range
    for total in (0, 1, 7, 1000, 1001):
        for world in (1, 2, 3, 8):
            parts = [shard_range(total, world, r) for r in range(world)]
            assert sum(c for _, c in parts) == total
            assert all(parts[r][0] + parts[r][1] == parts[r + 1][0] for r in range(world - 1))

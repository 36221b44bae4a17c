"""The multi-GPU code path on one GPU: two gloo ranks on cuda:0 run sharding.py's default compute
(_gpu_slice -> crimp_search on device tensors) and the real ToAFitter, and must give bit-identical results to
the unsharded device search and fits computed in the same processes (the exact search is partition invariant;
each ToA interval's fit is independent of the others in its batch). The NUFFT (the default, bench.py's value path)
is sharded the same way: a rank slice of whole rows is bit-identical to the unsharded grid; a 3-row grid whose
rank split cuts the middle row mid-way (each rank plans its own segment of it) agrees within the plans' error --
every power within 1e-6 relative, the median within 1e-12 -- and gives the same best trial. The nccl branch is the
same code with the collective's buffers on the device; the 8-GPU scaling curve itself is run by the driver, not
here."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _ragged(tm, dev):
    """Intervals of 3,000..25,000 photons from the worked example's template (rows 35-41 range 5,136-10,000)."""
    import torch
    from crimp_amd.synth import template_intervals_torch
    K = sum(1 for k in tm if k.startswith("amp_"))
    amps = [tm["amp_%d" % j]["value"] for j in range(1, K + 1)]
    phs = [tm["ph_%d" % j]["value"] for j in range(1, K + 1)]
    sizes = [25_000, 3_000, 12_000, 6_000, 18_000, 4_000, 9_000]
    xs, Es = [], []
    for i, n in enumerate(sizes):
        x, _, E, _ = template_intervals_torch(1, n, tm["norm"]["value"], amps, phs, seed=30 + i, device=dev)
        xs.append(x)
        Es.append(float(np.asarray(E)[0]))
    off = torch.as_tensor(np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64), device=dev)
    return torch.cat(xs), off, np.array(Es)


def _worker(rank, world, port, out_path):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from crimp_amd import ops
    from crimp_amd.readPPtemplate import readPPtemplate
    from crimp_amd.sharding import sharded_search, sharded_toa_fit
    from crimp_amd.synth import pulsed_events, template_intervals_torch
    from crimp_amd.toafit import ToAFitter
    dev = torch.device("cuda", 0)
    t_h = pulsed_events(200_000, 2.0e5, 7.123456789, pulsed_frac=0.05, seed=11)
    f_h = 7.123456789 + (np.arange(40_000) - 20_000) / 2.0e6
    fd = np.array([-12.0, -10.5])
    t = torch.as_tensor(t_h, device=dev)
    f = torch.as_tensor(f_h, device=dev)
    full = sharded_search(t, f, 2, 0, freq_dot=fd, gather="all", precision="exact")
    best = sharded_search(t, f, 3, 1, freq_dot=fd, gather="best", precision="exact")
    t0 = float((t[0] + t[-1]).item()) / 2
    fdd = torch.as_tensor(fd, device=dev)
    ref = ops.search(t, t0, f, 2, 0, log10_negfdot=fdd, precision="exact")
    refh = ops.search(t, t0, f, 3, 1, log10_negfdot=fdd, precision="exact").cpu().numpy()
    nu = _nufft_cases(t, f, t0, dev)
    tm = readPPtemplate(os.path.join(ROOT, "tests", "golden", "1e2259_template.txt"))
    K = sum(1 for k in tm if k.startswith("amp_"))
    x, off, E, _ = template_intervals_torch(9, 20_000, tm["norm"]["value"], [tm["amp_%d" % j]["value"] for j in
                                            range(1, K + 1)], [tm["ph_%d" % j]["value"] for j in range(1, K + 1)],
                                            seed=3, device=dev)
    toa = sharded_toa_fit(x, off, E, tm, brutemin=True)
    rtoa = ToAFitter(x, off, E, tm).fit(brutemin=True)
    xr, offr, Er = _ragged(tm, dev)   # ragged intervals: photon-balanced blocks
    tr = sharded_toa_fit(xr, offr, Er, tm, brutemin=True)
    rtr = ToAFitter(xr, offr, Er, tm).fit(brutemin=True)
    if rank == 0:
        keys = sorted(toa)
        np.savez(out_path, full=full.cpu().numpy(), full_is_dev=np.array(full.is_cuda), ref=ref.cpu().numpy(),
                 best=np.array(best, dtype=np.float64), refh=refh, keys=np.array(keys),
                 toa=np.stack([toa[k] for k in keys]), rtoa=np.stack([rtoa[k] for k in keys]),
                 tr=np.stack([tr[k] for k in keys]), rtr=np.stack([rtr[k] for k in keys]), **nu)
    dist.barrier()
    dist.destroy_process_group()


def _nufft_cases(t, f, t0, dev):
    """The NUFFT through the collective, as bench.py's value path runs it (sharded_search with the default precision
    and with precision="nufft"): a 2-row grid (the two ranks' slices are whole rows), a 3-row grid (the split cuts
    the middle row at trial 20,000 of 40,000) for Z^2_2 (gather='all') and H_3 (gather='best'), with the unsharded
    searches beside them and the kernel family each rank's slice took."""
    import torch
    from crimp_amd import ops, _native as N
    from crimp_amd.sharding import sharded_search
    fd2, fd3 = np.array([-12.0, -10.5]), np.array([-12.0, -11.0, -10.5])
    out = {}
    for tag, fd in (("r2", fd2), ("r3", fd3)):
        fdd = torch.as_tensor(fd, device=dev)
        for prec in (None, "nufft"):
            p = prec or "default"
            out["nu_%s_%s_all" % (tag, p)] = sharded_search(t, f, 2, 0, freq_dot=fd, gather="all",
                                                            precision=prec).cpu().numpy()
            out["nu_%s_%s_path" % (tag, p)] = np.array(N.load().crimp_last_search_path())
            out["nu_%s_%s_best" % (tag, p)] = np.array(sharded_search(t, f, 3, 1, freq_dot=fd, gather="best",
                                                                      precision=prec), dtype=np.float64)
        out["nu_%s_ref" % tag] = ops.search(t, t0, f, 2, 0, log10_negfdot=fdd).cpu().numpy()
        out["nu_%s_refh" % tag] = ops.search(t, t0, f, 3, 1, log10_negfdot=fdd).cpu().numpy()
    return out


def _check_nufft(r, world):
    for tag in ("r2", "r3"):
        ref, refh = r["nu_%s_ref" % tag], r["nu_%s_refh" % tag]
        for p in ("default", "nufft"):
            got = r["nu_%s_%s_all" % (tag, p)]
            assert int(r["nu_%s_%s_path" % (tag, p)]) == 2
            b = r["nu_%s_%s_best" % (tag, p)]
            assert int(b[1]) == int(np.argmax(refh))
            if tag == "r2" or world == 1:  # whole rows per rank: bit-identical
                np.testing.assert_array_equal(got, ref)
                assert b[0] == refh.max()
            else:                           # the middle row cut mid-way: each rank plans its own segment
                rel = np.abs(got - ref) / np.abs(ref)
                assert rel.max() <= 1e-6 and np.median(rel) <= 1e-12, (rel.max(), np.median(rel))
                assert not np.array_equal(got, ref)      # the cut row really was planned per segment
                assert abs(b[0] - refh.max()) <= 1e-12 * refh.max()


def test_two_gloo_ranks_on_gpu_bit_identical_to_unsharded(tmp_path):
    out = str(tmp_path / "r.npz")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    r = np.load(out)
    assert bool(r["full_is_dev"])
    np.testing.assert_array_equal(r["full"], r["ref"])
    assert r["best"][0] == r["refh"].max() and int(r["best"][1]) == int(np.argmax(r["refh"]))
    np.testing.assert_array_equal(r["toa"], r["rtoa"])
    np.testing.assert_array_equal(r["tr"], r["rtr"])
    _check_nufft(r, 2)


def _nccl_worker(rank, world, port, out_path):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    from crimp_amd import ops
    from crimp_amd.readPPtemplate import readPPtemplate
    from crimp_amd.sharding import sharded_search, sharded_toa_fit
    from crimp_amd.synth import pulsed_events, template_intervals_torch
    from crimp_amd.toafit import ToAFitter
    t_h = pulsed_events(200_000, 2.0e5, 7.123456789, pulsed_frac=0.05, seed=11)
    f = torch.as_tensor(7.123456789 + (np.arange(40_000) - 20_000) / 2.0e6, device=dev)
    fd = np.array([-12.0, -10.5])
    t = torch.as_tensor(t_h, device=dev)
    full = sharded_search(t, f, 2, 0, freq_dot=fd, gather="all", precision="exact")
    best = sharded_search(t, f, 3, 1, freq_dot=fd, gather="best", precision="exact")
    t0 = float((t[0] + t[-1]).item()) / 2
    fdd = torch.as_tensor(fd, device=dev)
    ref = ops.search(t, t0, f, 2, 0, log10_negfdot=fdd, precision="exact")
    refh = ops.search(t, t0, f, 3, 1, log10_negfdot=fdd, precision="exact").cpu().numpy()
    nu = _nufft_cases(t, f, t0, dev)
    tm = readPPtemplate(os.path.join(ROOT, "tests", "golden", "1e2259_template.txt"))
    K = sum(1 for k in tm if k.startswith("amp_"))
    x, off, E, _ = template_intervals_torch(5, 20_000, tm["norm"]["value"], [tm["amp_%d" % j]["value"] for j in
                                            range(1, K + 1)], [tm["ph_%d" % j]["value"] for j in range(1, K + 1)],
                                            seed=3, device=dev)
    toa = sharded_toa_fit(x, off, E, tm, brutemin=True)
    rtoa = ToAFitter(x, off, E, tm).fit(brutemin=True)
    keys = sorted(toa)
    np.savez(out_path, full=full.cpu().numpy(), full_is_dev=np.array(full.is_cuda), ref=ref.cpu().numpy(),
             best=np.array(best, dtype=np.float64), refh=refh, backend=np.array(dist.get_backend()),
             toa=np.stack([toa[k] for k in keys]), rtoa=np.stack([rtoa[k] for k in keys]), **nu)
    dist.destroy_process_group()


def test_nccl_backend_single_rank_on_gpu(tmp_path):
    """The nccl (RCCL) branch of sharding.py -- collective buffers on the device, the best-trial selection on the
    device -- executed for real: one rank (RCCL needs one GPU per rank, and this box has one), results equal to
    the unsharded device search and fits."""
    out = str(tmp_path / "n.npz")
    mp.spawn(_nccl_worker, args=(1, _free_port(), out), nprocs=1, join=True)
    r = np.load(out)
    assert str(r["backend"]) == "nccl" and bool(r["full_is_dev"])
    np.testing.assert_array_equal(r["full"], r["ref"])
    assert r["best"][0] == r["refh"].max() and int(r["best"][1]) == int(np.argmax(r["refh"]))
    np.testing.assert_array_equal(r["toa"], r["rtoa"])
    _check_nufft(r, 1)

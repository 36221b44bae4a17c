"""crimp_best (ops.best): the best trial of a device power array with np.argmax semantics -- what
sharding.sharded_search(gather='best') returns per rank -- against numpy on ties, NaN, -inf, ragged sizes around the
kernel's grid-stride slices, and a full config-3-sized array."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _check(x):
    import torch
    from crimp_amd import ops
    d = torch.as_tensor(x, device="cuda")
    v, i = ops.best(d)
    j = int(np.argmax(x))
    assert i == j, (i, j)
    if np.isnan(x[j]):
        assert np.isnan(v)
    else:
        assert v == x[j]


@pytest.mark.parametrize("n", [1, 2, 7, 255, 256, 2048, 2049, 524287, 1_000_000, 2 * 1024 * 2048 + 3])
def test_best_random_sizes(n):
    rng = np.random.default_rng(n)
    _check(rng.standard_normal(n))


def test_best_ties_nan_inf():
    x = np.zeros(100_000)
    x[[5, 70_000, 99_999]] = 3.0  # ties: the lowest index
    _check(x)
    x[[123, 50_000]] = np.nan     # NaN above every number, the first one wins
    _check(x)
    y = np.full(4099, -np.inf)    # all -inf: index 0
    _check(y)
    y[4098] = -1e300
    _check(y)


def test_best_matches_torch_max_path():
    """sharded_search(gather='best') on a device search equals np.argmax over the powers of the same call."""
    import torch
    from crimp_amd import ops
    from crimp_amd.sharding import sharded_search
    rng = np.random.default_rng(3)
    t = np.sort(rng.uniform(0, 1e4, 20_000))
    f = 0.5 + np.arange(4096) * 1e-5
    td, fd = torch.as_tensor(t, device="cuda"), torch.as_tensor(f, device="cuda")
    t0 = (t[0] + t[-1]) / 2
    z = ops.search(td, t0, fd, 2, 0).cpu().numpy()
    bv, bi = sharded_search(td, fd, 2, 0, gather="best", t0=t0)
    assert bi == int(np.argmax(z)) and bv == z[bi]


@pytest.mark.parametrize("precision", [None, "exact", "f64"])
def test_search_best_equals_search_and_argmax(precision):
    """crimp_search_best (the rank step of sharded_search(gather='best')): the same powers as crimp_search and the
    best trial np.argmax gives over them -- the NUFFT (best read back with the fix-up count), the exact and fp64
    paths (best after the search), a trial sub-range, host and device inputs, and a forced fix-up of many trials
    (CRIMP_FIXUP_REL in a child process: the best then follows the fp64 recomputation)."""
    import torch
    from crimp_amd import ops
    from crimp_amd import _native as N
    rng = np.random.default_rng(4)
    t = np.sort(rng.uniform(0, 2e4, 50_000))
    f = 0.5 + np.arange(3000) * 2e-6
    t0 = (t[0] + t[-1]) / 2
    for dev in (False, True):
        tt = torch.as_tensor(t, device="cuda") if dev else t
        ff = torch.as_tensor(f, device="cuda") if dev else f
        for first, count in ((0, 3000), (700, 1500)):
            z = ops.search(tt, t0, ff, 2, 0, first=first, count=count, precision=precision)
            z = z.cpu().numpy() if dev else z
            zb, bv, bi = ops.search_best(tt, t0, ff, 2, 0, first=first, count=count, precision=precision)
            zb = zb.cpu().numpy() if dev else zb
            np.testing.assert_array_equal(zb, z)
            assert bi == int(np.argmax(z)) and bv == z[bi]
            assert N.load().crimp_last_search_path() == {None: 2, "exact": 1, "f64": 0}[precision]


def test_search_best_after_fixups():
    import os
    import subprocess
    import sys
    import tempfile
    from conftest import ROOT
    code = ("import sys, numpy as np; sys.path.insert(0, %r); from crimp_amd import ops, _native as N; "
            "rng = np.random.default_rng(6); t = np.sort(rng.uniform(0, 2e4, 50000)); f = 0.5 + np.arange(3000) * 2e-6; "
            "t0 = (t[0] + t[-1]) / 2; z, bv, bi = ops.search_best(t, t0, f, 3, 1); nfix = N.load().crimp_last_fixups(); "
            "path = N.load().crimp_last_search_path(); z2 = ops.search(t, t0, f, 3, 1); "
            "np.savez(sys.argv[1], z=z, z2=z2, bv=bv, bi=bi, nfix=nfix, path=path)") % ROOT
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "b.npz")
        subprocess.run([sys.executable, "-c", code, out], check=True, timeout=300,
                       env=dict(os.environ, CRIMP_FIXUP_REL="1e-13"))
        r = np.load(out)
    assert int(r["path"]) == 2 and int(r["nfix"]) > 100
    np.testing.assert_array_equal(r["z"], r["z2"])
    assert int(r["bi"]) == int(np.argmax(r["z"])) and float(r["bv"]) == r["z"].max()

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

"""readvaryparam host driver: the interval-batched projected-Newton maximisation and 1-sigma scan
(crimp_amd/toafit_vary.py) give every interval exactly what a one-interval run gives, with fewer
evaluation batches. The device evaluation is replaced by a smooth per-interval test function, so this
runs on the CPU; the device path itself is covered by tests/test_gpu_parity.py::test_readvaryparam_*."""
import math

import numpy as np

from crimp_amd.toafit_vary import VaryParamFitter

NINT, P = 6, 5


def _fitter(rng):
    C = rng.normal(size=(NINT, P))
    M = rng.uniform(0.5, 3.0, size=(NINT, P))
    f = object.__new__(VaryParamFitter)
    f.blo, f.bhi = np.full(P, -2.0), np.full(P, 2.0)
    f.vary = np.array([True, True, False, True, True])
    f.nint, f.res, f.pb, f.model = NINT, 1000, math.pi, "cauchy"
    f.evals = np.zeros(NINT, dtype=np.int64)
    f.batches = 0
    f.off = 0   # interval index offset (one-interval fitters stand for interval `off` of the full set)

    def evaluate_theta(iv, thetas):
        iv = np.asarray(iv).reshape(-1) + f.off
        th = np.asarray(thetas, dtype=np.float64).reshape(iv.size, -1)
        f.batches += 1
        d = th - C[iv]
        ll = -np.sum(M[iv] * d ** 2, 1) - 0.1 * np.sum(d ** 4, 1) + np.sin(th[:, 0])
        g = -2 * M[iv] * d - 0.4 * d ** 3
        g[:, 0] += np.cos(th[:, 0])
        return ll, g

    f.evaluate_theta = evaluate_theta
    return f


def test_batched_maximise_matches_single_interval():
    f = _fitter(np.random.default_rng(3))
    start = np.tile(np.array([0.1, 0.2, 0.3, 0.0, 0.1]), (NINT, 1))
    single = [f._maximise(i, start[i], f.vary) for i in range(NINT)]
    n_single = f.batches
    f.batches = 0
    th, ll = f._maximise_batch(np.arange(NINT), start, f.vary)
    assert f.batches < n_single
    for i in range(NINT):
        assert np.array_equal(single[i][0], th[i])
        assert single[i][1] == ll[i]
    # the 1-sigma scan: every interval's step count is that of its own scan
    lo, up = f._scan(th, ll)
    for i in range(NINT):
        g = _fitter(np.random.default_rng(3))
        g.nint, g.off, g.evals = 1, i, np.zeros(1, dtype=np.int64)
        lo1, up1 = g._scan(th[i:i + 1], ll[i:i + 1])
        assert lo1[0] == lo[i] and up1[0] == up[i]
    assert np.all(lo > 0) and np.all(up > 0)

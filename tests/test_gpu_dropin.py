"""Drop-in details behind measureToAs and the C-ABI, on the GPU:

* interval selection without torch compute -- crimp_is_sorted, crimp_select_intervals and crimp_gather_ranges against
  the reference's own mask TIME[(TIME >= start) & (TIME <= end)] (measureToAs.py:173-174) and np.all(t[1:] >= t[:-1]),
  empty and NaN-bounded intervals, host and device inputs;
* the two in-kernel unit conversions measureToAs needs: crimp_search_sets with CRIMP_FLAG_TIME_DAYS equals the
  host's TIME_toa * 86400 (:211) bit for bit, crimp_calcphase with CRIMP_FLAG_FOLD_RADIANS the host's
  folded * (2 pi) (:195, :200);
* concurrent calls from two threads (the C-ABI serialises them process-wide) give the single-threaded results."""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _mask_select(T, starts, ends):
    sel = [T[(T >= a) & (T <= b)] for a, b in zip(starts, ends)]
    return sel


@pytest.mark.parametrize("device", [False, True])
def test_select_and_gather_match_the_reference_mask(gpu, device):
    import torch
    from crimp_amd import ops
    rng = np.random.default_rng(5)
    T = np.sort(58000.0 + rng.uniform(0.0, 30.0, 200_000))
    starts = np.sort(rng.uniform(57999.0, 58031.0, 300))
    ends = starts + rng.uniform(-0.1, 2.0, 300)          # some end before their start: empty
    starts[7], ends[9] = np.nan, np.nan                  # NaN bounds select nothing
    starts[11], ends[11] = T[1000], T[1000]              # a one-photon interval on a photon's exact time
    starts[12], ends[12] = T[-1], T[-1] + 1.0            # the last photon
    Tin = torch.as_tensor(T, device=gpu) if device else T
    assert ops.is_sorted(Tin)
    lo, cnt, first, last = ops.select_intervals(Tin, starts, ends)
    ref = _mask_select(T, starts, ends)
    np.testing.assert_array_equal(cnt, [r.size for r in ref])
    for i, r in enumerate(ref):
        if r.size:
            np.testing.assert_array_equal(T[lo[i]:lo[i] + cnt[i]], r)
            assert first[i] == r[0] and last[i] == r[-1]
        else:
            assert np.isnan(first[i]) and np.isnan(last[i])
    keep = cnt > 0
    offs = np.concatenate([[0], np.cumsum(cnt[keep])]).astype(np.int64)
    allt = ops.gather_ranges(Tin, lo[keep], offs)
    allt = allt.cpu().numpy() if hasattr(allt, "cpu") else allt
    np.testing.assert_array_equal(allt, np.concatenate([r for r in ref if r.size]))
    # order checks as np.all(t[1:] >= t[:-1]): a swapped pair, a NaN, ties
    for bad in (lambda x: x.__setitem__(slice(5000, 5002), x[5000:5002][::-1].copy()),
                lambda x: x.__setitem__(123456, np.nan)):
        U = T.copy()
        bad(U)
        assert not ops.is_sorted(torch.as_tensor(U, device=gpu) if device else U)
    assert ops.is_sorted(np.repeat(T[:1000], 3))
    with pytest.raises(Exception):  # a range beyond the photons is refused before any copy
        ops.gather_ranges(Tin, np.array([T.size - 5]), np.array([0, 10]))


def test_search_sets_days_and_calcphase_radians_match_host_conversions(gpu):
    import torch
    from crimp_amd import ops, _native as N
    from crimp_amd.calcphase import Phases
    rng = np.random.default_rng(8)
    t_days = np.sort(58000.0 + rng.uniform(0.0, 3.0, 60_000))
    offs = np.array([0, 10_000, 10_001, 35_000, 60_000], dtype=np.int64)
    freqs = np.array([0.14, 0.1430001, 2.5, 7.123456789])
    for dev in (False, True):
        tin = torch.as_tensor(t_days, device=gpu) if dev else t_days
        oin = torch.as_tensor(offs, device=gpu) if dev else offs
        fin = torch.as_tensor(freqs, device=gpu) if dev else freqs
        a = ops.search_sets(tin, oin, fin, 5, N.STAT_H, flags=N.FLAG_TIME_DAYS)
        b = ops.search_sets(tin * 86400, oin, fin, 5, N.STAT_H)
        a, b = [x.cpu().numpy() if hasattr(x, "cpu") else x for x in (a, b)]
        np.testing.assert_array_equal(a, b)
    tm = {"PEPOCH": 58001.0, "F0": 0.143, "F1": -1.2e-14, "F2": 3e-23}
    ph = Phases(t_days, tm)
    _, cyc = ops.calcphase(ph.timeMJD, ph.timModParam)
    _, rad = ops.calcphase(ph.timeMJD, ph.timModParam, flags=N.FLAG_FOLD_RADIANS)
    np.testing.assert_array_equal(rad, cyc * (2 * np.pi))
    _, rad1 = ops.calcphase(ph.timeMJD[1:], ph.timModParam, flags=N.FLAG_FOLD_RADIANS)  # odd count: scalar kernel
    np.testing.assert_array_equal(rad1, cyc[1:] * (2 * np.pi))


def test_concurrent_calls_from_two_threads(gpu):
    """The library's one mutex serialises calls process-wide: two threads searching and folding at once get exactly
    the results of the same calls made one after another."""
    from crimp_amd import ops
    from crimp_amd.synth import pulsed_events
    t = pulsed_events(100_000, 1.0e5, 3.0, pulsed_frac=0.1, seed=2)
    t0 = (t[0] + t[-1]) / 2
    f = 3.0 + np.arange(-1000, 1000) / 1.0e6
    tm = {"PEPOCH": 58000.0, "F0": 3.0}
    mjd = 58000.0 + t / 86400.0
    want_z = ops.search(t, t0, f, 2, 0)
    want_p = ops.calcphase(mjd, tm)[1]
    got, errs = {}, []

    def worker(k):
        try:
            for _ in range(5):
                got[("z", k)] = ops.search(t, t0, f, 2, 0)
                got[("p", k)] = ops.calcphase(mjd, tm)[1]
        except Exception as e:  # pragma: no cover - reported below
            errs.append(e)

    th = [threading.Thread(target=worker, args=(k,)) for k in range(2)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errs, errs
    for k in range(2):
        np.testing.assert_array_equal(got[("z", k)], want_z)
        np.testing.assert_array_equal(got[("p", k)], want_p)

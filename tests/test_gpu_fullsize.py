"""Parity at BASELINE.json's full sizes (configs 3 and 4): the device search over every trial, checked
against the oracle on a sample of trials computed over ALL photons (plain per-trial relative error), plus
size-independent properties (injected signal found at its trial, trial partitions bit-identical to the
whole, NUFFT vs exact path agreement on every trial, the chi^2_4 noise mean). Tolerances as tests/test_gpu_parity.py."""
import math

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _rel_err(got, ref):
    return np.abs(got - ref) / np.abs(ref)


def test_config3_full_size(gpu):
    import torch
    from crimp_amd import ops
    from crimp_amd.synth import pulsed_events
    n, M, span, f0 = 10_000_000, 1_000_000, 1.0e6, 7.123456789
    t_h = pulsed_events(n, span, f0, pulsed_frac=0.1, seed=0)
    df = 1.0 / (10.0 * span)
    f_h = f0 + (np.arange(M) - M // 2) * df
    t = torch.as_tensor(t_h, device=gpu)
    f = torch.as_tensor(f_h, device=gpu)
    t0 = (t_h[0] + t_h[-1]) / 2
    from crimp_amd import _native as N
    z = ops.search(t, t0, f, 2, 0, precision="exact").cpu().numpy()
    assert N.load().crimp_last_search_path() == 1
    # fix-up ceiling: the exact kernel, not the fp64 recomputation, must produce these powers (a kernel regression
    # that the certificate catches would send most trials through the fix-up and still pass the checks below)
    assert N.load().crimp_last_fixups() <= 16
    assert int(np.argmax(z)) == M // 2                       # the injected frequency's trial
    # oracle on sampled trials over all 1e7 photons
    rng = np.random.default_rng(1)
    idx = np.unique(np.concatenate([[M // 2, M // 2 - 1, M // 2 + 1, 0, M - 1], rng.integers(0, M, 11)]))
    zr = O.search(t_h, f_h[idx], 2)
    assert _rel_err(z[idx], zr).max() <= 1e-6
    # every trial of two 65536-trial windows (the peak's and the grid's start) against the fp64 kernel over all
    # photons (itself <= 4e-10 of the reference): the per-trial contract on 13 % of the grid
    z64 = {}
    for w0 in (0, M // 2 - 32768):
        z64[w0] = ops.search(t, t0, f, 2, 0, first=w0, count=65536, precision="f64").cpu().numpy()
        assert _rel_err(z[w0:w0 + 65536], z64[w0]).max() <= 1e-6
    # sharding: two halves computed separately equal the whole, bit for bit
    a = ops.search(t, t0, f, 2, 0, first=0, count=M // 2 + 123, precision="exact").cpu().numpy()
    b = ops.search(t, t0, f, 2, 0, first=M // 2 + 123, count=M - (M // 2 + 123), precision="exact").cpu().numpy()
    np.testing.assert_array_equal(np.concatenate([a, b]), z)
    # the default call (the reference's own PeriodSearch(t, f, 2).ztest() reaches it) runs the NUFFT over the whole
    # grid: every trial within 1e-6 relative of the exact path (both within 1e-6 of the reference), same best
    # trial, the sampled oracle trials at plain 1e-6, and its fix-up list small
    zn = ops.search(t, t0, f, 2, 0).cpu().numpy()
    assert N.load().crimp_last_search_path() == 2
    assert N.load().crimp_last_fixups() <= 16
    assert _rel_err(zn, z).max() <= 1e-6
    assert int(np.argmax(zn)) == M // 2
    assert _rel_err(zn[idx], zr).max() <= 1e-6
    for w0, ref in z64.items():
        assert _rel_err(zn[w0:w0 + 65536], ref).max() <= 1e-6
    # noise statistic: Z^2_2 of unpulsed trials is chi^2 with 4 dof (mean 4) far from the signal
    far = z[: M // 4]
    assert abs(far.mean() - 4.0) < 0.05


@pytest.mark.parametrize("precision", ["exact", None])
def test_config4_windows_vs_oracle(gpu, precision):
    """Config 4 at plain 1e-6 against the oracle over all 1e8 photons, on contiguous trial windows: 32 noise-level
    trials at the start of the far row (log10|fdot| = -13.5), 32 beside the peak and the peak with its neighbours in
    the row of the injected fdot (tests/golden/config4_windows.npz; the oracle needs ~16 s of 8 cores per trial, so
    its values are committed with checksums of the regenerated photons, tests/golden/gen_config4_windows.py).
    ``ref`` follows the reference's operation order (periodsearch.py:93-98, :118-123); ``true`` is the same formula
    with the argument carried exactly, so ref-vs-true is the reference's own argument rounding (<= 1.6e-7 here).
    The default (NUFFT) computes the windows' rows whole (1e5 trials each: a 32-trial range is below the NUFFT's
    64-trial minimum and would take the exact rule) and checks the windows cut from them."""
    import os
    import sys
    import torch
    from crimp_amd import ops, _native as N
    from crimp_amd.synth import pulsed_events
    from conftest import ROOT
    sys.path.insert(0, os.path.join(str(ROOT), "tests", "golden"))
    from gen_config4_windows import FD, FREQ, M, N as NPH, SPAN, F0, FDOT, WINDOWS, photon_checksums
    fx = np.load(os.path.join(str(ROOT), "tests", "golden", "config4_windows.npz"))
    t_h = pulsed_events(NPH, SPAN, F0, pulsed_frac=0.05, fdot=FDOT, seed=1)
    np.testing.assert_array_equal(photon_checksums(t_h), fx["checksums"])   # the fixture's photons, bit for bit
    t = torch.as_tensor(t_h, device=gpu)
    t0 = (t_h[0] + t_h[-1]) / 2
    del t_h
    f = torch.as_tensor(FREQ, device=gpu)
    fd = torch.as_tensor(FD, device=gpu)
    got, nfix, rows = [], 0, {}
    for r, j0, cnt in WINDOWS:
        if precision is None:
            if r not in rows:
                rows[r] = ops.search(t, t0, f, 20, 1, log10_negfdot=fd, first=r * M, count=M).cpu().numpy()
                assert N.load().crimp_last_search_path() == 2
                nfix += N.load().crimp_last_fixups()
            got.append(rows[r][j0:j0 + cnt])
            continue
        got.append(ops.search(t, t0, f, 20, 1, log10_negfdot=fd, first=r * M + j0, count=cnt,
                              precision="exact").cpu().numpy())
        assert N.load().crimp_last_search_path() == 1
        nfix += N.load().crimp_last_fixups()
    h = np.concatenate(got)
    assert _rel_err(h, fx["ref"]).max() <= 1e-6          # measured 2.6e-7 (profiles/r03/config4_windows.json)
    assert _rel_err(h, fx["true"]).max() <= 1e-6         # measured 1.4e-7
    assert np.median(_rel_err(h, fx["ref"])) <= 1e-7
    assert int(np.argmax(h)) == int(np.argmax(fx["ref"]))
    assert nfix <= (8 if precision == "exact" else 64)  # default: fix-ups over two whole rows of 1e5 trials


@pytest.mark.parametrize("precision", ["exact", None])
def test_config4_full_photon_count_h20(gpu, precision):
    """1e8 photons with fdot, 2-D H-test m=20 on a 3 x 8192 trial sub-grid (the full 1e7-trial grid runs sharded
    on 8 GPUs in the bench configuration) whose rows include both ends of config 4's log10|fdot| range: oracle over
    all photons on 8 sampled trials (plain per-trial relative error), and every fd row computed as its own trial
    range bit-identical to the whole grid (the exact path; the default NUFFT with its MFMA-slot spread)."""
    import torch
    from crimp_amd import ops, _native as N
    from crimp_amd.synth import pulsed_events
    n, span, f0, fdot = 100_000_000, 1.0e7, 7.123456789, -1.0e-12
    t_h = pulsed_events(n, span, f0, pulsed_frac=0.05, fdot=fdot, seed=1)
    df = 1.0 / (10.0 * span)
    M = 8192
    f_h = f0 + (np.arange(M) - M // 2) * df
    fd = np.array([-13.5, -12.0, -11.5])
    t = torch.as_tensor(t_h, device=gpu)
    f = torch.as_tensor(f_h, device=gpu)
    fdd = torch.as_tensor(fd, device=gpu)
    t0 = (t_h[0] + t_h[-1]) / 2
    hf = ops.search(t, t0, f, 20, 1, log10_negfdot=fdd, precision=precision).cpu().numpy()
    assert N.load().crimp_last_search_path() == (1 if precision == "exact" else 2)
    h = hf.reshape(3, M)
    r, j = np.unravel_index(int(np.argmax(h)), h.shape)
    assert r == 1 and j == M // 2                              # fdot = -1e-12 -> log10 = -12, f0 at index M/2
    for row in range(3):                                       # row-sharded, as 3 ranks would compute it
        hr = ops.search(t, t0, f, 20, 1, log10_negfdot=fdd, first=row * M, count=M, precision=precision).cpu().numpy()
        np.testing.assert_array_equal(hr, h[row])
    rng = np.random.default_rng(4)
    sample = [(1, M // 2), (1, M // 2 + 1), (0, 100), (2, M - 1)] + [(int(a), int(b)) for a, b in
                                                                       zip(rng.integers(0, 3, 4), rng.integers(0, M, 4))]
    for rr, jj in sample:
        ref = O.search(t_h, f_h[jj:jj + 1], 20, freq_dot=fd[rr:rr + 1], stat="h")[0]
        assert abs(h[rr, jj] - ref) <= 1e-6 * abs(ref), (rr, jj, h[rr, jj], ref)
    # every trial of the peak row's central 1024 against the fp64 kernel over all 1e8 photons. Two fp64
    # implementations that round the harmonic argument in different operation orders (the reference's
    # 2 pi k (f dt + ...), the fp64 kernel's k-fold angle additions, the exact kernel's factorised f_j dt) differ
    # per term by ~2^-53 of it: at k = 20, f = 7 Hz, |dt| ~ 3e6 s that is sigma_e ~ 5.6e-7 rad between two of them,
    # which moves H by ~2 sigma_e sqrt(sum_k Z_k) -- above 1e-6 of H only for noise-level H. The allowance is
    # 10 x that beside the 1e-6 relative contract; the oracle, which follows the reference's
    # operation order, checks the sampled trials above at plain 1e-6.
    w0 = M + M // 2 - 512
    h64 = ops.search(t, t0, f, 20, 1, log10_negfdot=fdd, first=w0, count=1024, precision="f64").cpu().numpy()
    dt = t_h - t0
    sig_e = 2 * 2.0 ** -53 * 2 * np.pi * 20 * f_h.max() * np.sqrt(np.mean(dt * dt))
    allow = 1e-6 * np.abs(h64) + 10 * 2 * sig_e * np.sqrt(np.maximum(h64, 0) + 4 * 19)
    got = hf[w0:w0 + 1024]
    assert np.all(np.abs(got - h64) <= allow), np.max(np.abs(got - h64) / allow)
    assert np.median(_rel_err(got, h64)) <= 1e-7


def test_trial_blocks_and_fixup(gpu, monkeypatch):
    """Trial blocking and the fp64 fix-up of the exact path. With a 4 MiB per-search buffer budget
    (CRIMP_SEARCH_BUDGET_MB) an H_20 search over 900k trials runs in ~70 trial blocks; with the fix-up
    threshold raised to 1e-3 (CRIMP_FIXUP_REL, a test hook) a large share of the trials goes through the fp64
    kernel. Both return, bit for bit, what the unblocked search and the fp64 path give for those trials, and
    every sampled trial is within 1e-6 relative of the oracle."""
    import torch
    from crimp_amd import ops
    from crimp_amd import _native as N
    from crimp_amd.synth import pulsed_events
    n, M, span, f0 = 2_000_000, 900_000, 1.0e6, 7.123456789
    t_h = pulsed_events(n, span, f0, pulsed_frac=0.1, seed=4)
    f_h = f0 + (np.arange(M) - M // 2) / (10.0 * span)
    t = torch.as_tensor(t_h, device=gpu)
    f = torch.as_tensor(f_h, device=gpu)
    t0 = (t_h[0] + t_h[-1]) / 2
    h = ops.search(t, t0, f, 20, 1, precision="exact").cpu().numpy()
    assert int(np.argmax(h)) == M // 2
    monkeypatch.setenv("CRIMP_SEARCH_BUDGET_MB", "4")
    hb = ops.search(t, t0, f, 20, 1, precision="exact").cpu().numpy()
    np.testing.assert_array_equal(hb, h)
    idx = np.array([0, 450_000, 450_559, 450_560, 450_561, M - 1])
    hr = O.search(t_h, f_h[idx], 20, stat="h")
    assert _rel_err(h[idx], hr).max() <= 1e-6
    # fix-up: a 2048-trial window in a fresh process-level setting (the thresholds are read once per process,
    # so the hook is exercised through a subprocess)
    import subprocess
    import sys
    code = ("import sys, numpy as np; sys.path.insert(0, %r); from crimp_amd import ops, _native as N; "
            "from crimp_amd.synth import pulsed_events; t = pulsed_events(200000, 2.0e5, 7.123456789, "
            "pulsed_frac=0.05, seed=4); f = 7.123456789 + np.arange(-1024, 1024) / 2.0e6; t0 = (t[0] + t[-1]) / 2; "
            "z = ops.search(t, t0, f, 2, 0, precision='exact'); nfix = N.load().crimp_last_fixups(); "
            "z64 = ops.search(t, t0, f, 2, 0, precision='f64'); np.savez(sys.argv[1], z=z, z64=z64, nfix=nfix)") % (
        str(__import__("conftest").ROOT))
    import tempfile
    import os
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "fx.npz")
        # at 3e-8 the error bound (10 sigma of 2^30 roundings, ~2e-8 of Z for a noise trial at 2e5 photons)
        # flags the low-power trials but not all of them
        env = dict(os.environ, CRIMP_FIXUP_REL="3e-8")
        subprocess.run([sys.executable, "-c", code, out], check=True, env=env, timeout=300)
        r = np.load(out)
    z, z64, nfix = r["z"], r["z64"], int(r["nfix"])
    assert 0 < nfix < z.size
    # the flagged trials hold fp64 sums (the fix-up kernel's photon splits differ from the f64 path's, so equal to
    # ~1e-15, where the exact kernel and the fp64 path differ by ~1e-9)
    fixed = np.abs(z - z64) <= 1e-12 * np.abs(z64)
    assert fixed.sum() >= nfix
    zr = O.search(pulsed_events(200000, 2.0e5, 7.123456789, pulsed_frac=0.05, seed=4),
                  f0 + np.arange(-1024, 1024) / 2.0e6, 2)
    assert _rel_err(z, zr).max() <= 1e-6


def _fit_vs_oracle(r, i, x, E, tm):
    """One interval of a device fit against O.fit_toa (measureToAs.py:254-403 restated): phShift within 1e-6
    cycles, the 1-sigma scan bounds identical (they are lattice values), redChi2 within 1e-6 relative."""
    import math
    o = O.fit_toa(x, E, tm, brutemin=True)
    assert abs(r["phShi"][i] - o["phShi"]) / (2 * math.pi) <= 1e-6, (i, r["phShi"][i], o["phShi"])
    assert r["phShi_LL"][i] == o["phShi_LL"] and r["phShi_UL"][i] == o["phShi_UL"], i
    assert abs(r["reducedChi2"][i] - o["reducedChi2"]) <= 1e-6 * abs(o["reducedChi2"]), i
    return o


def _grid_margins(f):
    """Relative gap between the best and the second-best point of each interval's brute grid (device grid, the
    same LL assembly as ToAFitter.brute)."""
    from crimp_amd import ops
    from crimp_amd.toafit import _is_torch
    nphi = int(np.ceil((2 * f.pb) / 0.05))
    phis = np.arange(nphi) * 0.05 + (-f.pb)
    norms = np.arange(20) * ((f.hi - f.lo) / 19.0) + f.lo
    ln, hmin = ops.toa_grid(f.x, f.offsets, f.tpl, f._arr(np.tile(norms, (f.nint, 1)), np.float64),
                            f._arr(phis, np.float64))
    if _is_torch(ln):
        ln, hmin = ln.cpu().numpy(), hmin.cpu().numpy()
    N, E, nn = f.N[:, None, None], f.E[:, None, None], norms[None, :, None]
    with np.errstate(divide="ignore", invalid="ignore"):
        ll = -nn * E + N * np.log(nn * E) + (ln - N * np.log(nn))
    ll = np.where(((hmin[:, None, :] + nn) > 0) & np.isfinite(ll), ll, -np.inf).reshape(f.nint, -1)
    top2 = -np.sort(-ll, axis=1)[:, :2]
    return (top2[:, 0] - top2[:, 1]) / np.abs(top2[:, 0])


def test_config5_toas_vs_oracle(gpu):
    """Config 5 per GPU: 1250 intervals x 1e5 photons (bench.py's workload, seed 2), batched device fits
    (brute + MLE + 1-sigma scan + redChi2), compared with the oracle on sampled intervals -- including the
    intervals whose fp32-evaluated brute grid has the closest top-two points (a lattice tie can hand the
    maximiser a different start)."""
    import os
    from crimp_amd.readPPtemplate import readPPtemplate
    from crimp_amd.synth import template_intervals_torch
    from crimp_amd.toafit import ToAFitter
    from conftest import gpath
    O.set_threads(min(16, os.cpu_count() or 1))
    tm = readPPtemplate(gpath("1e2259_template.txt"))
    K = sum(1 for k in tm if k.startswith("amp_"))
    amps = [tm["amp_%d" % j]["value"] for j in range(1, K + 1)]
    phs = [tm["ph_%d" % j]["value"] for j in range(1, K + 1)]
    x, off, E, shifts = template_intervals_torch(1250, 100_000, tm["norm"]["value"], amps, phs, seed=2, device=gpu)
    f = ToAFitter(x, off, E, tm)
    r = f.fit(brutemin=True)
    d = np.angle(np.exp(1j * (r["phShi"] - shifts)))
    assert np.sqrt(np.mean(d ** 2)) / (2 * np.pi) < 5e-3                # all 1250 recover their injected shift
    margins = _grid_margins(ToAFitter(x, off, E, tm))
    ties = [int(i) for i in np.argsort(margins)[:2]]
    sample = sorted(set([0, 1, 417, 833, 1249, 600] + ties))
    xh, oh = x.cpu().numpy(), off.cpu().numpy()
    for i in sample:
        _fit_vs_oracle(r, i, xh[oh[i]:oh[i + 1]], E[i], tm)
    assert margins[ties[0]] < 1e-5       # the sample did include a near-tie of the lattice
    clipped = _every_interval_vs_oracle_profile(r, xh, oh, E, tm)
    print("config 5 per GPU: %d clipped scan positions checked" % clipped)


def _scan_position(phi, side, k, step, pb, fourier):
    """phShift of the reference's 1-sigma scan at its k-th step on one side (measureToAs.py:330-376 as O.fit_toa
    restates it, lmfit's clip-to-bound semantics): the target phi + side k step clipped to the phShift bounds
    +-pb; for Fourier templates a step taken while the previous one sat on +-pi moves that bound to the target
    (the scan then walks past +-pi), for Cauchy / von Mises the scan stays on the bound."""
    pmin, pmax, cur = -pb, pb, phi
    for kk in range(1, k + 1):
        target = phi + side * kk * step
        if fourier:
            if side < 0 and kk > 1 and cur <= -math.pi:
                pmin = target
            if side > 0 and kk > 1 and cur >= math.pi:
                pmax = target
        cur = min(max(target, pmin), pmax)
    return cur


def _every_interval_vs_oracle_profile(r, xh, oh, E, tm, ph_shift_res=1000, workers=None):
    """Every interval of a device fit against the oracle's fp64 extended likelihood (templatemodels.py:98-121), a
    few likelihood passes each instead of a whole oracle fit (measureToAs.py:320-376):
    * optimum: at the device's (norm, phShift) the profile's Newton step -g_phi / (H_pp - H_pn^2 / H_nn) is below
      1e-6 cycles and the norm's -g_n / H_nn below 1e-9 of the norm (the device optimum is the oracle's);
    * 1-sigma scan: with k* = kk - 1 the scan step the reported bound kk * step + step / 2 implies on each side, the
      norm-profiled LL at the scan's step k* - 1 lies within 0.5 chi2_1(0.6827) = 0.500021713558733 of LLmax and at
      step k* beyond it -- the crossing is exactly where the device reported it. The scan's positions follow lmfit's
      clip to the phShift bounds (_scan_position: the intervals whose scan reaches +-pi are checked on the clipped
      and bound-moving steps, not skipped); a scan that reached the phShiftRes / 2 cap is checked inside up to it."""
    import math
    import os
    from concurrent.futures import ThreadPoolExecutor
    thr = 0.500021713558733
    tarr = O.template_arrays(tm)
    fourier = str(tm["model"]).lower() == "fourier"
    pb = math.pi if fourier else 1.5 * math.pi
    n0 = float(tm["norm"]["value"])
    lo, hi = n0 / 100.0, 500.0
    step = 2 * math.pi / ph_shift_res

    def one(i):  # the oracle's C calls release the GIL: intervals run on a thread pool
        x = xh[oh[i]:oh[i + 1]]
        phi, n = float(r["phShi"][i]), float(r["norm"][i])
        o = O.toa_eval(x, E[i], tarr, n, phi)
        heff = o[5] - o[4] * o[4] / o[3]
        step_phi = -(o[2] - o[4] * o[1] / o[3]) / heff  # profile Newton step (norm re-maximised)
        if abs(phi) >= pb - 1e-9 and step_phi * phi > 0:
            wphi = 0.0  # the maximum lies past the phShift bound: the bounded fit stops there (lmfit's bounds)
        else:
            wphi = abs(step_phi) / (2 * math.pi)
        wn = abs(o[1] / o[3]) / n if lo < n < hi else 0.0
        llmax = O._profile_norm(x, E[i], tarr, phi, lo, hi, n)[1][0]
        bad, clipped = [], 0
        for side, bound in ((-1, r["phShi_LL"][i]), (1, r["phShi_UL"][i])):
            kk = int(round((bound - step / 2) / step))
            kstar = kk - 1
            capped = kstar + 1 > ph_shift_res / 2
            checks = [(kstar - 1, True)] if capped else [(kstar - 1, True), (kstar, False)]
            for k, inside in checks:
                if k < 1:
                    continue
                p = _scan_position(phi, side, k, step, pb, fourier)
                clipped += p != phi + side * k * step
                _, ok = O._profile_norm(x, E[i], tarr, p, lo, hi, n)
                diff = llmax - ok[0]
                if not ((diff <= thr) if inside else (diff > thr)):
                    bad.append((i, side, k, kstar, diff))
        return wphi, wn, bad, clipped

    workers = workers or max(1, min(16, len(os.sched_getaffinity(0))))
    with ThreadPoolExecutor(workers) as ex:
        res = list(ex.map(one, range(len(E))))
    bad = [b for _, _, bb, _ in res for b in bb]
    assert not bad, bad[:5]
    iphi = int(np.argmax([w for w, _, _, _ in res]))
    inrm = int(np.argmax([w for _, w, _, _ in res]))
    worst_phi, worst_n = res[iphi][0], res[inrm][1]
    assert worst_phi <= 1e-6, (iphi, worst_phi, float(r["phShi"][iphi]), float(r["norm"][iphi]))
    assert worst_n <= 1e-9, (inrm, worst_n, float(r["phShi"][inrm]), float(r["norm"][inrm]))
    return sum(c for _, _, _, c in res)


@pytest.mark.timeout(900)
def test_config5_whole_every_interval_vs_oracle(gpu):
    """The whole of config 5 on one GPU -- 1e4 intervals x 1e5 photons, bench.py's toa_full_config5 workload (seed
    12) -- every interval against the oracle's profile likelihood as above, the bound-adjacent intervals included
    (their scans replayed with lmfit's clip-to-bound steps)."""
    import os
    import torch
    from crimp_amd.readPPtemplate import readPPtemplate
    from crimp_amd.synth import template_intervals_torch
    from crimp_amd.toafit import ToAFitter
    from conftest import gpath
    O.set_threads(1)
    tm = readPPtemplate(gpath("1e2259_template.txt"))
    K = sum(1 for k in tm if k.startswith("amp_"))
    amps = [tm["amp_%d" % j]["value"] for j in range(1, K + 1)]
    phs = [tm["ph_%d" % j]["value"] for j in range(1, K + 1)]
    x, off, E, shifts = template_intervals_torch(10_000, 100_000, tm["norm"]["value"], amps, phs, seed=12, device=gpu)
    r = ToAFitter(x, off, E, tm).fit(brutemin=True)
    d = np.angle(np.exp(1j * (r["phShi"] - shifts)))
    assert np.sqrt(np.mean(d ** 2)) / (2 * np.pi) < 5e-3
    xh, oh = x.cpu().numpy(), off.cpu().numpy()
    del x
    torch.cuda.empty_cache()
    near = int(np.sum(np.abs(r["phShi"]) + 60 * 2 * np.pi / 1000 >= np.pi))
    clipped = _every_interval_vs_oracle_profile(r, xh, oh, E, tm, workers=max(1, min(16, len(os.sched_getaffinity(0)))))
    print("config 5 whole: %d intervals, %d fitted within 60 scan steps of +-pi, %d clipped scan positions checked"
          % (len(E), near, clipped))
    assert near > 0 and clipped > 0  # the bound-adjacent intervals were checked, not skipped


def _sample_template(tm, n, shift, rng):
    """n phases in [0, 2 pi) from a Cauchy / von Mises template shifted by ``shift`` (rejection sampling on the
    oracle's curve, templatemodels.py:166-185, 271-290)."""
    tarr = O.template_arrays(tm)
    n0 = tm["norm"]["value"]
    ymax = 1.05 * O.curve(tarr, n0, shift, np.linspace(0, 2 * np.pi, 20001)).max()
    out = np.empty(0)
    while out.size < n:
        xx = rng.uniform(0, 2 * np.pi, 3 * n)
        keep = rng.uniform(0, ymax, xx.size) < O.curve(tarr, n0, shift, xx)
        out = np.concatenate([out, xx[keep]])
    return out[:n]


def test_cauchy_vonmises_blocks_1e5(gpu):
    """One Cauchy and one von Mises block (3 intervals x 1e5 photons each) fitted on the device against
    O.fit_toa (measureToAs.py:406-548, :551-693)."""
    import json
    import os
    from crimp_amd.toafit import ToAFitter
    from conftest import gpath
    O.set_threads(min(16, os.cpu_count() or 1))
    tc = json.load(open(gpath("cauchy_vm_theta.json")))
    rng = np.random.default_rng(7)
    for model in ("cauchy", "vonmises"):
        tm = {"model": model, "norm": {"value": tc["norm"], "vary": True}}
        for j in (1, 2):
            for nm in ("amp", "cen", "wid"):
                tm["%s_%d" % (nm, j)] = {"value": tc["%s_%d" % (nm, j)], "vary": True}
        n = 100_000
        rate = tc["norm"] + (tc["amp_1"] + tc["amp_2"]) / (2 * np.pi)   # mean of the template over a turn
        xs = [_sample_template(tm, n, s, rng) for s in (0.3, -2.0, 3.5)]
        x = np.concatenate(xs)
        off = np.arange(len(xs) + 1, dtype=np.int64) * n
        E = np.full(len(xs), n / rate)
        r = ToAFitter(x, off, E, tm).fit(brutemin=True)
        for i in range(len(xs)):
            _fit_vs_oracle(r, i, xs[i], E[i], tm)


@pytest.mark.parametrize("precision", ["exact", None])
def test_exact_vs_f64_every_trial(gpu, precision):
    """The per-trial contract on every trial of larger grids, near-zero powers included: the exact (+ fix-up) path
    and the default (NUFFT + fix-up) against the fp64 path (itself within 1e-8 of the reference's outputs), 1e6
    photons, Z^2_4 over 16384 trials and 2-D H_20 over 2 x 8192 trials."""
    import torch
    from crimp_amd import ops, _native as N
    from crimp_amd.synth import pulsed_events
    t_h = pulsed_events(1_000_000, 1.0e6, 7.123456789, pulsed_frac=0.02, fdot=-1e-12, seed=9)
    t = torch.as_tensor(t_h, device=gpu)
    t0 = (t_h[0] + t_h[-1]) / 2
    f = torch.as_tensor(7.123456789 + (np.arange(16384) - 8192) / 1.0e7, device=gpu)
    z = ops.search(t, t0, f, 4, 0, precision=precision).cpu().numpy()
    assert N.load().crimp_last_search_path() == (1 if precision == "exact" else 2)
    z64 = ops.search(t, t0, f, 4, 0, precision="f64").cpu().numpy()
    assert _rel_err(z, z64).max() <= 1e-6
    fd = torch.as_tensor(np.array([-12.0, -11.0]), device=gpu)
    h = ops.search(t, t0, f[4096:12288], 20, 1, log10_negfdot=fd, precision=precision).cpu().numpy()
    nfix = N.load().crimp_last_fixups()
    h64 = ops.search(t, t0, f[4096:12288], 20, 1, log10_negfdot=fd, precision="f64").cpu().numpy()
    assert _rel_err(h, h64).max() <= 1e-6
    assert nfix < h.size // 10


def test_exact_many_harmonics_and_ragged_partitions(gpu):
    """H_64 on the exact path against the fp64 path on every trial, and a 2-D grid of rows that are not a whole
    number of 1024-trial tiles split at arbitrary flat indices (mid-row, mid-tile): the pieces equal the whole
    bit for bit."""
    import torch
    from crimp_amd import ops
    from crimp_amd.synth import pulsed_events
    t_h = pulsed_events(200_000, 2.0e5, 3.3, pulsed_frac=0.05, seed=12)
    t = torch.as_tensor(t_h, device=gpu)
    t0 = (t_h[0] + t_h[-1]) / 2
    f = torch.as_tensor(3.3 + (np.arange(1000) - 500) / 2.0e6, device=gpu)
    h = ops.search(t, t0, f, 64, 1, precision="exact").cpu().numpy()
    h64 = ops.search(t, t0, f, 64, 1, precision="f64").cpu().numpy()
    assert _rel_err(h, h64).max() <= 1e-6
    hd = ops.search(t, t0, f, 64, 1).cpu().numpy()   # the default (NUFFT) at 64 harmonics
    assert _rel_err(hd, h64).max() <= 1e-6
    fd = torch.as_tensor(np.array([-13.0, -12.0, -11.0]), device=gpu)
    whole = ops.search(t, t0, f, 2, 0, log10_negfdot=fd, precision="exact").cpu().numpy()
    cuts = [0, 1, 999, 1500, 2047, 2100, 3000]
    parts = [ops.search(t, t0, f, 2, 0, log10_negfdot=fd, first=a, count=b - a, precision="exact").cpu().numpy()
             for a, b in zip(cuts[:-1], cuts[1:])]
    np.testing.assert_array_equal(np.concatenate(parts), whole)


def test_exact_path_above_2_27_photons(gpu):
    """The exact kernel's int64 totals hold < 2^27 photons; 1.5e8 photons (a config-4-style search, which
    periodsearch.py:57-71 puts no limit on) run in two photon chunks, each into its own totals, summed exactly by the
    finalize: the exact path (not the fp64 kernel) runs, with few fix-ups, within 1e-6 of the fp64 path on every
    trial; the NUFFT agrees too. Just below 2^27 a single chunk runs and matches the same way."""
    import torch
    from crimp_amd import ops, _native as N
    g = torch.Generator(device=gpu)
    g.manual_seed(5)
    n = 150_000_000
    t = torch.sort(5.0e9 + torch.rand(n, generator=g, dtype=torch.float64, device=gpu) * 1.0e6).values
    f = torch.as_tensor(1.7 + (np.arange(256) - 128) / 1.0e7, device=gpu)
    t0 = float((t[0] + t[-1]).item()) / 2
    for nn in (n, (1 << 27) - 1):
        tt = t[:nn]
        z = ops.search(tt, t0, f, 2, 0, precision="exact").cpu().numpy()
        assert N.load().crimp_last_search_path() == 1
        assert N.load().crimp_last_fixups() <= 8
        z64 = ops.search(tt, t0, f, 2, 0, precision="f64").cpu().numpy()
        assert _rel_err(z, z64).max() <= 1e-6
        assert not np.array_equal(z, z64)       # a different (exact) kernel ran
        zn = ops.search(tt, t0, f, 2, 0).cpu().numpy()   # the default
        assert N.load().crimp_last_search_path() == 2
        assert _rel_err(zn, z64).max() <= 1e-6


def test_exact_long_splits_fold_path_bit_identical(gpu):
    """Splits longer than one fold period (131072 photons) keep int64 running sums in global scratch between
    folds; the default split choice avoids them whenever it can, so a test hook (CRIMP_EXACT_LONG_SPLITS) forces
    the earlier policy. The totals are exact integers, so both give the same powers bit for bit (4e6 photons: 1-D
    Z^2_3 over 2e6 trials, splits of ~444k photons with three intermediate folds; 2-D H_8 over 2 x 524288
    trials, ~250k photons and one)."""
    import os
    import subprocess
    import sys
    import tempfile
    code = (
        "import sys, numpy as np; sys.path.insert(0, %r); from crimp_amd import ops; "
        "from crimp_amd.synth import pulsed_events; "
        "import torch; t_h = pulsed_events(4000000, 1.0e6, 7.123456789, pulsed_frac=0.05, seed=6); "
        "t = torch.as_tensor(t_h, device='cuda'); t0 = (t_h[0] + t_h[-1]) / 2; "
        "f = torch.as_tensor(7.123456789 + np.arange(-1000000, 1000000) / 1.0e7, device='cuda'); "
        "z = ops.search(t, t0, f, 3, 0, precision='exact').cpu().numpy(); "
        "fd = torch.as_tensor(np.array([-13.0, -12.0]), device='cuda'); "
        "h = ops.search(t, t0, f[:524288], 8, 1, log10_negfdot=fd, precision='exact').cpu().numpy(); "
        "np.savez(sys.argv[1], z=z, h=h)") % (str(__import__("conftest").ROOT))
    with tempfile.TemporaryDirectory() as d:
        res = []
        for hook in (False, True):
            out = os.path.join(d, "ls%d.npz" % hook)
            env = dict(os.environ)
            if hook:
                env["CRIMP_EXACT_LONG_SPLITS"] = "1"
            subprocess.run([sys.executable, "-c", code, out], check=True, env=env, timeout=300)
            res.append(np.load(out))
    np.testing.assert_array_equal(res[0]["z"], res[1]["z"])
    np.testing.assert_array_equal(res[0]["h"], res[1]["h"])

"""The exact search path's per-trial certificate under inputs that correlate its 2^30 roundings, the routing and
trial-blocking edge cases of crimp_search, and varyAmps bounds per template model.

The exact kernel (csrc/search_exact.h) flags for the fp64 fix-up every trial whose 10-sigma error bound (an
independent-rounding model: per-term rms 1e-9) cannot place it within 1e-6 relative. These tests hold the model to
inputs built to break the independence -- photon times on a 1/(4096 f0) lattice (every photon's phase lands on the
same table cells with zero residual rotation), every photon duplicated, a 90 %-pulsed source -- by comparing every
trial with the fp64 path, and the trials where that differs by more than 1e-6 with the oracle in the reference's
operation order: the default result (fix-up on) at plain 1e-6, and the raw kernel (FLAG_NO_FIXUP) at plain 1e-6 on
every trial the certificate passed."""
import math
import os
import subprocess
import sys
import tempfile

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _rel(got, ref):
    return np.abs(got - ref) / np.abs(ref)


def _correlated_inputs():
    from crimp_amd.synth import pulsed_events
    f0, n = 7.123456789, 1_000_000
    base = pulsed_events(n, 1.0e6, f0, pulsed_frac=0.1, seed=21)
    q = 1.0 / (4096.0 * f0)
    quant = np.round(base / q) * q                           # times on the table lattice of the fundamental
    half = pulsed_events(n // 2, 1.0e6, f0, pulsed_frac=0.1, seed=22)
    dup = np.sort(np.concatenate([half, half]))              # every photon twice
    strong = pulsed_events(n, 1.0e6, f0, pulsed_frac=0.9, seed=23)
    return f0, {"quantised": quant, "duplicated": dup, "pulsed90": strong}


def _within_1e6_of_reference(got, z64, t_h, f_h, nharm, stat, name, what):
    """Every trial within 1e-6 relative of the fp64 path or, where it is not, of the oracle in the reference's
    operation order (``ref``). At m = 20 two fp64 evaluations with different argument roundings (the reference's
    2 pi k f dt, the fp64 kernel's angle additions, the exact kernel's f_j dt, the NUFFT's f_0 + j delta model of
    the grid, whose values deviate from the array's by a few ulp) differ by ~2^-53 of the k = 20 argument per term,
    which moves a noise-level H by up to ~1e-6 where H = Z^2_m - 4 (m - 1) cancels (duplicated photons double it
    coherently): there the reference itself is that far from the exact-argument value (``true``, the same formula
    with the argument carried exactly), and the contract is DESIGN.md section 8's exception -- the device as close to
    ``true`` as the reference is, plus 1e-6. Measured (tools/diag_cert.py, tools/diag_nufft_harm.py,
    profiles/r06/diag_nufft_harm_duplicated.log): duplicated photons, H_20, trial 7429, H = Z^2_20 - 76 = 0.4985
    (153x cancellation): the reference 2.5e-6 from ``true``, the exact path 1.8e-6, the NUFFT 1.1e-6, the fp64
    kernel 8.6e-8."""
    e = _rel(got, z64)
    off = np.flatnonzero(e > 1e-6)
    assert off.size <= 32, (name, what, off.size)
    if off.size:
        ref = O.search(t_h, f_h[off], nharm, stat="h" if stat else "z2")
        er = _rel(got[off], ref)
        tru = O.search(t_h, f_h[off], nharm, stat="h" if stat else "z2", exact_argument=True)
        exc = np.abs(got[off] - tru) <= np.abs(ref - tru) + 1e-6 * np.abs(tru)
        ok = (er <= 1e-6) | ((_rel(ref, tru) > 1e-6) & exc)
        assert ok.all(), (name, what, er[~ok], _rel(ref, tru)[~ok], int(off[~ok][0]))
    return e, off.size


@pytest.mark.parametrize("precision", ["exact", None])
@pytest.mark.parametrize("nharm,stat", [(2, 0), (20, 1)])
def test_certificate_holds_on_correlated_inputs(gpu, nharm, stat, precision):
    """precision="exact": the exact kernel's statistical certificate; None: the default NUFFT's truncation-bound
    certificate (crimp_last_search_path() == 2) on the same correlated inputs."""
    import torch
    from crimp_amd import ops, _native as N
    O.set_threads(min(16, os.cpu_count() or 1))
    f0, inputs = _correlated_inputs()
    f_h = f0 + (np.arange(8192) - 4096) / 1.0e7
    f = torch.as_tensor(f_h, device=gpu)
    for name, t_h in inputs.items():
        t = torch.as_tensor(t_h, device=gpu)
        t0 = (t_h[0] + t_h[-1]) / 2
        z = ops.search(t, t0, f, nharm, stat, precision=precision).cpu().numpy()
        assert N.load().crimp_last_search_path() == (1 if precision == "exact" else 2)
        nfix = N.load().crimp_last_fixups()
        raw = ops.search(t, t0, f, nharm, stat, flags=N.FLAG_NO_FIXUP, precision=precision).cpu().numpy()
        z64 = ops.search(t, t0, f, nharm, stat, precision="f64").cpu().numpy()
        e, noff = _within_1e6_of_reference(z, z64, t_h, f_h, nharm, stat, name, "default")
        flagged = z != raw                                   # the fix-up rewrote exactly the flagged trials
        assert flagged.sum() <= nfix, (name, flagged.sum(), nfix)
        cert = np.flatnonzero(~flagged)
        er, _ = _within_1e6_of_reference(raw[cert], z64[cert], t_h, f_h[cert], nharm, stat, name,
                                         "raw kernel on a certified trial")
        assert nfix <= 64, (name, nfix)                      # a kernel regression would flag most trials
        assert int(np.argmax(z)) == int(np.argmax(z64))
        print("%s %s m=%d: max rel vs fp64 %.2e (raw certified %.2e), %d checked against the oracle, fix-ups %d" % (
            precision or "default", name, nharm, e.max(), er.max(), noff, nfix))


def _run_child(code, env_extra, out):
    env = dict(os.environ, **env_extra)
    subprocess.run([sys.executable, "-c", code, out], check=True, env=env, timeout=300)
    return np.load(out)


def test_fold_path_many_ragged_trial_blocks_2d(gpu):
    """Splits longer than one fold period (CRIMP_EXACT_LONG_SPLITS) over a 2-D grid cut into many trial blocks
    (CRIMP_SEARCH_BUDGET_MB=1: 8192 trials per block) whose rows (3000 trials: one full tile and a ragged one)
    start at every offset inside a block: the fold scratch is sized over all blocks and the powers equal the
    default search's bit for bit (integer sums)."""
    code = ("import sys, numpy as np; sys.path.insert(0, %r); from crimp_amd import ops, _native as N; "
            "from crimp_amd.synth import pulsed_events; import torch; "
            "t_h = pulsed_events(3000000, 1.0e6, 7.123456789, pulsed_frac=0.05, seed=31); "
            "t = torch.as_tensor(t_h, device='cuda'); t0 = (t_h[0] + t_h[-1]) / 2; "
            "f = torch.as_tensor(7.123456789 + (np.arange(3000) - 1500) / 1.0e7, device='cuda'); "
            "fd = torch.as_tensor(np.linspace(-13.0, -11.0, 40), device='cuda'); "
            "h = ops.search(t, t0, f, 8, 1, log10_negfdot=fd, first=1234, count=100000, precision='exact').cpu().numpy(); "
            "np.savez(sys.argv[1], h=h)") % (str(__import__("conftest").ROOT))
    with tempfile.TemporaryDirectory() as d:
        a = _run_child(code, {}, os.path.join(d, "a.npz"))
        b = _run_child(code, {"CRIMP_EXACT_LONG_SPLITS": "1", "CRIMP_SEARCH_BUDGET_MB": "1"}, os.path.join(d, "b.npz"))
    np.testing.assert_array_equal(a["h"], b["h"])


def test_short_rows_2d_route_to_fp64(gpu):
    """A 2-D grid of 2-trial rows (300 rows) would fill 2048-trial tiles with dead columns: it takes the fp64
    kernel (bit-identical to precision='f64'); 256-trial rows take the NUFFT by default and the exact kernel with
    precision='exact'."""
    import torch
    from crimp_amd import ops
    from crimp_amd.synth import pulsed_events
    t_h = pulsed_events(200_000, 2.0e5, 3.3, pulsed_frac=0.05, seed=12)
    t = torch.as_tensor(t_h, device=gpu)
    t0 = (t_h[0] + t_h[-1]) / 2
    fd = torch.as_tensor(np.linspace(-13.0, -10.0, 300), device=gpu)
    f2 = torch.as_tensor(3.3 + np.arange(2) / 2.0e6, device=gpu)
    z = ops.search(t, t0, f2, 2, 0, log10_negfdot=fd).cpu().numpy()
    z64 = ops.search(t, t0, f2, 2, 0, log10_negfdot=fd, precision="f64").cpu().numpy()
    np.testing.assert_array_equal(z, z64)
    f256 = torch.as_tensor(3.3 + np.arange(256) / 2.0e6, device=gpu)
    from crimp_amd import _native as N
    assert N.load().crimp_last_search_path() == 0
    z64 = ops.search(t, t0, f256, 2, 0, log10_negfdot=fd[:4], precision="f64").cpu().numpy()
    for prec, path in ((None, 2), ("exact", 1)):
        z = ops.search(t, t0, f256, 2, 0, log10_negfdot=fd[:4], precision=prec).cpu().numpy()
        assert N.load().crimp_last_search_path() == path
        assert not np.array_equal(z, z64) and _rel(z, z64).max() <= 1e-6


def _sample_template(tm, n, shift, rng):
    tarr = O.template_arrays(tm)
    n0 = tm["norm"]["value"]
    ymax = 1.05 * O.curve(tarr, n0, shift, np.linspace(0, 2 * np.pi, 20001)).max()
    out = np.empty(0)
    while out.size < n:
        xx = rng.uniform(0, 2 * np.pi, 3 * n)
        keep = rng.uniform(0, ymax, xx.size) < O.curve(tarr, n0, shift, xx)
        out = np.concatenate([out, xx[keep]])
    return out[:n]


def test_vary_amps_bounds_per_model(gpu):
    """varyAmps frees ampShift in [0.01, 100] for Fourier (measureToAs.py:308), [0, inf) for Cauchy (:461) and
    [0, 500] for von Mises (:605). Photons drawn from a template whose amplitudes are 150x the fitting template's
    push ampShift to ~150: Cauchy and von Mises fit it freely, Fourier stops at 100. Device fits (k_toa_fit_amp)
    against the oracle's restatement (parity unpinned beyond the oracle: no reference output uses varyAmps)."""
    import json
    from crimp_amd.toafit import ToAFitter
    from conftest import gpath
    O.set_threads(min(16, os.cpu_count() or 1))
    tc = json.load(open(gpath("cauchy_vm_theta.json")))
    rng = np.random.default_rng(17)
    n = 10_000
    for model in ("cauchy", "vonmises"):
        gen = {"model": model, "norm": {"value": tc["norm"], "vary": True}}
        fit = {"model": model, "norm": {"value": tc["norm"], "vary": True}}
        for j in (1, 2):
            for nm in ("amp", "cen", "wid"):
                v = tc["%s_%d" % (nm, j)]
                gen["%s_%d" % (nm, j)] = {"value": v, "vary": True}
                fit["%s_%d" % (nm, j)] = {"value": v / 150.0 if nm == "amp" else v, "vary": True}
        x = _sample_template(gen, n, 0.4, rng)
        rate = tc["norm"] + (tc["amp_1"] + tc["amp_2"]) / (2 * np.pi)
        E = n / rate
        r = ToAFitter(x, np.array([0, n], dtype=np.int64), np.array([E]), fit).fit(brutemin=True, vary_amps=True)
        o = O.fit_toa_vary_amps(x, E, fit, brutemin=True)
        assert r["ampShift"][0] > 100.0, (model, r["ampShift"][0])
        assert r["ampShift"][0] == pytest.approx(o["ampShift"], rel=1e-5), model
        assert abs(r["phShi"][0] - o["phShi"]) / (2 * math.pi) < 1e-6, model
        assert r["phShi_LL"][0] == o["phShi_LL"] and r["phShi_UL"][0] == o["phShi_UL"], model


def test_pruned_brute_grid_equals_full_grid(gpu):
    """crimp_toa_fit evaluates only the brute-grid norms that can hold a phShift's maximum (the extended LL is
    strictly concave in norm). The fits must equal, bit for bit, the fits that evaluate all 20
    norms of lmfit's grid (CRIMP_TOA_FULL_GRID test hook; read per call, so one process runs both): config-5-style
    Fourier intervals and the Cauchy / von Mises templates, the device records compared whole."""
    import json
    from crimp_amd.synth import template_intervals_torch
    from crimp_amd.toafit import ToAFitter
    from conftest import gpath
    from bench import T2259, _tmpl
    x, off, E, _ = template_intervals_torch(300, 100_000, T2259["norm"]["value"], T2259["amp"], T2259["ph"], seed=5,
                                            device=gpu)
    cases = [(x, off, E, _tmpl())]
    tc = json.load(open(gpath("cauchy_vm_theta.json")))
    rng = np.random.default_rng(3)
    for model in ("cauchy", "vonmises"):
        tm = {"model": model, "norm": {"value": tc["norm"], "vary": True}}
        for j in (1, 2):
            for nm in ("amp", "cen", "wid"):
                tm["%s_%d" % (nm, j)] = {"value": tc["%s_%d" % (nm, j)], "vary": True}
        xs = [_sample_template(tm, 20_000, s, rng) for s in (0.3, -2.0, 3.5, 1.0)]
        rate = tc["norm"] + (tc["amp_1"] + tc["amp_2"]) / (2 * np.pi)
        cases.append((np.concatenate(xs), np.arange(5, dtype=np.int64) * 20_000, np.full(4, 20_000 / rate), tm))
    os.environ["CRIMP_TOA_GRID_SLOW"] = "1"  # the same grid kernel for both (the fast form: the test below)
    try:
        for xx, oo, ee, tm in cases:
            a = ToAFitter(xx, oo, ee, tm).fit(brutemin=True)
            os.environ["CRIMP_TOA_FULL_GRID"] = "1"
            try:
                b = ToAFitter(xx, oo, ee, tm).fit(brutemin=True)
            finally:
                del os.environ["CRIMP_TOA_FULL_GRID"]
            for k in ("phShi", "phShi_LL", "phShi_UL", "reducedChi2", "norm", "LLmax"):
                np.testing.assert_array_equal(a[k], b[k], err_msg="%s %s" % (tm["model"], k))
    finally:
        del os.environ["CRIMP_TOA_GRID_SLOW"]


def test_fast_brute_grid_equals_full_kernel(gpu, monkeypatch):
    """The device fit's fast brute grid (k_toa_grid_mf with log2 of products of eight model values, and without the
    per-phShift min h where the template's bound makes every candidate point valid; crimp_toa_fit certifies both)
    against the full kernel (CRIMP_TOA_GRID_SLOW): config-5-style Fourier intervals, every interval. The lattice LL
    values differ only by fp32 rounding, so the lattice point is the same and the fits reach the same maximum (the
    parabola-vertex start moves by rounding only): phShift within 1e-9 cycles, identical 1-sigma bounds, LLmax within
    1e-12 relative. (Config 5's lower candidate norm, norm0/100, is lazy and shown invalid by the phase histogram:
    mode 6.)"""
    from crimp_amd import _native as N
    from crimp_amd.synth import template_intervals_torch
    from crimp_amd.toafit import ToAFitter
    from bench import T2259, _tmpl
    x, off, E, _ = template_intervals_torch(400, 100_000, T2259["norm"]["value"], T2259["amp"], T2259["ph"], seed=6,
                                            device=gpu)
    monkeypatch.delenv("CRIMP_TOA_GRID_SLOW", raising=False)
    a = ToAFitter(x, off, E, _tmpl()).fit(brutemin=True)
    assert N.load().crimp_last_toa_grid_fast() == 6  # eight factors, lazy norms by the histogram certificate
    monkeypatch.setenv("CRIMP_TOA_GRID_SLOW", "1")
    b = ToAFitter(x, off, E, _tmpl()).fit(brutemin=True)
    assert N.load().crimp_last_toa_grid_fast() == 0
    np.testing.assert_allclose(a["phShi"], b["phShi"], rtol=0, atol=2 * np.pi * 1e-9)
    np.testing.assert_array_equal(a["phShi_LL"], b["phShi_LL"])
    np.testing.assert_array_equal(a["phShi_UL"], b["phShi_UL"])
    np.testing.assert_allclose(a["LLmax"], b["LLmax"], rtol=1e-12)


def test_lazy_norm_certificate_equals_min_path(gpu, monkeypatch):
    """The brute grid's lazy-norm certificate (kGridCert: the lazy points shown invalid by photon-holding histogram
    bins whose template bound is below -norm, no per-phShift min h) against the same kernel with the min
    (CRIMP_TOA_NO_CERT): identical records and redChi2 for config-5-style intervals, host and device inputs, and the
    same shape 2 times brighter and 100 times fainter; and no
    certificate where no norm is lazy (a weak template: every candidate norm valid everywhere)."""
    from crimp_amd import _native as N
    from crimp_amd.synth import template_intervals_torch
    from crimp_amd.toafit import ToAFitter
    from bench import T2259, _tmpl
    x, off, E, _ = template_intervals_torch(300, 50_000, T2259["norm"]["value"], T2259["amp"], T2259["ph"], seed=8,
                                            device=gpu)
    for scale, (xs, os_) in ((1.0, (x, off)), (1.0, (x.cpu().numpy(), off.cpu().numpy())), (2.0, (x, off)),
                             (0.01, (x, off))):
        tm = _tmpl()  # the same shape 2 times brighter / 100 times fainter (lmfit's lattice keeps a lazy lowest norm)
        for k in tm:
            if k == "norm" or k.startswith("amp_"):
                tm[k] = {"value": tm[k]["value"] * scale}
        Es = E / scale
        monkeypatch.delenv("CRIMP_TOA_NO_CERT", raising=False)
        a = ToAFitter(xs, os_, Es, tm).fit(brutemin=True)
        assert N.load().crimp_last_toa_grid_fast() == 6
        monkeypatch.setenv("CRIMP_TOA_NO_CERT", "1")
        b = ToAFitter(xs, os_, Es, tm).fit(brutemin=True)
        assert N.load().crimp_last_toa_grid_fast() == 2
        for k in a:
            np.testing.assert_array_equal(np.asarray(a[k]), np.asarray(b[k]), err_msg=k)
    monkeypatch.delenv("CRIMP_TOA_NO_CERT", raising=False)
    weak = _tmpl()
    for k in weak:
        if k.startswith("amp_"):
            weak[k] = {"value": weak[k]["value"] * 0.01}
    xw, offw, Ew, _ = template_intervals_torch(20, 20_000, T2259["norm"]["value"], [a_ * 0.01 for a_ in T2259["amp"]],
                                               T2259["ph"], seed=9, device=gpu)
    ToAFitter(xw, offw, Ew, weak).fit(brutemin=True)
    assert N.load().crimp_last_toa_grid_fast() & 4 == 0

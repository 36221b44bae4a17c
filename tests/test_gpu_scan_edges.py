"""The reference's 1-sigma-scan edge cases on the device fit (crimp_toa_fit), against the oracle.

measureToAs.py:331-376 (and the Cauchy / von Mises copies) steps phShift away from the best fit by
2 pi / phShiftRes with lmfit's bound semantics, and stops at the first LLmax - LL > 0.5 chi2_1(0.6827) or once its
counter passes phShiftRes/2, logging 'Could not estimate lower/upper-bound uncertainty on <ToA>'. The cases below
put the fitted phShift 0-3 steps from each bound of each model (Fourier: the first step past +-pi is clipped and
later steps move the bound; Cauchy / von Mises: every step past +-1.5 pi is clipped, so the scan stays on the
bound until the cap), one Fourier interval whose maximum lies beyond -pi (the ascent stops on the bound), and
weakly pulsed 200-photon intervals at phShiftRes = 20 whose likelihood never drops by 0.5 before the cap.
Photons are rejection-sampled from the shifted template (seeded). Each case: phShift within 1e-6 cycles of
oracle.fit_toa, phShift_LL / phShift_UL identical (capped value (res/2 + 1) step + step/2 included), redChi2
within 1e-6 relative, the capped sides as expected, and the drop-in measureToA_* logs the reference's warning.
"""
import json
import logging
import math
import os

import numpy as np
import pytest

from conftest import gpath
import oracle.oracle as O

pytestmark = pytest.mark.gpu

STEP = 2 * math.pi / 1000


def _fourier():
    from crimp_amd.readPPtemplate import readPPtemplate
    return readPPtemplate(gpath("1e2259_template.txt"))


def _cv(model):
    tc = json.load(open(gpath("cauchy_vm_theta.json")))
    tm = {"model": model, "norm": {"value": tc["norm"], "vary": True}}
    for j in (1, 2):
        for nm in ("amp", "cen", "wid"):
            tm["%s_%d" % (nm, j)] = {"value": tc["%s_%d" % (nm, j)], "vary": True}
    return tm


def _weak(tm, f):
    t = {k: (dict(v) if isinstance(v, dict) else v) for k, v in tm.items()}
    for k in t:
        if k.startswith("amp_"):
            t[k]["value"] *= f
    return t


def _rate(tm):
    amps = sum(v["value"] for k, v in tm.items() if k.startswith("amp_"))
    return tm["norm"]["value"] + (0.0 if tm["model"] == "fourier" else amps / (2 * math.pi))


def _sample(tm, n, shift, seed):
    """n phases (cycles for Fourier, radians otherwise) from the template shifted by ``shift`` (the oracle's
    curve, templatemodels.py:64-82, :166-185, :271-290), exposure n / mean rate."""
    rng = np.random.default_rng(seed)
    tarr = O.template_arrays(tm)
    n0 = tm["norm"]["value"]
    up = 1.0 if tm["model"] == "fourier" else 2 * math.pi
    ymax = 1.05 * O.curve(tarr, n0, shift, np.linspace(0, up, 20001)).max()
    out = np.empty(0)
    while out.size < n:
        x = rng.uniform(0, up, 3 * n)
        keep = rng.uniform(0, ymax, x.size) < O.curve(tarr, n0, shift, x)
        out = np.concatenate([out, x[keep]])
    return out[:n], n / _rate(tm)


# (model, name, template, photons, injected shift, seed, phShiftRes, brutemin, fitted-phShift window in steps
#  from (-bound, +bound), expected capped (lower, upper))
PB = {"fourier": math.pi, "cauchy": 1.5 * math.pi, "vonmises": 1.5 * math.pi}
CASES = [
    ("fourier", "near-bound", 30000, -math.pi + 1.5 * STEP, 101, 1000, True, ("lo", 1, 4), (False, False)),
    ("fourier", "near+bound", 30000, math.pi - 3.0 * STEP, 101, 1000, True, ("hi", 1, 4), (False, False)),
    ("fourier", "beyond-bound", 30000, math.pi - 1.0 * STEP, 101, 1000, True, ("lo", 0, 0), (False, False)),
    ("cauchy", "near+bound", 30000, 1.5 * math.pi - 2 * STEP, 101, 1000, True, ("hi", 1, 4), (False, True)),
    ("cauchy", "near-bound", 30000, -1.5 * math.pi + 1.2 * STEP, 102, 1000, True, ("lo", 0, 4), (True, False)),
    ("vonmises", "near+bound", 30000, 1.5 * math.pi - 2 * STEP, 102, 1000, True, ("hi", 1, 4), (False, True)),
    ("vonmises", "on-bound", 30000, -1.5 * math.pi + 1.2 * STEP, 102, 1000, True, ("lo", 0, 0), (True, False)),
] + [(m, "weak-capped-bm%d" % bm, 200, 0.7, 5, 20, bool(bm), None, (True, True))
     for m in ("fourier", "cauchy", "vonmises") for bm in (1, 0)]


def _template(model, name):
    tm = _fourier() if model == "fourier" else _cv(model)
    return _weak(tm, 0.03) if name.startswith("weak") else tm


@pytest.mark.parametrize("case", CASES, ids=["%s-%s" % (c[0], c[1]) for c in CASES])
def test_scan_edge_vs_oracle(gpu, case, caplog):
    from crimp_amd.measureToAs import measureToA_cauchy, measureToA_fourier, measureToA_vonmises
    from crimp_amd.toafit import ToAFitter, scan_capped
    model, name, n, shift, seed, res, bm, window, capped = case
    O.set_threads(min(16, os.cpu_count() or 1))
    tm = _template(model, name)
    x, E = _sample(tm, n, shift, seed)
    r = ToAFitter(x, np.array([0, x.size]), np.array([E]), tm, ph_shift_res=res).fit(brutemin=bm)
    o = O.fit_toa(x, E, tm, ph_shift_res=res, brutemin=bm)
    phi = float(r["phShi"][0])
    if window is not None:  # the case sits where it is meant to: `k` steps inside the named bound
        side, k0, k1 = window
        steps = (phi + PB[model]) / STEP if side == "lo" else (PB[model] - phi) / STEP
        assert k0 - 1e-9 <= steps <= k1, (phi, steps)
    assert abs(phi - o["phShi"]) / (2 * math.pi) <= 1e-6, (phi, o["phShi"])
    assert r["phShi_LL"][0] == o["phShi_LL"] and r["phShi_UL"][0] == o["phShi_UL"], (r["phShi_LL"], r["phShi_UL"],
                                                                                  o["phShi_LL"], o["phShi_UL"])
    assert abs(r["reducedChi2"][0] - o["reducedChi2"]) <= 1e-6 * abs(o["reducedChi2"])
    cap = (bool(scan_capped(r["phShi_LL"], res)[0]), bool(scan_capped(r["phShi_UL"], res)[0]))
    assert cap == capped
    step = 2 * math.pi / res
    for c, v in zip(cap, (r["phShi_LL"][0], r["phShi_UL"][0])):
        if c:  # the capped bound is (res/2 + 1) steps + half a step, as the reference's loop leaves kk
            assert v == (res // 2 + 1) * step + step / 2
    # the drop-in logs the reference's warning text for each capped side (measureToAs.py:348-350, :373-375)
    fn = {"fourier": measureToA_fourier, "cauchy": measureToA_cauchy, "vonmises": measureToA_vonmises}[model]
    with caplog.at_level(logging.WARNING):
        caplog.clear()
        d = fn(tm, x, E, outFile="ToA7", phShiftRes=res, brutemin=bm)
    assert d["phShi"] == phi and d["phShi_LL"] == r["phShi_LL"][0] and d["phShi_UL"] == r["phShi_UL"][0]
    msgs = [rec.getMessage() for rec in caplog.records]
    for c, side in zip(cap, ("lower", "upper")):
        text = "Could not estimate {}-bound uncertainty on ToA7".format(side)
        assert (text in msgs) == c, (text, msgs)


def _scaled_fourier(f):
    t = _fourier()
    t = {k: (dict(v) if isinstance(v, dict) else v) for k, v in t.items()}
    for k in t:
        if k.startswith("amp_") or k == "norm":
            t[k]["value"] *= f
    return t


@pytest.mark.parametrize("scale", [1e-3, 3e4])
def test_brute_grid_faint_and_bright_templates_vs_oracle(gpu, scale):
    """k_toa_grid_mf carries the template coefficients as hi + lo f16: a faint template (amplitudes ~1e-3 counts/s)
    would put the lo parts among the f16 subnormals and a bright one (amplitudes > 65504) would overflow; the kernel
    scales the coefficients and norms by a power of two (grid_mf_scale) and undoes it exactly. The lattice LL and its
    argmax against the oracle's fp64 grid, as test_brute_grid_vs_oracle does for the bundled template."""
    from crimp_amd import ops
    tm = _scaled_fourier(scale)
    tarr = O.template_arrays(tm)
    tpl = ops.make_template("fourier", tarr[2], tarr[3])
    n0 = tm["norm"]["value"]
    xs = [_sample(tm, 20000, s, seed)[0] for s, seed in ((0.4, 11), (-2.2, 12))]
    x = np.concatenate(xs)
    off = np.array([0, xs[0].size, x.size])
    norms = np.linspace(0.6 * n0, 1.4 * n0, 20)
    phis = np.arange(126) * 0.05 - np.pi
    ln, hmin = ops.toa_grid(x, off, tpl, np.tile(norms, (2, 1)), phis)
    for i, xi in enumerate(xs):
        E = xi.size / n0
        ref = O.toa_grid(xi, E, tarr, norms, phis)
        N = xi.size
        got = -norms[:, None] * E + N * np.log(norms[:, None] * E) + ln[i] - N * np.log(norms[:, None])
        got = np.where(hmin[i][None, :] + norms[:, None] > 0, got, -np.inf)
        fin = np.isfinite(ref)
        assert fin.all() and np.array_equal(fin, np.isfinite(got))
        # fp32 log2 of products of four model values: ~1e-7 of each term, as for the bundled template
        np.testing.assert_allclose(got, ref, rtol=2e-7, atol=0.05)
        assert np.unravel_index(np.argmax(got), got.shape) == np.unravel_index(np.argmax(ref), ref.shape)
        # min h over the photons at each phShift: the template's own scale (not 2^se times it)
        hm_ref = np.array([np.min(O.curve(tarr, 0.0, p, xi)) for p in phis[::25]])
        np.testing.assert_allclose(hmin[i][::25], hm_ref, rtol=1e-5, atol=1e-6 * np.max(np.abs(hm_ref)))


def _double_peaked(model):
    """Templates with two nearly equal peaks per turn (a start in the wrong basin would reach the other maximum)."""
    if model == "fourier":
        return {"model": "fourier", "norm": {"value": 12.0, "vary": True},
                "amp_1": {"value": 0.4, "vary": True}, "ph_1": {"value": 0.3, "vary": True},
                "amp_2": {"value": 4.0, "vary": True}, "ph_2": {"value": -0.8, "vary": True},
                "amp_3": {"value": 0.6, "vary": True}, "ph_3": {"value": 1.1, "vary": True}}
    return {"model": "vonmises", "norm": {"value": 5.0, "vary": True},
            "amp_1": {"value": 6.0, "vary": True}, "cen_1": {"value": 1.0, "vary": True}, "wid_1": {"value": 0.3, "vary": True},
            "amp_2": {"value": 5.5, "vary": True}, "cen_2": {"value": 1.0 + math.pi, "vary": True},
            "wid_2": {"value": 0.3, "vary": True}}


@pytest.mark.parametrize("model", ["fourier", "vonmises"])
def test_ascent_start_reaches_the_lattice_points_maximum(gpu, model, monkeypatch):
    """The device ascent starts at the brute lattice phShift with the norm at the photon rate N/E and the phShift at
    the parabola vertex (k_toa_grid_best), where lmfit hands its second minimiser the lattice point itself
    (measureToAs.py:292-299). On double-peaked templates, where the two starts could fall into different basins,
    every interval's fit from the shipped start equals the fit from the plain lattice point (test hook
    CRIMP_TOA_LATTICE_START): the same phShift (1e-9 cycles), LLmax (1e-12 relative) and identical 1-sigma bounds."""
    from crimp_amd.toafit import ToAFitter
    tm = _double_peaked(model)
    rng = np.random.default_rng(21)
    shifts = rng.uniform(-0.9 * PB[model], 0.9 * PB[model], 48)
    xs = [_sample(tm, 4000 + 500 * (i % 7), s, 300 + i)[0] for i, s in enumerate(shifts)]
    x = np.concatenate(xs)
    off = np.concatenate([[0], np.cumsum([a.size for a in xs])])
    E = np.array([a.size / _rate(tm) for a in xs])
    monkeypatch.delenv("CRIMP_TOA_LATTICE_START", raising=False)
    a = ToAFitter(x, off, E, tm).fit(brutemin=True)
    monkeypatch.setenv("CRIMP_TOA_LATTICE_START", "1")
    b = ToAFitter(x, off, E, tm).fit(brutemin=True)
    np.testing.assert_allclose(a["phShi"], b["phShi"], rtol=0, atol=2 * math.pi * 1e-9)
    np.testing.assert_allclose(a["LLmax"], b["LLmax"], rtol=1e-12)
    assert np.array_equal(a["phShi_LL"], b["phShi_LL"]) and np.array_equal(a["phShi_UL"], b["phShi_UL"])


def test_projected_ascent_on_the_bound_device_equals_host(gpu):
    """A maximum beyond -pi: the ascent stops on the bound and holds phShift there while the norm takes its own
    Newton steps (projected Newton, k_toa_fit's fit_newton_dir and toafit._newton_step); the device driver and the
    host-driven iterations agree (phShift exactly -pi, norm and LLmax to 1e-12, identical 1-sigma bounds), and the
    norm is the profile maximum there (dLL/dnorm ~ 0), which is what the redChi2 against the oracle needs."""
    from crimp_amd.toafit import ToAFitter
    case = [c for c in CASES if c[1] == "beyond-bound"][0]
    model, name, n, shift, seed, res, bm, window, capped = case
    tm = _template(model, name)
    x, E = _sample(tm, n, shift, seed)
    f = ToAFitter(x, np.array([0, x.size]), np.array([E]), tm, ph_shift_res=res)
    d = f.fit(brutemin=True)
    h = f.fit_host(brutemin=True)
    assert d["phShi"][0] == -math.pi and h["phShi"][0] == -math.pi
    np.testing.assert_allclose(d["norm"], h["norm"], rtol=1e-12)
    np.testing.assert_allclose(d["LLmax"], h["LLmax"], rtol=1e-12)
    assert d["phShi_LL"][0] == h["phShi_LL"][0] and d["phShi_UL"][0] == h["phShi_UL"][0]
    ll, g, H = f.evaluate(np.array([0]), d["norm"], d["phShi"])
    assert abs(g[0, 0]) <= 1e-6 * abs(E)        # dLL/dnorm = -E + sum 1/m vanishes at the profiled norm

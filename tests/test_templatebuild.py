"""Template building (pulseprofile.py of CRIMP v2.3.0) against the bundled worked example.

Pin: ``data/1e2259_template.log`` records that ``data/1e2259_template.txt`` is the BFGS fit of the
bundled observation (1-5 keV, 70 bins, Fourier, 6 harmonics); its chi2 57.248608783903634 for
57 dof is reproduced exactly from the bundled events + GTIs (tests/golden/events_1e2259.npz,
gti_1e2259.npz) -- that pins livetime, phases, binning, the model curve and measurechi2. lmfit
(absent) stopped its BFGS 5.6e-8 (relative) above the chi2 minimum; the fits here must reach the
minimum found independently by the oracle (least squares, tight tolerances), so parameters are
compared through chi2 and the model curve, not digit by digit.
"""
import numpy as np
import pytest

from conftest import gold, gpath
from crimp_amd.pulseprofile import (ModelPulseProfile, calcpulseproperties, calcuncertaintypulseproperties,
                                    measurechi2, writetemplatefile)
from crimp_amd.readPPtemplate import readPPtemplate
from crimp_amd.templatemodels import Fourier

GOLD_CHI2 = 57.248608783903634
NBINS, ELO, EHI = 70, 1.0, 5.0


def _events():
    ev, g = gold("events_1e2259.npz"), gold("gti_1e2259.npz")
    mjdref = int(ev["MJDREFI"]) + float(ev["MJDREFF"])
    gti = np.vstack((g["START"], g["STOP"])).T / 86400 + mjdref
    return ev, g, mjdref, np.sum(gti[:, 1] - gti[:, 0]) * 86400


@pytest.fixture(scope="module")
def profile():
    from oracle import oracle as O
    ev, _, mjdref, live = _events()
    pi = ev["PI"] * 0.01
    keep = (pi >= ELO) & (pi <= EHI)
    _, fol = O.calcphase(ev["TIME"][keep] / 86400 + mjdref, gpath("1e2259.par"))
    return O.binned_profile(fol, NBINS, live)


def _theta(t):
    return {k: float(v["value"]) for k, v in t.items() if isinstance(v, dict)}


def test_golden_template_chi2_reproduced(profile):
    t = readPPtemplate(gpath("1e2259_template.txt"))
    th = dict(_theta(t), phShift=0.0, ampShift=1.0)
    model = Fourier(th, profile["ppBins"]).fourseries()
    r = measurechi2(profile, model, 13)
    assert r["dof"] == 57
    assert r["chi2"] == pytest.approx(GOLD_CHI2, rel=1e-12)


def test_writetemplatefile_reproduces_golden_text(tmp_path):
    t = readPPtemplate(gpath("1e2259_template.txt"))
    lines = open(gpath("1e2259_template.txt")).read().splitlines()
    res = dict(_theta(t), phShift=0.0, ampShift=1.0, chi2=float(lines[-3].split()[1]), dof=int(lines[-2].split()[1]),
               redchi2=float(lines[-1].split()[1]), model="fourier")
    writetemplatefile(str(tmp_path / "t"), res)
    assert open(tmp_path / "t.txt").read() == open(gpath("1e2259_template.txt")).read()


def test_fourier_fit_reaches_the_chi2_minimum(profile):
    from oracle import oracle as O
    t = readPPtemplate(gpath("1e2259_template.txt"))
    _, cmin = O.fit_binned_template(profile, "fourier", _theta(t))
    assert cmin <= GOLD_CHI2 and cmin == pytest.approx(GOLD_CHI2, rel=1e-7)
    gold_curve = Fourier(dict(_theta(t), phShift=0.0, ampShift=1.0), profile["ppBins"]).fourseries()
    for init in (gpath("1e2259_template.txt"), None):  # from the template, and from the default start
        res, model = ModelPulseProfile(dict(profile), 6, init).fouriermodel()
        assert res["dof"] == 57 and res["model"] == "fourier"
        assert res["chi2"] == pytest.approx(cmin, rel=2e-8)
        assert res["chi2"] <= GOLD_CHI2
        # same optimum as the reference's template: curves within 1e-3 of the error bars
        assert np.max(np.abs(model - gold_curve) / profile["countRateErr"]) < 1e-3


def test_fix_phases_keeps_them_and_counts_like_the_reference(profile):
    t = readPPtemplate(gpath("1e2259_template.txt"))
    res, _ = ModelPulseProfile(dict(profile), 6, gpath("1e2259_template.txt"), fixPhases=True).fouriermodel()
    for k in range(1, 7):
        assert res["ph_%d" % k] == float(t["ph_%d" % k]["value"])
    assert res["dof"] == 57  # pulseprofile.py:335-338 counts the template's vary flags, not fixPhases
    # fixed phases at the template's values: no worse than the template, no better than the free minimum
    assert 57.248605589 * (1 - 1e-9) <= res["chi2"] <= GOLD_CHI2


@pytest.mark.parametrize("model", ["cauchy", "vonmises"])
def test_peaked_models_reach_a_chi2_minimum(profile, model):
    from oracle import oracle as O
    pp = dict(profile)
    pp["ppBins"] = profile["ppBins"] * 2 * np.pi
    mp = ModelPulseProfile(pp, 2)
    res, curve = mp.cauchymodel() if model == "cauchy" else mp.vonmisesmodel()
    assert res["dof"] == NBINS - 5 and res["model"] == model
    th = {k: res[k] for k in res if k.split("_")[0] in ("norm", "amp", "cen", "wid")}
    assert 0 <= th["norm"] <= np.max(pp["countRate"])
    assert all(0 <= th["cen_%d" % j] <= 2 * np.pi for j in (1, 2))
    bounds = {"norm": (0, np.max(pp["countRate"]))}
    bounds.update({k: (0, np.inf) for k in th if k[:3] in ("amp", "wid")})
    bounds.update({k: (0, 2 * np.pi) for k in th if k[:3] == "cen"})
    _, cpol = O.fit_binned_template(pp, model, th, bounds)
    assert res["chi2"] == pytest.approx(O.chi2_of(pp, model, th), rel=1e-12)
    assert res["chi2"] == pytest.approx(cpol, rel=1e-8)  # the oracle's polish finds nothing lower


def test_pulsed_properties_known_answer():
    x = np.linspace(0, 1, 32, endpoint=False) + 1 / 64
    n, a1, a2 = 10.0, 2.0, 0.5
    pp = {"ppBins": x, "countRate": n + a1 * np.cos(2 * np.pi * x + 0.3) + a2 * np.cos(4 * np.pi * x - 1.1),
          "countRateErr": np.zeros_like(x)}
    p = calcpulseproperties(pp, 2)
    assert p["harmonicPulsedFractions"] == pytest.approx([a1 ** 2 / 4, a2 ** 2 / 4], rel=1e-12)
    assert p["pulsedFlux"] == pytest.approx(np.sqrt((a1 ** 2 + a2 ** 2) / 2), rel=1e-12)
    assert p["pulsedFraction"] == pytest.approx(p["pulsedFlux"] / n, rel=1e-12)
    # error terms enter as the reference writes them: (sum err^2 cos^2 / N^2)^2 subtracted
    e = np.full_like(x, 0.4)
    p2 = calcpulseproperties(dict(pp, countRateErr=e), 2)
    s = np.sum(e ** 2 * np.cos(2 * np.pi * x) ** 2) / 32 ** 2, np.sum(e ** 2 * np.sin(2 * np.pi * x) ** 2) / 32 ** 2
    assert p2["harmonicPulsedFractions"][0] == pytest.approx(a1 ** 2 / 4 - (s[0] ** 2 + s[1] ** 2), rel=1e-12)
    u = calcuncertaintypulseproperties(dict(pp, countRateErr=e), 2, rng=np.random.default_rng(5))
    u2 = calcuncertaintypulseproperties(dict(pp, countRateErr=e), 2, rng=np.random.default_rng(5))
    assert u["pulsedFluxErr"] == u2["pulsedFluxErr"] and 0 < u["pulsedFluxErr"] < 0.2
    assert u["harmonicPulsedFractionsErr"].shape == (2,)


@pytest.mark.gpu
def test_template_cli_end_to_end(gpu, tmp_path, profile):
    """templatepulseprofile on a FITS file rebuilt from the bundled events and GTIs, phases and the
    histogram on the device: counts identical to the oracle's, chi2 at the minimum."""
    from crimp_amd.eventfile import write_fits
    from crimp_amd.pulseprofile import PulseProfileFromEventFile, main
    from oracle import oracle as O
    ev, g, _, _ = _events()
    kw = {"TELESCOP": "NICER", "MJDREFI": int(ev["MJDREFI"]), "MJDREFF": float(ev["MJDREFF"]), "TIMESYS": "TDB"}
    evf = str(tmp_path / "obs.fits")
    write_fits(evf, [("EVENTS", [("TIME", "1D", ev["TIME"]), ("PI", "1I", ev["PI"])], kw),
                     ("GTI", [("START", "1D", g["START"]), ("STOP", "1D", g["STOP"])], kw)])
    pp = PulseProfileFromEventFile(evf, gpath("1e2259.par"), ELO, EHI, NBINS).createpulseprofile()
    np.testing.assert_array_equal(pp["ppBins"], profile["ppBins"])
    np.testing.assert_array_equal(pp["countRate"], profile["countRate"])
    np.testing.assert_array_equal(pp["countRateErr"], profile["countRateErr"])
    out = str(tmp_path / "tpl")
    main([evf, gpath("1e2259.par"), "-el", "1", "-eh", "5", "-nb", "70", "-it", gpath("1e2259_template.txt"),
          "-tf", out, "-fg", out])
    t = readPPtemplate(out + ".txt")
    assert t["model"] == "fourier" and int(t["nbrComp"]) == 6
    lines = open(out + ".txt").read().splitlines()
    assert lines[-2] == "dof 57"
    _, cmin = O.fit_binned_template(profile, "fourier", _theta(readPPtemplate(gpath("1e2259_template.txt"))))
    assert float(lines[-3].split()[1]) == pytest.approx(cmin, rel=2e-8)
    assert (tmp_path / "tpl.pdf").stat().st_size > 0 and (tmp_path / "tpl.log").stat().st_size > 0

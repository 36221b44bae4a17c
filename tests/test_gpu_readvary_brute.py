"""readvaryparam + brutemin (measureToAs.py:292-295 with the Parameters of :727-801): lmfit's brute lattice over
every free parameter, on the device (VaryParamFitter.brute_lattice, one crimp_toa_grid launch per lattice template),
against the oracle's restatement (oracle.readvary_brute + fit_toa_readvary). Parity unpinned beyond the oracle: no
reference output uses readvaryparam, and lmfit (absent) aborts brute after max_nfev = 1e4 evaluations."""
import math

import numpy as np
import pytest

from conftest import gpath
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _case():
    """1e2259 template with norm and ph_2 free; photons drawn from it with ph_2 moved by 2 rad and shifted by
    2 rad: from the template start (phShift 0) the local maximum is a different, lower mode than the lattice's."""
    from crimp_amd.readPPtemplate import readPPtemplate
    from crimp_amd.synth import template_phases
    tm = readPPtemplate(gpath("1e2259_template.txt"))
    K = 6
    amps = [tm["amp_%d" % j]["value"] for j in range(1, K + 1)]
    phs = [tm["ph_%d" % j]["value"] for j in range(1, K + 1)]
    phs[1] = (phs[1] + 2.0 + np.pi) % (2 * np.pi) - np.pi
    x = template_phases(5000, tm["norm"]["value"], amps, phs, 2.0, np.random.default_rng(5))
    t = {k: (dict(v) if isinstance(v, dict) else v) for k, v in tm.items()}
    for k, v in t.items():
        if isinstance(v, dict):
            v["vary"] = k in ("norm", "ph_2")
    return x, 5000 / tm["norm"]["value"], t


def test_readvaryparam_brute_lattice_changes_the_optimum(gpu):
    from crimp_amd.toafit_vary import VaryParamFitter
    x, E, t = _case()
    off = np.array([0, x.size], dtype=np.int64)
    rb = VaryParamFitter(x, off, np.array([E]), t).fit(brutemin=True)
    rn = VaryParamFitter(x, off, np.array([E]), t).fit(brutemin=False)
    o = O.fit_toa_readvary(x, E, t, brutemin=True)
    # the lattice start leads to the oracle's optimum ...
    assert abs(rb["phShi"][0] - o["phShi"]) / (2 * math.pi) < 1e-6, (rb["phShi"][0], o["phShi"])
    assert rb["LLmax"][0] == pytest.approx(o["LLmax"], abs=1e-6)
    assert rb["phShi_LL"][0] == o["phShi_LL"] and rb["phShi_UL"][0] == o["phShi_UL"]
    # ... which is not the one the template start reaches (a different, lower local maximum)
    assert abs(rn["phShi"][0] - rb["phShi"][0]) > 1.0
    assert rn["LLmax"][0] < rb["LLmax"][0] - 1.0


def test_readvaryparam_brute_start_equals_oracle_lattice(gpu):
    """The lattice argmax itself (before the local maximisation): the device's fp32 grid and the oracle's fp64
    lattice pick the same point."""
    from crimp_amd.toafit_vary import VaryParamFitter
    x, E, t = _case()
    f = VaryParamFitter(x, np.array([0, x.size], dtype=np.int64), np.array([E]), t)
    st = f.brute_lattice()
    th, _ = O.readvary_brute(x, E, t)
    np.testing.assert_allclose(st[0], th, rtol=0, atol=1e-12)

"""HIP path (through the C-ABI) against the oracle and the reference's golden vectors.

Tolerances (BASELINE.json north_star): Z^2/H powers within 1e-6 relative PER TRIAL (plain relative error,
no scale floor: ``close_rel``) for the default search path (the NUFFT where it applies, else the exact rule),
precision="exact" (exact-integer i8 MFMA kernel, fp64 kernel on other grids) and the fp64 path; best-trial index
bit-exact; ToA phase shifts within 1e-4 cycles; calcphase within 1e-9 cycles; LL within 1e-9 relative (fp64
kernel). NUFFT internals (raw powers, plans, row shards): tests/test_gpu_nufft.py.
"""
import json
import math

import numpy as np
import pandas as pd
import pytest

from conftest import gold, gpath
from oracle import oracle as O

pytestmark = pytest.mark.gpu
RTOL = 1e-6


def close_rel(got, ref, rtol=RTOL):
    """Plain per-trial relative error (no scale floor): the default and fp64 paths' contract."""
    got, ref = np.asarray(got), np.asarray(ref)
    err = np.abs(got - ref) / np.abs(ref)
    assert err.max() <= rtol, "max relative error %.3g at %d" % (err.max(), int(err.argmax()))
    return err.max()


@pytest.mark.parametrize("precision,path", [(None, 2), ("exact", 1)])
def test_z2_h_config1_golden(gpu, precision, path):
    """Config 1 through the reference's own call, PeriodSearch(time, freq, m).ztest() / .htest() / .twod_ztest(): the
    default reaches the NUFFT (crimp_last_search_path() == 2) on the 400-trial progression of the 1E 2259 events;
    precision="exact" the exact kernel (20 launches for H_20)."""
    from crimp_amd.periodsearch import PeriodSearch
    from crimp_amd import _native as N
    g = gold("periodsearch_1e2259.npz")
    z = PeriodSearch(g["time"], g["freq"], 2, precision=precision).ztest()
    assert N.load().crimp_last_search_path() == path
    assert int(np.argmax(z)) == 200
    close_rel(z, g["z2_m2"])
    h = PeriodSearch(g["time"], g["freq"], 20, precision=precision).htest()
    assert N.load().crimp_last_search_path() == path
    assert int(np.argmax(h)) == 200
    close_rel(h, g["h_m20"])
    arr, df = PeriodSearch(g["time"], g["fsub"], 2, precision=precision).twod_ztest(g["fd"])
    np.testing.assert_array_equal(arr[:, :2], g["z2d_m2"][:, :2])
    close_rel(arr[:, 2], g["z2d_m2"][:, 2])
    assert list(df.columns) == ["Freq", "Freq_dot", "Z2pow"]


@pytest.mark.parametrize("precision", [None, "exact"])
def test_search_synthetic_golden_and_edges(gpu, precision):
    from crimp_amd.periodsearch import PeriodSearch
    g = gold("periodsearch_synth.npz")
    t, f = g["time"], g["freq"]
    P = precision
    for m in (1, 2, 3, 5):
        z = PeriodSearch(t, f, m, precision=P).ztest()
        close_rel(z, g["z_m%d" % m])
        assert np.argmax(z) == np.argmax(g["z_m%d" % m])
    for m in (1, 5, 20):
        close_rel(PeriodSearch(t, f, m, precision=P).htest(), g["h_m%d" % m])
    close_rel(PeriodSearch(t, f[64:128], 2, precision=P).twod_ztest(g["fd"])[0][:, 2], g["z2d_m2"][:, 2])
    close_rel(PeriodSearch(t, f[64:128], 3, precision=P).twod_ztest(g["fd"])[0][:, 2], g["z2d_m3"][:, 2])
    close_rel(PeriodSearch(g["time_perm"], g["freq_nu"], 2, precision=P).ztest(), g["z_nonuniform_m2"])
    close_rel(PeriodSearch(g["time_perm"], g["freq_nu"], 4, precision=P).htest(), g["h_nonuniform_m4"])
    close_rel(PeriodSearch(t[:1], f[:8], 2, precision=P).ztest(), g["z_n1"])
    close_rel(PeriodSearch(t[:2], f[:8], 2, precision=P).ztest(), g["z_n2"])
    close_rel(PeriodSearch(t[:2], f[:8], 3, precision=P).htest(), g["h_n2"])
    close_rel(PeriodSearch(t, f[100:101], 2, precision=P).ztest(), g["z_m1trial"])
    assert PeriodSearch(t, f[:0], 2, precision=P).ztest().size == 0
    with pytest.raises(IndexError):
        PeriodSearch(t[:0], f, 2, precision=P)


@pytest.mark.parametrize("mode", ["default", "exact", "f64", "nufft"])
def test_search_vs_oracle_larger(gpu, mode):
    """Every search path on 2e5 photons x 2048 trials (Z^2_2) and a 3 x 1024 2-D grid (H_3): per trial within 1e-6
    relative; best trial exact."""
    from crimp_amd.periodsearch import PeriodSearch
    from crimp_amd.synth import pulsed_events
    from crimp_amd import _native as N
    prec = {"default": None, "exact": "exact", "f64": "f64", "nufft": "nufft"}[mode]
    check = close_rel
    t = pulsed_events(200000, 2.0e5, 7.123456789, pulsed_frac=0.05, seed=4)
    f = 7.123456789 + (np.arange(-1024, 1024) / (10 * 2.0e5))
    z = PeriodSearch(t, f, 2, precision=prec).ztest()
    zr = O.search(t, f, 2)
    assert int(np.argmax(z)) == int(np.argmax(zr))
    check(z, zr)
    fd = np.array([-13.0, -12.0, -11.5])
    a = PeriodSearch(t, f[512:1536], 3, precision=prec).twod_htest(fd)[0][:, 2]
    ar = O.search(t, f[512:1536], 3, freq_dot=fd, stat="h")
    assert int(np.argmax(a)) == int(np.argmax(ar))
    check(a, ar)
    assert N.load().crimp_last_search_path() == {"default": 2, "exact": 1, "f64": 0, "nufft": 2}[mode]


def test_search_f64_strict_relative_vs_reference_goldens(gpu):
    """precision='f64' (k_search_f64): every trial, near-zero noise bins included, within 1e-8 relative of
    the reference's own NumPy outputs (periodsearch.py:57-125 run here, tests/golden/gen_golden.py)."""
    from crimp_amd.periodsearch import PeriodSearch
    g = gold("periodsearch_1e2259.npz")
    z = PeriodSearch(g["time"], g["freq"], 2, precision="f64").ztest()
    assert int(np.argmax(z)) == 200
    close_rel(z, g["z2_m2"], 1e-8)
    h = PeriodSearch(g["time"], g["freq"], 20, precision="f64").htest()
    assert int(np.argmax(h)) == 200
    close_rel(h, g["h_m20"], 1e-8)
    arr, _ = PeriodSearch(g["time"], g["fsub"], 2, precision="f64").twod_ztest(g["fd"])
    close_rel(arr[:, 2], g["z2d_m2"][:, 2], 1e-8)
    s = gold("periodsearch_synth.npz")
    for m in (1, 2, 3, 5):
        close_rel(PeriodSearch(s["time"], s["freq"], m, precision="f64").ztest(), s["z_m%d" % m], 1e-8)
    for m in (1, 5, 20):
        close_rel(PeriodSearch(s["time"], s["freq"], m, precision="f64").htest(), s["h_m%d" % m], 1e-8)
    close_rel(PeriodSearch(s["time"], s["freq"][64:128], 3, precision="f64").twod_ztest(s["fd"])[0][:, 2],
              s["z2d_m3"][:, 2], 1e-8)
    close_rel(PeriodSearch(s["time_perm"], s["freq_nu"], 4, precision="f64").htest(), s["h_nonuniform_m4"], 1e-8)
    close_rel(PeriodSearch(s["time"][:2], s["freq"][:8], 3, precision="f64").htest(), s["h_n2"], 1e-8)


def test_search_f64_larger_vs_oracle(gpu):
    """fp64 path vs the fp64 oracle on 2e5 photons x 2048 trials (Z^2_2 and H_20): 1e-7 relative per trial,
    no scale floor (a NumPy model of the kernel's arithmetic reaches 4e-9 / 2.2e-8 here: the two fp64 phase
    constructions differ by ~1e-10 cycles per photon at 1.4e6 cycles, which a near-zero bin amplifies)."""
    from crimp_amd.periodsearch import PeriodSearch
    from crimp_amd.synth import pulsed_events
    t = pulsed_events(200000, 2.0e5, 7.123456789, pulsed_frac=0.05, seed=4)
    f = 7.123456789 + (np.arange(-1024, 1024) / (10 * 2.0e5))
    close_rel(PeriodSearch(t, f, 2, precision="f64").ztest(), O.search(t, f, 2), 1e-7)
    hr = O.search(t, f[:256], 20, stat="h")
    close_rel(PeriodSearch(t, f[:256], 20, precision="f64").htest(), hr, 1e-7)
    with pytest.raises(ValueError):
        PeriodSearch(t, f, 2, precision="f16").ztest()
    with pytest.raises(ValueError):  # the fp32 fast path was retired (round 5)
        PeriodSearch(t, f, 2, precision="fast").ztest()


def test_search_sharded_ranges_equal_full(gpu):
    """precision="exact": a search split into flat-trial ranges (what each rank computes) equals the unsplit search
    bit for bit (integer totals); the default (NUFFT) split at row edges is bit-identical too, a cut row agrees within
    its plans' error."""
    from crimp_amd import ops
    from crimp_amd.synth import pulsed_events
    t = pulsed_events(50000, 1.0e5, 3.0, pulsed_frac=0.1, seed=9)
    f = 3.0 + np.arange(-300, 300) / 1.0e6
    fd = np.array([-12.0, -11.0])
    t0 = (t[0] + t[-1]) / 2
    from crimp_amd import _native as N
    full = ops.search(t, t0, f, 2, 0, log10_negfdot=fd, precision="exact")
    # the exact kernel, not its fp64 fix-up, must produce these (a broken exact kernel is hidden by a fix-up of
    # every trial; at 5e4 photons and powers ~1 the error bound flags none)
    assert N.load().crimp_last_fixups() <= 12
    parts = [ops.search(t, t0, f, 2, 0, log10_negfdot=fd, first=a, count=b - a, precision="exact")
             for a, b in ((0, 333), (333, 901), (901, 1200))]
    np.testing.assert_array_equal(np.concatenate(parts), full)
    dfull = ops.search(t, t0, f, 2, 0, log10_negfdot=fd)
    assert N.load().crimp_last_search_path() == 2
    drows = [ops.search(t, t0, f, 2, 0, log10_negfdot=fd, first=a, count=600) for a in (0, 600)]
    np.testing.assert_array_equal(np.concatenate(drows), dfull)
    dparts = [ops.search(t, t0, f, 2, 0, log10_negfdot=fd, first=a, count=b - a)
              for a, b in ((0, 333), (333, 901), (901, 1200))]
    close_rel(np.concatenate(dparts), dfull, 1e-6)
    close_rel(dfull, full, 1e-6)
    for twod in (None, fd):  # raw exact-kernel powers (fix-up off) within the kernel's error model of fp64
        ref = ops.search(t, t0, f, 2, 0, log10_negfdot=twod, precision="f64")
        z = ops.search(t, t0, f, 2, 0, log10_negfdot=twod, flags=N.FLAG_NO_FIXUP, precision="exact")
        close_rel(z, ref, 1e-6)


def test_calcphase_golden(gpu):
    from crimp_amd.calcphase import calcphase, Phases
    g = gold("calcphase.npz")
    tot, fol = calcphase(g["t"], gpath("1e2259.par"))
    assert np.max(np.abs(tot - g["total_par"])) <= 1e-9
    d = np.abs(fol - g["folded_par"])
    assert np.max(np.minimum(d, 1 - d)) <= 1e-9
    tm = json.load(open(gpath("timing_model_dict.json")))
    tot, fol = calcphase(g["t"], tm)
    assert np.max(np.abs(tot - g["total_dict"])) <= 1e-9
    ts, fs = calcphase(float(g["t_scalar"]), gpath("1e2259.par"))
    assert isinstance(ts, float) and abs(ts - float(g["total_scalar"])) <= 1e-9
    t2, f2 = calcphase(g["t2d"], tm)
    assert t2.shape == (20, 30) and np.max(np.abs(t2 - g["total_2d"])) <= 1e-9
    ph = Phases(g["t"][:100], tm)
    te, gl, wv = ph.taylorexpansion(), ph.glitches(), ph.waves()
    np.testing.assert_allclose(te + gl + wv, g["total_dict"][:100], rtol=0, atol=1e-9)
    with pytest.raises(TypeError):
        Phases(g["t"], 3.0)


def test_fourier_ll_golden_points(gpu):
    from crimp_amd.templatemodels import Fourier
    g = gold("toa_1e2259.npz")
    iv = pd.read_csv(gpath("timIntToAs_1e2259.txt"), sep=r"\s+", comment="#")
    tm = json.load(open(gpath("parsed.json")))["template"]
    for k in range(g["ll_val"].size):
        i = int(np.nonzero(g["ids"] == g["ll_toa"][k])[0][0])
        x = g["folded"][g["offsets"][i]:g["offsets"][i + 1]]
        th = {"norm": g["ll_norm"][k], "ampShift": 1.0, "phShift": g["ll_phi"][k]}
        for j in range(1, 7):
            th["amp_%d" % j] = tm["amp_%d" % j]["value"]
            th["ph_%d" % j] = tm["ph_%d" % j]["value"]
        ll = Fourier(th, x).loglikelihoodFSnormalized(float(iv["ToA_exposure"][g["ll_toa"][k]]))
        assert abs(ll - g["ll_val"][k]) <= 1e-9 * abs(g["ll_val"][k])
    th["norm"], th["phShift"] = 0.5, 0.0
    assert Fourier(th, g["folded"][:g["offsets"][1]]).loglikelihoodFSnormalized(600.0) == -np.inf


def test_cauchy_vonmises_ll_golden(gpu):
    from crimp_amd.templatemodels import WrappedCauchy, VonMises
    g = gold("templatemodels.npz")
    tc = json.load(open(gpath("cauchy_vm_theta.json")))
    i = 0
    for p in (-4.0, -0.5, 0.3, 2.2):
        for nv in (3.0, 5.0, 8.0):
            th = dict(tc, phShift=p, norm=nv)
            assert abs(WrappedCauchy(th, g["x"]).loglikelihoodCAnormalized(250.0) - g["cauchy"][i]) <= 1e-9 * abs(
                g["cauchy"][i])
            assert abs(VonMises(th, g["x"]).loglikelihoodVMnormalized(250.0) - g["vonmises"][i]) <= 1e-9 * abs(
                g["vonmises"][i])
            i += 1


def test_toa_points_derivatives_vs_oracle(gpu):
    from crimp_amd import ops
    g = gold("templatemodels.npz")
    tc = json.load(open(gpath("cauchy_vm_theta.json")))
    x = g["x"]
    for model in ("cauchy", "vonmises"):
        tarr = O.template_arrays(dict(tc, model=model))
        tpl = ops.make_template(model, tarr[2], tarr[3], tarr[4])
        s = ops.toa_points(x, np.array([0, x.size]), tpl, np.zeros(3, np.int64), np.array([4.0, 5.0, 6.0]),
                           np.array([0.1, -1.0, 2.0]))
        for p, (nv, ph) in enumerate(((4.0, 0.1), (5.0, -1.0), (6.0, 2.0))):
            o = O.toa_eval(x, 250.0, tarr, nv, ph)
            np.testing.assert_allclose([s[p, 1] - 250.0, s[p, 2], s[p, 3], s[p, 4], s[p, 5]], o[1:6], rtol=1e-9)


def test_brute_grid_vs_oracle(gpu):
    from crimp_amd import ops
    g = gold("toa_1e2259.npz")
    tm = json.load(open(gpath("parsed.json")))["template"]
    tarr = O.template_arrays(tm)
    tpl = ops.make_template("fourier", tarr[2], tarr[3])
    x, off = g["folded"], g["offsets"]
    norms = np.linspace(0.17, 500, 20)
    phis = np.arange(126) * 0.05 - np.pi
    ln, hmin = ops.toa_grid(x, off, tpl, np.tile(norms, (off.size - 1, 1)), phis)
    for i in (0, 6):
        xi = x[off[i]:off[i + 1]]
        E = 600.0
        ref = O.toa_grid(xi, E, tarr, norms, phis)
        N = xi.size
        got = -norms[:, None] * E + N * np.log(norms[:, None] * E) + ln[i] - N * np.log(norms[:, None])
        got = np.where(hmin[i][None, :] + norms[:, None] > 0, got, -np.inf)
        fin = np.isfinite(ref)
        assert np.array_equal(fin, np.isfinite(got))
        np.testing.assert_allclose(got[fin], ref[fin], rtol=2e-7, atol=0.05)
        assert np.unravel_index(np.argmax(got), got.shape) == np.unravel_index(np.argmax(ref), ref.shape)


def test_binphases_device_counts(gpu):
    from crimp_amd import ops
    g = gold("toa_1e2259.npz")
    x, off = g["folded"], g["offsets"]
    edges = np.linspace(0, 1, 16)
    c = ops.binphases_counts(x, off, edges)
    for i in range(off.size - 1):
        assert np.array_equal(c[i], np.histogram(x[off[i]:off[i + 1]], bins=edges)[0])
    assert np.array_equal(c[0], g["bp_cts"])


def test_binphases_split_blocks_ragged(gpu):
    """Photon splits per interval (several blocks add into one interval's counts): ragged intervals from 1 to 3e5
    photons, values outside the edges and on them, 1 to 256 bins (16 and 17: both sides of the packed per-thread
    counters), [0, 1] and [0, 2 pi] (the Cauchy / von Mises phases), host and device inputs -- np.histogram exactly."""
    import torch
    from crimp_amd import ops
    rng = np.random.default_rng(17)
    sizes = np.array([1, 7, 300000, 4096, 4097, 123457, 2, 65536])
    u = rng.uniform(-0.1, 1.1, sizes.sum())
    off = np.concatenate([[0], np.cumsum(sizes)])
    for nb, upper in ((1, 1.0), (15, 1.0), (16, 1.0), (17, 1.0), (15, 2 * np.pi), (256, 1.0)):
        edges = np.linspace(0, upper, nb + 1)
        x = u * upper
        x[::97] = edges[rng.integers(0, nb + 1, x[::97].size)]  # on bin edges, the last one included
        e = edges[rng.integers(0, nb + 1, x[1::89].size)]  # one ulp either side of an edge
        x[1::89] = np.nextafter(e, np.where(rng.random(e.size) < 0.5, -np.inf, np.inf))
        ref = np.stack([np.histogram(x[off[i]:off[i + 1]], bins=edges)[0] for i in range(sizes.size)])
        assert np.array_equal(ops.binphases_counts(x, off, edges), ref)
        got = ops.binphases_counts(torch.tensor(x, device="cuda"), torch.tensor(off, device="cuda"),
                                   torch.tensor(edges, device="cuda"))
        assert np.array_equal(got.cpu().numpy(), ref)


def _golden_rows():
    g = gold("toa_1e2259.npz")
    iv = pd.read_csv(gpath("timIntToAs_1e2259.txt"), sep=r"\s+", comment="#")
    ref = pd.read_csv(gpath("ToAs_2259.txt"), sep=r"\s+", comment="#")
    return g, iv, ref


def test_toa_fits_match_reference_and_oracle(gpu):
    """Config 2: ToAs 35-41 of the worked example, batched on the device."""
    from crimp_amd.toafit import ToAFitter
    from crimp_amd.readPPtemplate import readPPtemplate
    g, iv, ref = _golden_rows()
    tm = readPPtemplate(gpath("1e2259_template.txt"))
    E = iv["ToA_exposure"].to_numpy()[g["ids"]]
    r = ToAFitter(g["folded"], g["offsets"], E, tm).fit(brutemin=True)
    for i, tid in enumerate(g["ids"]):
        row = ref[ref["ToA"] == tid].iloc[0]
        x = g["folded"][g["offsets"][i]:g["offsets"][i + 1]]
        o = O.fit_toa(x, E[i], tm, brutemin=True)
        assert abs(r["phShi"][i] - row["phShift"]) / (2 * math.pi) < 1e-4
        assert abs(r["phShi"][i] - o["phShi"]) / (2 * math.pi) < 1e-6
        assert r["phShi_LL"][i] == pytest.approx(row["phShift_LL"], abs=1e-12)
        assert r["phShi_UL"][i] == pytest.approx(row["phShift_UL"], abs=1e-12)
        assert r["reducedChi2"][i] == pytest.approx(row["redChi2"], rel=5e-4)
        assert r["reducedChi2"][i] == pytest.approx(o["reducedChi2"], rel=1e-6)


@pytest.mark.parametrize("model", ["fourier", "cauchy"])
def test_toa_fit_redchi2_fused_equals_separate(gpu, model):
    """crimp_toa_fit_redchi2 (histogram on a second stream beside the grid and the fits; timed: after them) returns
    exactly crimp_toa_fit's records and crimp_toa_redchi2's values, host and device buffers, with and without the
    brute start and varyAmps."""
    import torch
    from crimp_amd import ops, _native as N
    from crimp_amd.toafit import ToAFitter
    from crimp_amd.readPPtemplate import readPPtemplate
    g, iv, _ = _golden_rows()
    if model == "fourier":
        tm, x, off = readPPtemplate(gpath("1e2259_template.txt")), g["folded"], g["offsets"]
        E = iv["ToA_exposure"].to_numpy()[g["ids"]]
    else:  # the Cauchy template and phases of the LL goldens, split into two intervals
        tc = json.load(open(gpath("cauchy_vm_theta.json")))
        tm = {"model": "cauchy", "norm": {"value": 5.0, "vary": True}}
        for j in (1, 2):
            for nm in ("amp", "cen", "wid"):
                tm["%s_%d" % (nm, j)] = {"value": tc["%s_%d" % (nm, j)], "vary": True}
        x = gold("templatemodels.npz")["x"]
        off = np.array([0, x.size // 2, x.size], dtype=np.int64)
        E = np.array([125.0, 125.0])
    for dev in (False, True):
        xs = torch.tensor(x, device=gpu) if dev else x
        os_ = torch.tensor(off, device=gpu) if dev else off
        f = ToAFitter(xs, os_, E, tm)
        edges, pp = f._bins()
        for brute, va in ((True, False), (False, False), (True, True)):
            for flags in (0, N.FLAG_TIME_KERNELS):
                rec, red = ops.toa_fit_redchi2(f.x, f.offsets, f.tpl, f._arr(f.E, np.float64), f.norm0, f.res, brute,
                                               va, f._arr(edges, np.float64), f._arr(pp, np.float64), 3 if va else 2,
                                               flags=flags)
                rec2 = ops.toa_fit(f.x, f.offsets, f.tpl, f._arr(f.E, np.float64), f.norm0, f.res, brute, va)
                red2 = ops.toa_redchi2(f.x, f.offsets, f.tpl, f._arr(f.E, np.float64), rec2,
                                       f._arr(edges, np.float64), f._arr(pp, np.float64), 3 if va else 2)
                h = [np.asarray(v.cpu().numpy() if hasattr(v, "cpu") else v) for v in (rec, red, rec2, red2)]
                np.testing.assert_array_equal(h[0], h[2])
                np.testing.assert_array_equal(h[1], h[3])


def test_device_toa_driver_equals_host_driver(gpu):
    """crimp_toa_fit (one workgroup per interval runs the whole fit) against the host-driven iterations."""
    from crimp_amd.toafit import ToAFitter
    from crimp_amd.readPPtemplate import readPPtemplate
    g, iv, ref = _golden_rows()
    tm = readPPtemplate(gpath("1e2259_template.txt"))
    E = iv["ToA_exposure"].to_numpy()[g["ids"]]
    for bm in (True, False):
        f = ToAFitter(g["folded"], g["offsets"], E, tm)
        d, h = f.fit(brutemin=bm), f.fit_host(brutemin=bm)
        np.testing.assert_allclose(d["phShi"], h["phShi"], rtol=0, atol=1e-9)
        np.testing.assert_array_equal(d["phShi_LL"], h["phShi_LL"])
        np.testing.assert_array_equal(d["phShi_UL"], h["phShi_UL"])
        np.testing.assert_allclose(d["LLmax"], h["LLmax"], rtol=1e-12)
        assert np.all(d["evaluations"] > 5)
    tc = json.load(open(gpath("cauchy_vm_theta.json")))
    gx = gold("templatemodels.npz")["x"]
    for model in ("cauchy", "vonmises"):
        t = {"model": model, "norm": {"value": 5.0, "vary": True}}
        for j in (1, 2):
            for nm in ("amp", "cen", "wid"):
                t["%s_%d" % (nm, j)] = {"value": tc["%s_%d" % (nm, j)], "vary": True}
        f = ToAFitter(gx, np.array([0, gx.size]), np.array([250.0]), t)
        d, h = f.fit(brutemin=True), f.fit_host(brutemin=True)
        np.testing.assert_allclose(d["phShi"], h["phShi"], rtol=0, atol=1e-9)
        np.testing.assert_array_equal(d["phShi_LL"], h["phShi_LL"])
        np.testing.assert_array_equal(d["phShi_UL"], h["phShi_UL"])


def test_moment_norm_profiles_equal_iterative(gpu, monkeypatch):
    """The 1-sigma scan's one-pass moment profiles (fit_profile_mom) against the iterative 1-D Newton profiles
    (CRIMP_FIT_MOM_R=0 forces them on every scan step, as the host-driven toafit.profile_norm runs): identical
    phShift, LLmax and 1-sigma bounds on the worked example (Fourier) and on the Cauchy / von Mises blocks, and
    more likelihood passes on the iterative side."""
    from crimp_amd.toafit import ToAFitter
    from crimp_amd.readPPtemplate import readPPtemplate
    g, iv, ref = _golden_rows()
    tm = readPPtemplate(gpath("1e2259_template.txt"))
    E = iv["ToA_exposure"].to_numpy()[g["ids"]]
    cases = [(g["folded"], g["offsets"], E, tm)]
    tc = json.load(open(gpath("cauchy_vm_theta.json")))
    gx = gold("templatemodels.npz")["x"]
    for model in ("cauchy", "vonmises"):
        t = {"model": model, "norm": {"value": 5.0, "vary": True}}
        for j in (1, 2):
            for nm in ("amp", "cen", "wid"):
                t["%s_%d" % (nm, j)] = {"value": tc["%s_%d" % (nm, j)], "vary": True}
        cases.append((gx, np.array([0, gx.size]), np.array([250.0]), t))
    for x, off, e, t in cases:
        monkeypatch.delenv("CRIMP_FIT_MOM_R", raising=False)
        m = ToAFitter(x, off, e, t).fit(brutemin=True)
        monkeypatch.setenv("CRIMP_FIT_MOM_R", "0")
        it = ToAFitter(x, off, e, t).fit(brutemin=True)
        np.testing.assert_array_equal(m["phShi"], it["phShi"])
        np.testing.assert_array_equal(m["LLmax"], it["LLmax"])
        np.testing.assert_array_equal(m["phShi_LL"], it["phShi_LL"])
        np.testing.assert_array_equal(m["phShi_UL"], it["phShi_UL"])
        assert np.all(it["evaluations"] > m["evaluations"])


def test_toa_fit_vary_amps_vs_oracle(gpu):
    """varyAmps (measureToAs.py:305-312): ampShift free in [0.01, 100]. No reference output exercises it
    (parity unpinned); checked against the oracle's optimum restatement."""
    from crimp_amd.measureToAs import measureToA_fourier
    from crimp_amd.toafit import ToAFitter
    from crimp_amd.readPPtemplate import readPPtemplate
    g, iv, ref = _golden_rows()
    tm = readPPtemplate(gpath("1e2259_template.txt"))
    E = iv["ToA_exposure"].to_numpy()[g["ids"]]
    r = ToAFitter(g["folded"], g["offsets"], E, tm).fit(brutemin=True, vary_amps=True)
    for i in (2,):  # the oracle's nested optimisation takes ~15 s per ToA on the host
        x = g["folded"][g["offsets"][i]:g["offsets"][i + 1]]
        o = O.fit_toa_vary_amps(x, E[i], tm, brutemin=True)
        assert abs(r["phShi"][i] - o["phShi"]) / (2 * math.pi) < 1e-6
        assert r["ampShift"][i] == pytest.approx(o["ampShift"], rel=1e-5)
        assert r["LLmax"][i] == pytest.approx(o["LLmax"], abs=1e-6)
        assert r["phShi_LL"][i] == o["phShi_LL"] and r["phShi_UL"][i] == o["phShi_UL"]
        assert r["reducedChi2"][i] == pytest.approx(o["reducedChi2"], rel=1e-5)
    s = measureToA_fourier(tm, g["folded"][g["offsets"][2]:g["offsets"][3]], E[2], brutemin=True, varyAmps=True)
    assert s["phShi"] == pytest.approx(r["phShi"][2], abs=1e-12)


def test_toa_fit_without_brute_and_other_templates(gpu):
    from crimp_amd.measureToAs import measureToA_fourier, measureToA_cauchy, measureToA_vonmises
    from crimp_amd.readPPtemplate import readPPtemplate
    g, iv, ref = _golden_rows()
    tm = readPPtemplate(gpath("1e2259_template.txt"))
    x = g["folded"][g["offsets"][2]:g["offsets"][3]]
    E = float(iv["ToA_exposure"][37])
    r = measureToA_fourier(tm, x, E)
    o = O.fit_toa(x, E, tm, brutemin=False)
    assert abs(r["phShi"] - o["phShi"]) / (2 * math.pi) < 1e-6
    assert r["phShi_LL"] == o["phShi_LL"] and r["phShi_UL"] == o["phShi_UL"]
    tc = json.load(open(gpath("cauchy_vm_theta.json")))
    gx = gold("templatemodels.npz")["x"]
    for fn, model in ((measureToA_cauchy, "cauchy"), (measureToA_vonmises, "vonmises")):
        t = {"model": model, "norm": {"value": 5.0, "vary": True}}
        for j in (1, 2):
            for nm in ("amp", "cen", "wid"):
                t["%s_%d" % (nm, j)] = {"value": tc["%s_%d" % (nm, j)], "vary": True}
        r = fn(t, gx, 250.0, brutemin=True)
        o = O.fit_toa(gx, 250.0, t, brutemin=True)
        assert abs(r["phShi"] - o["phShi"]) / (2 * math.pi) < 1e-6, model
        assert r["phShi_LL"] == o["phShi_LL"] and r["phShi_UL"] == o["phShi_UL"], model


def test_measuretoas_end_to_end(gpu, tmp_path):
    """measureToAs on a FITS file written from the bundled events: the golden table rows 35-41."""
    from crimp_amd.eventfile import write_events_fits
    from crimp_amd.measureToAs import measureToAs
    ev = gold("events_1e2259.npz")
    p = str(tmp_path / "ev.fits")
    write_events_fits(p, ev["TIME"], ev["PI"], int(ev["MJDREFI"]), float(ev["MJDREFF"]))
    out = str(tmp_path / "ToAs")
    tab = measureToAs(p, gpath("1e2259.par"), gpath("1e2259_template.txt"), gpath("timIntToAs_1e2259.txt"),
                      eneLow=1, eneHigh=5, toaStart=35, toaEnd=41, brutemin=True, toaFile=out)
    ref = pd.read_csv(gpath("ToAs_2259.txt"), sep=r"\s+", comment="#")
    ref = ref[(ref["ToA"] >= 35) & (ref["ToA"] <= 41)].reset_index(drop=True)
    assert list(tab.columns) == list(ref.columns)
    for c in ("ToA", "ToA_mid", "ToA_start", "ToA_end", "ToA_lenInt", "ToA_exp", "nbr_events", "count_rate",
              "phShift_LL", "phShift_UL"):
        np.testing.assert_array_equal(tab[c].to_numpy(), ref[c].to_numpy(), err_msg=c)
    assert np.all(np.abs(tab["phShift"] - ref["phShift"]) / (2 * np.pi) < 1e-4)
    g = gold("toa_1e2259.npz")
    np.testing.assert_allclose(tab["Hpower"].to_numpy(), g["h5"], rtol=1e-6)
    lines = open(out + ".txt").read().splitlines()
    assert lines[0] == open(gpath("ToAs_2259.txt")).read().splitlines()[0]


def test_measure_intervals_slice_gather_and_pinned_source(gpu):
    """measure_intervals: consecutive intervals (their photons one slice of the time array, no gather), a page-locked
    torch source (DMA from it), and the same intervals with photons left between two of them (the gather path) give
    identical records for every interval the change does not touch (each interval's fit and H test are independent
    of its batch)."""
    import torch
    from bench import T2259, _tmpl
    from crimp_amd.measureToAs import measure_intervals
    from crimp_amd.synth import template_intervals_torch
    x, off, E, _ = template_intervals_torch(6, 20000, T2259["norm"]["value"], T2259["amp"], T2259["ph"], seed=4,
                                            device=gpu)
    F0, pep = 0.5, 58000.0
    mjd = (pep + ((torch.arange(x.numel(), device=gpu, dtype=torch.float64) + x) / F0) / 86400.0).cpu().numpy()
    offh = off.cpu().numpy()
    starts, ends = mjd[offh[:-1]] - 1e-9, mjd[offh[1:] - 1] + 1e-9
    par = {"PEPOCH": pep, "F0": F0}
    tm = _tmpl()
    a = measure_intervals(mjd, par, tm, starts, ends, E, brutemin=True)
    b = measure_intervals(torch.from_numpy(mjd).pin_memory(), par, tm, starts, ends, E, brutemin=True)
    ends2 = ends.copy()
    ends2[2] = mjd[offh[3] - 11] + 1e-9  # interval 2 loses its last 10 photons: they sit between intervals 2 and 3
    c = measure_intervals(mjd, par, tm, starts, ends2, E, brutemin=True)
    keep = np.array([0, 1, 3, 4, 5])
    for k in a:
        va, vb, vc = (np.asarray(r[k]) for r in (a, b, c))
        np.testing.assert_array_equal(va, vb, err_msg=k)
        np.testing.assert_array_equal(va[keep], vc[keep], err_msg=k)
    assert not np.array_equal(np.asarray(a["phShi"])[2], np.asarray(c["phShi"])[2])


def test_measure_intervals_blocks_equal_one_shot(gpu, monkeypatch):
    """The pipelined measure_intervals (host times cut into shrinking blocks, block k + 1 uploaded by a second thread
    while block k is fitted) against the one-shot call: consecutive intervals, a gap
    (gather inside a block), a page-locked source, and unsorted times (detected on the device: the call falls back
    to the one-shot path's host mask). The brute grid's kernel choice is per call, so phShift is held to the
    fast-vs-full grid tolerance (1e-9 rad) and everything else to equality."""
    import torch
    from bench import T2259, _tmpl
    from crimp_amd.measureToAs import measure_intervals
    from crimp_amd.synth import template_intervals_torch
    x, off, E, _ = template_intervals_torch(6, 20000, T2259["norm"]["value"], T2259["amp"], T2259["ph"], seed=5,
                                            device=gpu)
    F0, pep = 0.5, 58000.0
    mjd = (pep + ((torch.arange(x.numel(), device=gpu, dtype=torch.float64) + x) / F0) / 86400.0).cpu().numpy()
    offh = off.cpu().numpy()
    starts, ends = mjd[offh[:-1]] - 1e-9, mjd[offh[1:] - 1] + 1e-9
    ends_gap = ends.copy()
    ends_gap[2] = mjd[offh[3] - 11] + 1e-9
    par = {"PEPOCH": pep, "F0": F0}
    tm = _tmpl()

    def same(a, b):
        for k in a:
            va, vb = np.asarray(a[k]), np.asarray(b[k])
            if k == "phShi":
                np.testing.assert_allclose(va, vb, rtol=0, atol=1e-9)
            else:
                np.testing.assert_array_equal(va, vb, err_msg=k)

    unsorted = mjd.copy()
    unsorted[offh[4] + 5], unsorted[offh[4] + 6] = mjd[offh[4] + 6], mjd[offh[4] + 5]
    # an out-of-order photon that no block uploads (after the last interval) whose time lies inside interval 1: the
    # reference's mask counts it; the host gap check sends the call to the one-shot path, which does too
    ends_tail = ends.copy()
    ends_tail[-1] = mjd[offh[-1] - 30] + 1e-9
    stray = mjd.copy()
    stray[offh[-1] - 5] = mjd[offh[1] + 100] + 1e-10
    perm = np.array([2, 0, 5, 1, 4, 3])  # intervals out of start order (the block's upload starts at its min lo)
    cases = ((mjd, starts, ends, E), (mjd, starts, ends_gap, E), (torch.from_numpy(mjd).pin_memory(), starts, ends, E),
             (unsorted, starts, ends, E), (mjd, starts[perm], ends[perm], np.asarray(E)[perm]),
             (stray, starts, ends_tail, E))
    for src, st, en, ex in cases:
        monkeypatch.setenv("CRIMP_E2E_MIN_PHOTONS", str(1 << 40))
        one = measure_intervals(src, par, tm, st, en, ex, brutemin=True)
        monkeypatch.setenv("CRIMP_E2E_MIN_PHOTONS", "1000")  # blocks of 3, 2 and 1 intervals
        same(one, measure_intervals(src, par, tm, st, en, ex, brutemin=True))


def test_measuretoas_rows_before_empty_interval(gpu, tmp_path, monkeypatch):
    """An interval without photons at position k: the reference's loop has written rows < k when
    TIME_toa[-1] raises (measureToAs.py:160-162, :182, :222-226). The drop-in writes them too (here in batches of
    one interval, CRIMP_TOA_BATCH_PHOTONS=1, so every row is flushed as soon as its fit is known), then raises the
    IndexError; the rows equal the full run's."""
    from crimp_amd.eventfile import write_events_fits
    from crimp_amd.measureToAs import measureToAs
    ev = gold("events_1e2259.npz")
    p = str(tmp_path / "ev.fits")
    write_events_fits(p, ev["TIME"], ev["PI"], int(ev["MJDREFI"]), float(ev["MJDREFF"]))
    full = str(tmp_path / "full")
    measureToAs(p, gpath("1e2259.par"), gpath("1e2259_template.txt"), gpath("timIntToAs_1e2259.txt"),
                eneLow=1, eneHigh=5, toaStart=35, toaEnd=41, brutemin=True, toaFile=full)
    lines = open(gpath("timIntToAs_1e2259.txt")).read().splitlines()
    k = 38
    cols = lines[k + 1].split("\t")
    cols[1], cols[2] = "70000.0", "70000.5"  # interval 38 now covers no photon
    lines[k + 1] = "\t".join(cols)
    ivf = str(tmp_path / "iv.txt")
    open(ivf, "w").write("\n".join(lines) + "\n")
    monkeypatch.setenv("CRIMP_TOA_BATCH_PHOTONS", "1")
    part = str(tmp_path / "part")
    with pytest.raises(IndexError):
        measureToAs(p, gpath("1e2259.par"), gpath("1e2259_template.txt"), ivf, eneLow=1, eneHigh=5, toaStart=35,
                    toaEnd=41, brutemin=True, toaFile=part)
    got = open(part + ".txt").read().splitlines()
    want = open(full + ".txt").read().splitlines()
    assert got == want[:1 + (k - 35)]          # header + ToAs 35, 36, 37


def _vary_template(base, free):
    t = {k: (dict(v) if isinstance(v, dict) else v) for k, v in base.items()}
    for k, v in t.items():
        if isinstance(v, dict):
            v["vary"] = k in free
    return t


# two-component peaked templates of the bundled 1-5 keV profile (Cauchy: the 70-bin fit of
# crimp_amd.pulseprofile, rates in counts/s; von Mises: the same peaks with wid 0.25)
PEAKED = {"cauchy": {"norm": 15.864028670406764, "amp_1": 2.729162017889153, "cen_1": 3.9150528740296684,
                     "wid_1": 0.15062796589359873, "amp_2": 1.3486800419057134, "cen_2": 3.418941216972105,
                     "wid_2": 0.13877334840312794},
          "vonmises": {"norm": 15.86, "amp_1": 2.73, "cen_1": 3.915, "wid_1": 0.25, "amp_2": 1.35, "cen_2": 3.419,
                       "wid_2": 0.25}}


def _cauchy_vm_template(model, th=None):
    th = th or PEAKED[model]
    t = {"model": model, "nbrComp": 2}
    for k, v in th.items():
        if k not in ("phShift", "ampShift"):
            t[k] = {"value": np.float64(v), "vary": False}
    return t


@pytest.mark.parametrize("model", ["fourier", "cauchy", "vonmises"])
def test_shape_gradient_sums_vs_oracle(gpu, model):
    """crimp_toa_shape_points: the extended LL and its gradient in every template parameter against the
    oracle's NumPy LL and central differences of it."""
    from crimp_amd.readPPtemplate import readPPtemplate
    from crimp_amd.toafit_vary import VaryParamFitter
    g, iv, _ = _golden_rows()
    x = g["folded"][g["offsets"][2]:g["offsets"][3]]
    E = float(iv["ToA_exposure"].to_numpy()[g["ids"]][2])
    if model == "fourier":
        tm = readPPtemplate(gpath("1e2259_template.txt"))
    else:
        tm = _cauchy_vm_template(model, json.load(open(gpath("cauchy_vm_theta.json"))))
        x = x * 2 * np.pi
    f = VaryParamFitter(x, np.array([0, x.size]), np.array([E]), tm)
    rng = np.random.default_rng(3)
    th = f.theta0.copy()
    th[-1] = 0.07
    th[1:-1] *= 1 + 0.05 * rng.standard_normal(th.size - 2)
    ll, gr = f.evaluate_theta([0], th[None, :])
    _, K, _, _, _, _, _, _ = O._readvary_setup(tm)
    ref = O.readvary_ll(x, E, model, K, th)
    assert ll[0] == pytest.approx(ref, rel=1e-12)
    for j in range(th.size):
        h = 1e-5 * max(1.0, abs(th[j]))
        tp, tm_ = th.copy(), th.copy()
        tp[j] += h
        tm_[j] -= h
        fd = (O.readvary_ll(x, E, model, K, tp) - O.readvary_ll(x, E, model, K, tm_)) / (2 * h)
        assert gr[0, j] == pytest.approx(fd, rel=2e-5, abs=1e-3), (model, f.names[j])


def test_readvaryparam_vs_oracle(gpu):
    """readvaryparam (measureToAs.py:727-801): template amplitudes 1-2 freed with the norm. No reference
    output exercises it (parity unpinned beyond the oracle's optimum restatement); with only the norm
    free it must reproduce the default fit."""
    from crimp_amd.measureToAs import measureToA_fourier, defineinitialfitparam
    from crimp_amd.readPPtemplate import readPPtemplate
    from crimp_amd.toafit import ToAFitter
    from crimp_amd.toafit_vary import VaryParamFitter
    g, iv, _ = _golden_rows()
    base = readPPtemplate(gpath("1e2259_template.txt"))
    E = iv["ToA_exposure"].to_numpy()[g["ids"]]
    tm = _vary_template(base, {"norm", "amp_1", "amp_2"})
    assert defineinitialfitparam(tm, readvaryparam=True)[1] == 3
    r = VaryParamFitter(g["folded"], g["offsets"], E, tm).fit()
    for i in (2, 5):
        x = g["folded"][g["offsets"][i]:g["offsets"][i + 1]]
        o = O.fit_toa_readvary(x, E[i], tm)
        assert abs(r["phShi"][i] - o["phShi"]) / (2 * math.pi) < 1e-6
        assert r["LLmax"][i] == pytest.approx(o["LLmax"], abs=1e-5)
        assert r["phShi_LL"][i] == o["phShi_LL"] and r["phShi_UL"][i] == o["phShi_UL"]
        assert r["LLmax"][i] >= o["LLmax"] - 1e-6
        # the LL is flat to 1e-7 along the freed amplitudes within 1e-3 sigma: two optimisers agree to ~1e-5
        assert r["reducedChi2"][i] == pytest.approx(o["reducedChi2"], rel=1e-4)
        np.testing.assert_allclose(r["theta"][i], o["theta"], rtol=1e-4, atol=1e-6)
    s = measureToA_fourier(tm, g["folded"][g["offsets"][2]:g["offsets"][3]], E[2], readvaryparam=True)
    assert s["phShi"] == pytest.approx(r["phShi"][2], abs=1e-9)
    # only the norm free: the default fit's optimum (its norm bounds are not active here)
    tn = _vary_template(base, {"norm"})
    rn = VaryParamFitter(g["folded"], g["offsets"], E, tn).fit()
    rd = ToAFitter(g["folded"], g["offsets"], E, base).fit()
    np.testing.assert_allclose(rn["phShi"], rd["phShi"], rtol=0, atol=2 * math.pi * 1e-7)
    np.testing.assert_array_equal(rn["phShi_LL"], rd["phShi_LL"])
    np.testing.assert_array_equal(rn["phShi_UL"], rd["phShi_UL"])
    np.testing.assert_allclose(rn["LLmax"], rd["LLmax"], rtol=0, atol=1e-6)


@pytest.mark.parametrize("model", ["cauchy", "vonmises"])
def test_readvaryparam_peaked_vs_oracle(gpu, model):
    from crimp_amd.toafit_vary import VaryParamFitter
    g, iv, _ = _golden_rows()
    i = 2
    x = g["folded"][g["offsets"][i]:g["offsets"][i + 1]] * 2 * np.pi
    E = float(iv["ToA_exposure"].to_numpy()[g["ids"]][i])
    tm = _vary_template(_cauchy_vm_template(model), {"norm", "cen_1", "wid_2" if model == "cauchy" else "amp_2"})
    r = VaryParamFitter(x, np.array([0, x.size]), np.array([E]), tm).fit()
    o = O.fit_toa_readvary(x, E, tm)
    assert abs(r["phShi"][0] - o["phShi"]) / (2 * math.pi) < 1e-6
    assert r["LLmax"][0] == pytest.approx(o["LLmax"], abs=1e-5)
    assert r["phShi_LL"][0] == o["phShi_LL"] and r["phShi_UL"][0] == o["phShi_UL"]
    assert r["LLmax"][0] >= o["LLmax"] - 1e-6
    np.testing.assert_allclose(r["theta"][0], o["theta"], rtol=1e-4, atol=1e-6)


def test_addphasecolumn_cli_phases(gpu, tmp_path):
    """addphasecolumn (eventfile.py:319-390) on a FITS file written from the bundled events: the PHASE column
    equals the oracle's calcphase of TIME/86400 + MJDREF (calcphase.py:152-176) within 1e-9 cycles, in both the
    barycentred file and the -ne file; the original columns are untouched."""
    from crimp_amd.eventfile import main, write_events_fits, read_fits, read_table
    ev = gold("events_1e2259.npz")
    paths = []
    for name in ("bary.fits", "nonbary.fits"):
        p = str(tmp_path / name)
        write_events_fits(p, ev["TIME"], ev["PI"], int(ev["MJDREFI"]), float(ev["MJDREFF"]))
        paths.append(p)
    main([paths[0], gpath("1e2259.par"), "-ne", paths[1]])
    mjd = ev["TIME"] / 86400 + (int(ev["MJDREFI"]) + float(ev["MJDREFF"]))
    from crimp_amd.readtimingmodel import ReadTimingModel
    _, ref = O.calcphase(mjd, ReadTimingModel(gpath("1e2259.par")).readfulltimingmodel()[0])
    for p in paths:
        raw, hdus = read_fits(p)
        cols = read_table(raw, hdus[1][0], hdus[1][1])
        np.testing.assert_array_equal(cols["TIME"], ev["TIME"])
        d = np.abs(cols["PHASE"] - ref)
        assert np.max(np.minimum(d, 1 - d)) <= 1e-9


def test_search_sets_equals_per_interval_search(gpu):
    """crimp_search_sets (one launch for every ToA interval's H_5 at f(ToA_mid), measureToAs.py:210-212) equals
    PeriodSearch(...).htest() interval by interval: the reference's H5 of ToAs 35-41 within 1e-9 relative, and
    the fp64 path on synthetic sets of 1..5000 photons within 1e-9 relative."""
    from crimp_amd import ops
    from crimp_amd.periodsearch import PeriodSearch
    from crimp_amd._native import STAT_H, STAT_Z2
    from crimp_amd.measureToAs import select_intervals
    g = gold("toa_1e2259.npz")
    ev = gold("events_1e2259.npz")
    keep = (ev["PI"] * 0.01 >= 1.0) & (ev["PI"] * 0.01 <= 5.0)
    mjd = ev["TIME"][keep] / 86400 + (int(ev["MJDREFI"]) + float(ev["MJDREFF"]))
    iv = pd.read_csv(gpath("timIntToAs_1e2259.txt"), sep=r"\s+", comment="#")
    t, off = select_intervals(mjd, iv["ToA_tstart"].to_numpy()[g["ids"]], iv["ToA_tend"].to_numpy()[g["ids"]])
    np.testing.assert_array_equal(np.diff(off), g["n"])
    h = ops.search_sets(t * 86400, off, g["freq"], 5, STAT_H)
    close_rel(h, g["h5"], 1e-9)
    rng = np.random.default_rng(5)
    sizes = np.array([1, 2, 3, 64, 1000, 5000])
    x = np.sort(rng.uniform(0, 1e4, sizes.sum())) + 5.0e9
    o = np.concatenate([[0], np.cumsum(sizes)])
    fr = rng.uniform(0.1, 3.0, sizes.size)
    for stat, m in ((STAT_Z2, 2), (STAT_H, 7), (STAT_H, 20)):
        got = ops.search_sets(x, o, fr, m, stat)
        for i in range(sizes.size):
            ps = PeriodSearch(x[o[i]:o[i + 1]], np.array([fr[i]]), m, precision="f64")
            ref = ps.ztest() if stat == STAT_Z2 else ps.htest()
            close_rel(got[i:i + 1], ref, 1e-9)


def test_readvaryparam_with_varyamps_vs_oracle(gpu):
    """readvaryparam + varyAmps (measureToAs.py:306-312 after :727-801): norm and ph_2 freed by the template,
    then ampShift freed in [0.01, 100] and everything refitted; the 1-sigma scan re-maximises all three. Against
    the oracle's restatement (parity unpinned: no reference output exercises the combination)."""
    from crimp_amd.measureToAs import measureToA_fourier
    from crimp_amd.readPPtemplate import readPPtemplate
    from crimp_amd.toafit_vary import VaryParamFitter
    g, iv, _ = _golden_rows()
    E = iv["ToA_exposure"].to_numpy()[g["ids"]]
    tm = _vary_template(readPPtemplate(gpath("1e2259_template.txt")), {"norm", "ph_2"})
    r = VaryParamFitter(g["folded"], g["offsets"], E, tm, vary_amps=True).fit()
    i = 2
    x = g["folded"][g["offsets"][i]:g["offsets"][i + 1]]
    o = O.fit_toa_readvary(x, E[i], tm, vary_amps=True)
    assert abs(r["phShi"][i] - o["phShi"]) / (2 * math.pi) < 1e-6
    assert r["LLmax"][i] == pytest.approx(o["LLmax"], abs=1e-5)
    assert r["LLmax"][i] >= o["LLmax"] - 1e-6
    assert r["ampShift"][i] == pytest.approx(o["ampShift"], rel=1e-4)
    assert r["phShi_LL"][i] == o["phShi_LL"] and r["phShi_UL"][i] == o["phShi_UL"]
    assert r["reducedChi2"][i] == pytest.approx(o["reducedChi2"], rel=1e-4)
    s = measureToA_fourier(tm, x, E[i], readvaryparam=True, varyAmps=True)
    assert s["phShi"] == pytest.approx(r["phShi"][i], abs=1e-9)

"""CPU-side checks: the C-ABI library loads and exports the header's symbols; host logic
(readers, event ingestion, scan-phase sequence) matches the reference's fixtures."""
import json
import os
import re

import numpy as np
import pandas as pd
import pytest

from conftest import ROOT, gold, gpath


def _declared():
    src = open(os.path.join(ROOT, "include", "crimp_hip.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|int64_t|double|const char\*)\s+(crimp_\w+)\s*\(", src, re.M)))


def test_library_exports_every_declared_symbol():
    from crimp_amd import _native
    L = _native.load(require_device=False)
    names = _declared()
    assert set(names) == set(_native.EXPORTS)
    for n in names:
        assert hasattr(L, n), n
    assert L.crimp_version() >= 1


def test_mfma_hazard_rules_hold_in_default_kernel():
    """The default search kernel keeps VALU reads of MFMA results and rewrites of MFMA operands away from the
    MFMA (crimp_amd/csrc/mfma_drain.h; tools/isa_hazards.py): guards against a compiler or code change that moves
    them back next to the matrix pipe, which made repeat runs differ."""
    import importlib.util
    from crimp_amd import _native
    if not os.path.exists(_native.LIB_PATH):
        pytest.skip("library not built")
    spec = importlib.util.spec_from_file_location("isa_hazards", os.path.join(ROOT, "tools", "isa_hazards.py"))
    H = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(H)
    funcs = H.disassemble(_native.LIB_PATH)
    checked = 0
    for name, insts in funcs.items():
        if "k_search_exact" in name:
            assert any(op.startswith(("v_mfma", "v_smfmac")) for _, op, _, _ in insts), name
            assert H.check_function(insts) == [], name
            assert set(H.agpr_users(insts)) <= {"v_mfma_i32_32x32x32_i8", "v_smfmac_i32_32x32x64_i8",
                                                 "v_accvgpr_read_b32", "v_accvgpr_write_b32"}, name
            assert not any(op.startswith("scratch_") for _, op, _, _ in insts), name  # no spills
            checked += 1
    assert checked == 2


def _agpr_check():
    import importlib.util
    spec = importlib.util.spec_from_file_location("agpr_check", os.path.join(ROOT, "tools", "agpr_check.py"))
    A = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(A)
    return A


def test_exact_kernel_accumulators_untouched_by_compiler(device_builds):
    """The exact kernel's accumulators live in AGPRs outside hipcc's register model (search_exact.h, ex_mfma):
    the compiled kernels may not touch an AGPR themselves (a VGPR spilled to an AGPR would overwrite them)."""
    res = _agpr_check().compiler_agpr_accesses(asm_path=device_builds["default"])
    assert len(res) == 2
    for name, bad in res.items():
        assert bad == [], (name, bad[:4])


def test_agpr_check_flags_the_unclobbered_build(device_builds):
    """The fault of round 3's no-ex_open build: without the AGPR clobbers on the MFMA statements, hipcc keeps a
    value of its own in an accumulator AGPR (the photon-time address, overwritten by tile 0's MFMAs ->
    hipErrorIllegalAddress). tools/agpr_check.py must see that in the build without clobbers and fences; the shipped
    build (clobbers on) has none (test above), and the clobbered no-fence build ran bit-identically on the GPU
    (profiles/r04/ab_fences.log)."""
    A = _agpr_check()
    bad = A.compiler_agpr_accesses(asm_path=device_builds["noclob_noopen"])
    assert any(v for v in bad.values()), bad
    ok = A.compiler_agpr_accesses(asm_path=device_builds["noopen"])
    assert all(v == [] for v in ok.values()), ok


def test_isa_hazards_rejects_the_unfenced_build(device_builds):
    """Without the ex_open fences hipcc rewrites MFMA A operands 32-64 issue cycles after the MFMA; on the GPU that
    build returned rows 16..31 of every 2-D tile differently from run to run (profiles/r04/ab_fences.log). The
    checker must reject it, as it accepts the shipped kernel (test_mfma_hazard_rules_hold_in_default_kernel)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("isa_hazards", os.path.join(ROOT, "tools", "isa_hazards.py"))
    H = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(H)
    funcs = {k: v for k, v in H.disassemble(device_builds["noopen_co"]).items() if "k_search_exact" in k}
    assert len(funcs) == 2
    for name, insts in funcs.items():
        bad = H.check_function(insts)
        assert any("rewrites A" in v[2] and v[3] < H.ISSUE_MIN for v in bad), name


def test_hot_path_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from crimp_amd import _native
    from crimp_amd.periodsearch import PeriodSearch
    with pytest.raises(_native.CrimpNativeError):
        PeriodSearch(np.arange(10.0), np.array([0.1]), 2).ztest()


def test_header_flags_match_python_bindings():
    from crimp_amd import _native
    src = open(os.path.join(ROOT, "include", "crimp_hip.h")).read()
    flags = dict(re.findall(r"#define CRIMP_(FLAG_\w+)\s+(\d+)u", src))
    assert "FLAG_F64" in flags
    for name, val in flags.items():
        assert getattr(_native, name) == int(val), name


def test_search_precision_option_validated_and_no_fallback():
    import torch
    from crimp_amd import _native
    from crimp_amd.periodsearch import PeriodSearch
    with pytest.raises(ValueError):
        PeriodSearch(np.arange(10.0), np.array([0.1]), 2, precision="f16").ztest()
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(_native.CrimpNativeError):
        PeriodSearch(np.arange(10.0), np.array([0.1]), 2, precision="f64").ztest()


def test_readtimingmodel_matches_reference():
    from crimp_amd.readtimingmodel import ReadTimingModel
    ref = json.load(open(gpath("parsed.json")))["par"]
    got = ReadTimingModel(gpath("1e2259.par")).readfulltimingmodel()[0]
    assert set(got) == set(ref)
    for k in ref:
        assert float(got[k]) == ref[k], k


def test_readpptemplate_matches_reference():
    from crimp_amd.readPPtemplate import readPPtemplate
    ref = json.load(open(gpath("parsed.json")))["template"]
    got = readPPtemplate(gpath("1e2259_template.txt"))
    assert list(got) == list(ref)
    for k, v in ref.items():
        if isinstance(v, dict):
            assert float(got[k]["value"]) == v["value"] and got[k]["vary"] == v["vary"], k
        else:
            assert got[k] == v, k


def test_eventfile_roundtrip_and_toa_mid(tmp_path):
    """Raw FITS ingestion: TIME/86400+MJDREF and PI*0.01 reproduce ToA_mid of ToAs 35-41 bit-exactly."""
    from crimp_amd.eventfile import EvtFileOps, write_events_fits
    ev = gold("events_1e2259.npz")
    p = str(tmp_path / "ev.fits")
    write_events_fits(p, ev["TIME"], ev["PI"], int(ev["MJDREFI"]), float(ev["MJDREFF"]))
    ef = EvtFileOps(p).build_time_energy_df().filtenergy(1.0, 5.0)
    t = ef.time_energy_df["TIME"].to_numpy()
    assert t.size == 68877
    iv = pd.read_csv(gpath("timIntToAs_1e2259.txt"), sep=r"\s+", comment="#")
    ref = pd.read_csv(gpath("ToAs_2259.txt"), sep=r"\s+", comment="#")
    for ii in range(35, 42):
        tt = t[(t >= iv["ToA_tstart"][ii]) & (t <= iv["ToA_tend"][ii])]
        mid = ((tt[-1] - tt[0]) / 2) + tt[0]
        assert str(mid) == str(ref[ref["ToA"] == ii]["ToA_mid"].iloc[0])


def test_eventfile_reads_bundled_fits_if_present():
    from crimp_amd.eventfile import EvtFileOps
    p = "/root/reference/data/1e2259_ni1020600110.fits"
    if not os.path.exists(p):
        pytest.skip("reference data not mounted")
    ev = gold("events_1e2259.npz")
    ef = EvtFileOps(p)
    df = ef.build_time_energy_df().time_energy_df
    assert np.array_equal(df["TIME"].to_numpy(), ev["TIME"] / 86400 + (int(ev["MJDREFI"]) + float(ev["MJDREFF"])))
    kw, gti = ef.readGTI()
    assert kw["TELESCOPE"] == "NICER" and gti.shape[1] == 2


def test_binphases_host_matches_reference():
    from crimp_amd.binphases import binphases
    g = gold("toa_1e2259.npz")
    x = g["folded"][g["offsets"][0]:g["offsets"][1]]
    b = binphases(x, 15)
    assert np.array_equal(b["ctsBins"], g["bp_cts"]) and np.array_equal(b["ppBins"], g["bp_ppBins"])


def test_ephemtmjd_matches_reference():
    from crimp_amd.ephemTmjd import ephemTmjd
    g = gold("toa_1e2259.npz")
    for mid, f, fd in zip(g["mid"], g["freq"], g["fdot"]):
        e = ephemTmjd(mid, gpath("1e2259.par"))
        assert e["freqAtTmjd"] == f and e["freqdotAtTmjd"] == fd


def test_ephemtmjd_vectorised_and_parsed_model():
    """measure_intervals evaluates ephemTmjd once over all ToA mids with the model parsed once: the frequencies
    (the H-test trials) equal the reference's per-ToA values to the last bit or within 1 ulp."""
    from crimp_amd.ephemTmjd import ephemTmjd
    from crimp_amd.readtimingmodel import ReadTimingModel
    g = gold("toa_1e2259.npz")
    tm = ReadTimingModel(gpath("1e2259.par")).readfulltimingmodel()[0]
    e = ephemTmjd(np.asarray(g["mid"]), tm)
    np.testing.assert_array_max_ulp(e["freqAtTmjd"], g["freq"], maxulp=1)
    np.testing.assert_array_max_ulp(e["freqdotAtTmjd"], g["fdot"], maxulp=1)


def test_select_intervals_equals_reference_mask():
    """Interval selection by binary search on time-sorted photons (and the reference's mask otherwise,
    measureToAs.py:173-174) returns the reference's photons, inclusive bounds, in order."""
    from crimp_amd.measureToAs import select_intervals
    rng = np.random.default_rng(7)
    t = np.sort(rng.uniform(0.0, 100.0, 5000))
    starts = np.array([1.0, t[10], 50.0, 99.9])
    ends = np.array([2.0, t[20], 50.0 + 1e-9, 120.0])
    for tt in (t, rng.permutation(t)):
        x, off = select_intervals(tt, starts, ends)
        ref = [tt[(tt >= a) & (tt <= b)] for a, b in zip(starts, ends)]
        assert off.tolist() == np.concatenate([[0], np.cumsum([r.size for r in ref])]).tolist()
        np.testing.assert_array_equal(x, np.concatenate(ref))
    assert select_intervals(t, starts, ends)[1][2] - select_intervals(t, starts, ends)[1][1] == 11  # t[10]..t[20]


def test_error_scan_phase_sequence_clip_semantics():
    """lmfit clips a stepped phShift to [-pi, pi] once, then the loop moves the bound (measureToAs.py:332-334)."""
    from crimp_amd.toafit import ToAFitter
    tm = {"model": "fourier", "norm": {"value": 10.0}, "amp_1": {"value": 1.0}, "ph_1": {"value": 0.0}}
    fit = ToAFitter.__new__(ToAFitter)
    fit.model, fit.res, fit.pb = "fourier", 1000, np.pi
    step = 2 * np.pi / 1000
    phi = np.array([-np.pi + 2.5 * step, 0.3])
    ks = np.arange(1, 6)
    seq = fit._scan_phases(phi, -1, ks)
    exp0 = phi[0] - ks * step
    exp0[2] = -np.pi  # third step is the first past the bound: evaluated at the bound itself
    np.testing.assert_array_equal(seq[0], exp0)
    np.testing.assert_array_equal(seq[1], phi[1] - ks * step)
    fit.model, fit.pb = "cauchy", 1.5 * np.pi
    seq = fit._scan_phases(np.array([1.5 * np.pi - step]), 1, ks)
    np.testing.assert_array_equal(seq[0], np.minimum(1.5 * np.pi - step + ks * step, 1.5 * np.pi))
    del tm


def test_scan_cap_detection_and_warning_text(caplog):
    """The reference's loop leaves kk = k + 1 and logs 'Could not estimate ...' once kk > phShiftRes/2
    (measureToAs.py:348-350, :373-375); toafit.scan_capped reads kk back from the bound kk*step + step/2."""
    import logging
    from crimp_amd.toafit import scan_capped, warn_capped
    for res in (20, 21, 1000):
        step = 2 * np.pi / res
        kk = np.arange(2, res // 2 + 3)
        sig = kk * step + step / 2
        np.testing.assert_array_equal(scan_capped(sig, res), kk > res / 2)
    res = 20
    step = 2 * np.pi / res
    r = {"phShi_LL": np.array([11 * step + step / 2, 3 * step + step / 2]),
         "phShi_UL": np.array([4 * step + step / 2, 11 * step + step / 2])}
    with caplog.at_level(logging.WARNING):
        warn_capped(r, res, ["ToA5", "ToA6"], logging.getLogger("crimp_amd.measureToAs"))
    assert [rec.getMessage() for rec in caplog.records] == ["Could not estimate lower-bound uncertainty on ToA5",
                                                            "Could not estimate upper-bound uncertainty on ToA6"]


def test_toa_batches_and_interval_counts():
    """measureToAs' batching of intervals by photon budget and its photon counts (inclusive bounds, the
    reference's mask for unsorted times, measureToAs.py:173-174)."""
    from crimp_amd.measureToAs import _batches, _interval_counts
    assert _batches([5, 5, 5, 5], 10) == [(0, 2), (2, 4)]
    assert _batches([50, 1, 1], 10) == [(0, 1), (1, 3)]
    assert _batches([1, 1, 1], 1) == [(0, 1), (1, 2), (2, 3)]
    assert _batches([], 10) == []
    rng = np.random.default_rng(3)
    t = np.sort(rng.uniform(0.0, 100.0, 3000))
    st, en = np.array([1.0, t[10], 60.0, 200.0]), np.array([2.0, t[20], 60.0, 300.0])
    want = [np.count_nonzero((t >= a) & (t <= b)) for a, b in zip(st, en)]
    assert _interval_counts(t, st, en).tolist() == want
    assert _interval_counts(rng.permutation(t), st, en).tolist() == want
    assert want[1] == 11 and want[3] == 0


def test_shrinking_pipeline_blocks():
    """measure_intervals' pipelined blocks: consecutive, covering every interval once, none empty, photon shares
    non-increasing (4 : 3 : 2 : 1 of the total where the interval sizes allow)."""
    from crimp_amd.measureToAs import _shrinking_blocks
    assert _shrinking_blocks(np.full(1250, 100000), 4) == [(0, 500), (500, 875), (875, 1125), (1125, 1250)]
    assert _shrinking_blocks(np.full(2, 7), 4) == [(0, 1), (1, 2)]
    rng = np.random.default_rng(5)
    for _ in range(50):
        c = rng.integers(1, 1000, rng.integers(2, 40))
        b = _shrinking_blocks(c, int(rng.integers(2, 6)))
        assert b[0][0] == 0 and b[-1][1] == c.size and all(x[1] == y[0] for x, y in zip(b, b[1:]))
        assert all(x[1] > x[0] for x in b)


def test_measuretoas_empty_first_interval_writes_header_then_raises(tmp_path):
    """An empty first interval: the reference has written only the header when TIME_toa[-1] raises at
    measureToAs.py:182; so does the drop-in (no device call is made before it)."""
    from crimp_amd.eventfile import write_events_fits
    from crimp_amd.measureToAs import HEADER, measureToAs
    ev = gold("events_1e2259.npz")
    p = str(tmp_path / "ev.fits")
    write_events_fits(p, ev["TIME"], ev["PI"], int(ev["MJDREFI"]), float(ev["MJDREFF"]))
    lines = open(gpath("timIntToAs_1e2259.txt")).read().splitlines()
    cols = lines[36].split("\t")
    cols[1], cols[2] = "70000.0", "70000.5"
    lines[36] = "\t".join(cols)
    ivf = str(tmp_path / "iv.txt")
    open(ivf, "w").write("\n".join(lines) + "\n")
    out = str(tmp_path / "ToAs")
    with pytest.raises(IndexError):
        measureToAs(p, gpath("1e2259.par"), gpath("1e2259_template.txt"), ivf, eneLow=1, eneHigh=5, toaStart=35,
                    toaEnd=41, toaFile=out)
    assert open(out + ".txt").read() == HEADER


def test_tim_writer_matches_reference_tim(tmp_path):
    """phshiftTotimfile on the reference's ToA table reproduces data/ToAs_2259.tim (all 84 rows); the
    current writer prefixes each data line with one space (timfile.py:159), the committed file predates it."""
    from crimp_amd.timfile import phshiftTotimfile, readtimfile
    out = str(tmp_path / "x")
    tab = phshiftTotimfile(gpath("ToAs_2259.txt"), gpath("1e2259.par"), out, tempModPP="1e2259_template.txt")
    got = open(out + ".tim").read().splitlines()
    ref = open(gpath("ToAs_2259.tim")).read().splitlines()
    assert got[0] == ref[0] == "FORMAT 1" and len(got) == len(ref) == 85
    for a, b in zip(got[1:], ref[1:]):
        assert a == " " + b
    back = readtimfile(gpath("ToAs_2259.tim"))
    np.testing.assert_allclose(back["pulse_ToA"].to_numpy(), tab["TOA"].to_numpy(), rtol=2e-16, atol=0)
    assert list(back.columns[:5]) == ["template", "frequency", "pulse_ToA", "pulse_ToA_err", "time_ref"]
    with pytest.raises(FileExistsError):
        phshiftTotimfile(gpath("ToAs_2259.txt"), gpath("1e2259.par"), out)


def test_ephem_integer_rotation_lands_on_integer_phase():
    from crimp_amd.ephemIntegerRotation import ephemIntegerRotation
    e = ephemIntegerRotation(58144.25468778948, gpath("1e2259.par"))
    assert abs(e["phase_residual_from_integer"]) < 1e-6 and e["Tmjd_intRotation"] <= 58144.25468778948


def test_crimp_import_name_and_entry_points():
    """``import crimp.<module>`` resolves to the drop-in modules; the reference's console scripts for the provided
    modules (pyproject.toml:36-48) are declared in pyproject.toml and setup.cfg and their targets exist."""
    import importlib
    import crimp.periodsearch
    import crimp_amd.periodsearch
    assert crimp.periodsearch is crimp_amd.periodsearch
    from crimp.measureToAs import measureToAs  # noqa: F401
    with pytest.raises(ImportError):
        importlib.import_module("crimp.plot_pps")  # out of scope
    want = {"timeintervalsfortoas": "buildtimeintervalsToAs", "templatepulseprofile": "pulseprofile",
            "measuretoas": "measureToAs", "addphasecolumn": "eventfile", "ephemintegerrotation": "ephemIntegerRotation",
            "phshifttotimfile": "timfile"}
    py = open(os.path.join(ROOT, "pyproject.toml")).read()
    cfg = open(os.path.join(ROOT, "setup.cfg")).read()
    for script, mod in want.items():
        line = '%s = "crimp_amd.%s:main"' % (script, mod)
        assert line in py, line
        assert "%s = crimp_amd.%s:main" % (script, mod) in cfg
        assert callable(getattr(importlib.import_module("crimp_amd." + mod), "main"))


def test_add_column_rewrites_events_table(tmp_path):
    """The FITS rewrite of addphasecolEF (eventfile.py:345-353): every original column, the other HDUs and the
    header keywords survive; the new double column reads back exactly; a duplicate name is refused."""
    from crimp_amd.eventfile import EvtFileOps, add_column, read_fits, read_table, write_fits
    p = str(tmp_path / "e.fits")
    t = np.linspace(0.0, 1.0e4, 777)
    flags = np.zeros((777, 8), bool)
    flags[::3, 2] = True
    write_fits(p, [("EVENTS", [("TIME", "D", t), ("PI", "J", np.arange(777) % 600), ("EVENT_FLAGS", "8L", flags)],
                    {"TELESCOP": "NICER", "MJDREFI": 56658, "MJDREFF": 0.000777592592592593}),
                   ("GTI", [("START", "D", np.array([0.0, 20.0])), ("STOP", "D", np.array([10.0, 30.0]))], {})])
    before = EvtFileOps(p).readEF()
    ph = np.random.default_rng(1).uniform(0, 1, 777)
    add_column(p, "EVENTS", "PHASE", ph)
    raw, hdus = read_fits(p)
    ev = read_table(raw, hdus[1][0], hdus[1][1])
    np.testing.assert_array_equal(ev["TIME"], t)
    np.testing.assert_array_equal(ev["PI"], np.arange(777) % 600)
    np.testing.assert_array_equal(ev["EVENT_FLAGS"], flags)
    np.testing.assert_array_equal(ev["PHASE"], ph)
    assert EvtFileOps(p).readEF() == before
    np.testing.assert_array_equal(EvtFileOps(p).readGTI()[1][:, 0], np.array([0.0, 20.0]) / 86400 + before["MJDREF"])
    with pytest.raises(ValueError):
        add_column(p, "EVENTS", "PHASE", ph)
    with pytest.raises(ValueError):
        add_column(p, "EVENTS", "PHASE2", ph[:5])


def test_phases_waves_scalar_without_wave_harmonics():
    """Phases.waves() without WAVEj terms returns the reference's scalar 0 * F0 (calcphase.py:135-149): no WAVE*
    key at all, or only WAVEEPOCH and WAVE_OM (the harmonic loop runs over len(WAVE*) - 2 = 0 terms). No GPU call."""
    from crimp_amd.calcphase import Phases
    t = 58000.0 + np.arange(4.0)
    for tm in ({"PEPOCH": 58000.0, "F0": 0.5},
               {"PEPOCH": 58000.0, "F0": 0.5, "WAVEEPOCH": 58000.0, "WAVE_OM": 0.01}):
        w = Phases(t, tm).waves()
        assert np.ndim(w) == 0 and w == 0.0 and isinstance(w, float)
    with pytest.raises(KeyError):  # as the reference, which reads F0 for the normalisation
        Phases(t, {"PEPOCH": 58000.0}).waves()


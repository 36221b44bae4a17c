"""ToA interval construction (buildtimeintervalsToAs.py) against data/timIntToAs_1e2259.txt.

The merged event file the reference ran on is missing, so rows 35-41 -- the
intervals inside the bundled observation -- are pinned: the bundled 1-5 keV events from ToA 35's
first photon on (tests/golden/events_1e2259.npz) plus the observation's GTI table
(tests/golden/gti_1e2259.npz), written to a FITS file, must give those 7 rows text-identical
(start/end photon, interval length, GTI-clipped exposure, counts, rate). The other rows and the
bunches file are unpinned. Merging and the NICER FPM correction are checked on synthetic inputs
against restated expectations."""
import numpy as np
import pandas as pd
import pytest

from conftest import gold, gpath
from crimp_amd.buildtimeintervalsToAs import merge_adjacent_intervals, timeintervalsToAs, main
from crimp_amd.eventfile import write_fits


def _kw(ev):
    return {"TELESCOP": "NICER", "MJDREFI": int(ev["MJDREFI"]), "MJDREFF": float(ev["MJDREFF"]), "TIMESYS": "TDB"}


def _bundled_fits(path, first_photon_mjd):
    ev, g = gold("events_1e2259.npz"), gold("gti_1e2259.npz")
    mjd = ev["TIME"] / 86400 + (int(ev["MJDREFI"]) + float(ev["MJDREFF"]))
    keep = mjd >= first_photon_mjd
    write_fits(path, [("EVENTS", [("TIME", "1D", ev["TIME"][keep]), ("PI", "1I", ev["PI"][keep])], _kw(ev)),
                      ("GTI", [("START", "1D", g["START"]), ("STOP", "1D", g["STOP"])], _kw(ev))])


def test_rows_35_41_of_reference_interval_file(tmp_path):
    lines = open(gpath("timIntToAs_1e2259.txt")).read().splitlines()
    want = [ln.split("\t", 1)[1] for ln in lines[36:43]]          # rows 35..41 without the ToA index
    t35 = float(want[0].split("\t")[0])
    # events strictly from ToA 35's first photon: its start was written rounded to 9 decimals
    evf = str(tmp_path / "obs.fits")
    ev = gold("events_1e2259.npz")
    mjd = np.sort(ev["TIME"] / 86400 + (int(ev["MJDREFI"]) + float(ev["MJDREFF"])))
    first = mjd[np.argmin(np.abs(mjd - t35))]
    _bundled_fits(evf, first)
    out = str(tmp_path / "tim")
    df = timeintervalsToAs(evf, totCtsEachToA=10000, waitTimeCutoff=1.0, eneLow=1.0, eneHigh=5.0, outputFile=out)
    got = [ln.split("\t", 1)[1] for ln in open(out + ".txt").read().splitlines()[1:]]
    assert len(df) == 7
    assert got == want
    assert open(out + ".txt").readline().rstrip("\n") == lines[0]


def test_merge_adjacent_intervals_rules():
    df = pd.DataFrame({"ToA_tstart": [0.0, 1.0, 1.5, 5.0, 5.2], "ToA_tend": [0.9, 1.4, 1.6, 5.1, 5.3],
                       "ToA_lenInt": [0.9, 0.4, 0.1, 0.1, 0.1], "ToA_exposure": [100., 100., 10., 100., 50.],
                       "Events": [1000., 1000., 100., 1000., 10.], "ct_rate": [10., 10., 10., 10., .2]})
    m = merge_adjacent_intervals(df, 500, 1.0)
    # row 2 (100 events, 0.1 d after row 1's end) merges into row 1; row 4 into row 3
    assert list(m["Events"]) == [1000.0, 1100.0, 1010.0]
    assert list(m["ToA_tend"]) == [0.9, 1.6, 5.3]
    assert m["ct_rate"][1] == 1100.0 / 110.0 and m["ToA_lenInt"][2] == 5.3 - 5.0
    assert merge_adjacent_intervals(df.iloc[:0], 500, 1.0).empty


def _synthetic(path, times_s, gti, fpm=None):
    kw = {"TELESCOP": "NICER", "MJDREFI": 56658, "MJDREFF": 0.000777592592592593, "TIMESYS": "TDB"}
    tabs = [("EVENTS", [("TIME", "1D", times_s), ("PI", "1I", np.full(times_s.size, 200))], kw),
            ("GTI", [("START", "1D", gti[:, 0]), ("STOP", "1D", gti[:, 1])], kw)]
    if fpm is not None:
        tabs.append(("FPM_SEL", [("TIME", "1D", fpm[0]), ("FPM_SEL", "56L", fpm[1]), ("FPM_ON", "56L", fpm[1])], kw))
    write_fits(path, tabs)


def test_bunches_slices_exposure_and_fpm_correction(tmp_path):
    rng = np.random.default_rng(5)
    # three GTIs: two 0.2 d apart (one bunch), a third 3 days later (new bunch at waitTimeCutoff=1)
    gti = np.array([[0.0, 1000.0], [0.2 * 86400, 0.2 * 86400 + 2000.0], [3.2 * 86400, 3.2 * 86400 + 500.0]])
    t = np.sort(np.concatenate([rng.uniform(a, b, int(b - a) * 2) for a, b in gti]))
    sel = np.zeros((t.size, 56), bool)
    sel[:, :48] = True
    evf = str(tmp_path / "s.fits")
    _synthetic(evf, t, gti, fpm=(t, sel))
    out = str(tmp_path / "iv")
    df = timeintervalsToAs(evf, totCtsEachToA=1500, waitTimeCutoff=1.0, eneLow=0.5, eneHigh=10, outputFile=out)
    b = pd.read_csv(out + "_bunches.txt", sep=r"\s+")
    assert len(b) == 2
    n1 = int(((t >= gti[0, 0]) & (t <= gti[1, 1])).sum())
    assert df["Events"].sum() == t.size
    # slices of 1500 in bunch 1; its remainder (< 750) merges into the previous slice only if close in time
    mjd = t / 86400 + (56658 + 0.000777592592592593)
    first = mjd[0]
    assert abs(df["ToA_tstart"][0] - float("%.9f" % first)) < 1e-12
    # exposure of the first slice: GTI 0 clipped to [first photon, 1500th photon]
    exp0 = (mjd[1499] - mjd[0]) * 86400
    assert abs(df["ToA_exposure"][0] - exp0) < 1e-4
    # a slice spanning GTIs 0 and 1: its exposure excludes the gap
    k = np.searchsorted(mjd, (gti[0, 1]) / 86400 + 56658.000777592592592593)
    s = (k // 1500) * 1500
    e = min(s + 1499, n1 - 1)
    assert df["ToA_exposure"][k // 1500] < (mjd[e] - mjd[s]) * 86400
    # FPM correction multiplies the rate by 52 * exposure / sum(selected detectors per second stamp)
    df2 = timeintervalsToAs(evf, totCtsEachToA=1500, waitTimeCutoff=1.0, outputFile=out + "c", correxposure=True)
    a, z = df2["ToA_tstart"][0], df2["ToA_tend"][0]
    nsel = 48.0 * ((mjd >= a) & (mjd <= z)).sum()
    assert df2["ct_rate"][0] == pytest.approx(df["ct_rate"][0] * 52 * df["ToA_exposure"][0] / nsel, rel=1e-12)


def test_cli_writes_interval_file_and_log(tmp_path, monkeypatch):
    gti = np.array([[0.0, 3000.0]])
    t = np.linspace(1.0, 2999.0, 4000)
    evf = str(tmp_path / "c.fits")
    _synthetic(evf, t, gti)
    monkeypatch.chdir(tmp_path)
    main([evf, "-tc", "1000", "-of", "cli"])
    df = pd.read_csv(tmp_path / "cli.txt", sep="\t")
    assert list(df.columns) == ["ToA", "ToA_tstart", "ToA_tend", "ToA_lenInt", "ToA_exposure", "Events", "ct_rate"]
    assert list(df["Events"]) == [1000.0] * 4
    assert (tmp_path / "cli.log").exists()

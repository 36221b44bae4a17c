"""The NUFFT (csrc/search_nufft.h; the default search path, also asked for by precision="nufft") through the C-ABI:
the non-uniform-FFT Z^2 / H search against the reference's goldens and the oracle at the per-trial contract (plain
1e-6 relative, best trial exact), its raw powers (fix-up off) against the fp64 kernel, determinism, row sharding,
and the inputs it declines to the exact rule (unsorted photons, short, non-uniform or descending grids, cells beyond
32 bits). Full-size configs: tests/test_gpu_fullsize.py."""
import numpy as np
import pytest

from conftest import gold
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def close_rel(got, ref, rtol=1e-6):
    got, ref = np.asarray(got), np.asarray(ref)
    err = np.abs(got - ref) / np.abs(ref)
    assert err.max() <= rtol, "max relative error %.3g at %d" % (err.max(), int(err.argmax()))
    return err.max()


def _path():
    from crimp_amd import _native as N
    return N.load().crimp_last_search_path()


SPREADS = ["auto", "gather", "mfma"]


def _spread(monkeypatch, spread):
    """auto: the library's choice (cell gather for <= 2 rows, MFMA slots otherwise); gather / mfma force one form."""
    if spread != "auto":
        monkeypatch.setenv("CRIMP_NUFFT_SPREAD", spread)


@pytest.mark.parametrize("spread", SPREADS)
def test_nufft_config1_goldens(gpu, spread, monkeypatch):
    """Config 1 (the reference's own outputs on the bundled 1e2259 events, 400-trial progression)."""
    from crimp_amd.periodsearch import PeriodSearch
    _spread(monkeypatch, spread)
    g = gold("periodsearch_1e2259.npz")
    z = PeriodSearch(g["time"], g["freq"], 2, precision="nufft").ztest()
    assert _path() == 2
    assert int(np.argmax(z)) == 200
    close_rel(z, g["z2_m2"])
    h = PeriodSearch(g["time"], g["freq"], 20, precision="nufft").htest()
    assert _path() == 2
    assert int(np.argmax(h)) == 200
    close_rel(h, g["h_m20"])
    arr, df = PeriodSearch(g["time"], g["fsub"], 2, precision="nufft").twod_ztest(g["fd"])
    np.testing.assert_array_equal(arr[:, :2], g["z2d_m2"][:, :2])
    close_rel(arr[:, 2], g["z2d_m2"][:, 2])
    assert list(df.columns) == ["Freq", "Freq_dot", "Z2pow"]


def test_nufft_synthetic_goldens_and_routes(gpu):
    """Synthetic goldens m = 1..20; grids the NUFFT does not take (non-uniform, < 64 trials, unsorted photons) go to
    the default path with the same results."""
    from crimp_amd.periodsearch import PeriodSearch
    g = gold("periodsearch_synth.npz")
    t, f = g["time"], g["freq"]
    for m in (1, 2, 3, 5):
        z = PeriodSearch(t, f, m, precision="nufft").ztest()
        assert _path() == 2
        close_rel(z, g["z_m%d" % m])
        assert np.argmax(z) == np.argmax(g["z_m%d" % m])
    for m in (1, 5, 20):
        close_rel(PeriodSearch(t, f, m, precision="nufft").htest(), g["h_m%d" % m])
        assert _path() == 2
    close_rel(PeriodSearch(t, f[64:128], 2, precision="nufft").twod_ztest(g["fd"])[0][:, 2], g["z2d_m2"][:, 2])
    assert _path() == 2
    close_rel(PeriodSearch(t, f[64:128], 3, precision="nufft").twod_ztest(g["fd"])[0][:, 2], g["z2d_m3"][:, 2])
    close_rel(PeriodSearch(g["time_perm"], g["freq_nu"], 2, precision="nufft").ztest(), g["z_nonuniform_m2"])
    assert _path() != 2
    close_rel(PeriodSearch(t[:2], f[:8], 3, precision="nufft").htest(), g["h_n2"])
    close_rel(PeriodSearch(t, f[100:101], 2, precision="nufft").ztest(), g["z_m1trial"])


@pytest.mark.parametrize("spread", SPREADS)
def test_nufft_vs_oracle_larger(gpu, spread, monkeypatch):
    """2e5 photons x 2048 trials (Z^2_2), a 3 x 1024 2-D grid (H_3) and H_20 on 4096 trials against the oracle."""
    from crimp_amd.periodsearch import PeriodSearch
    _spread(monkeypatch, spread)
    from crimp_amd.synth import pulsed_events
    from crimp_amd import _native as N
    t = pulsed_events(200000, 2.0e5, 7.123456789, pulsed_frac=0.05, seed=4)
    f = 7.123456789 + (np.arange(-1024, 1024) / (10 * 2.0e5))
    z = PeriodSearch(t, f, 2, precision="nufft").ztest()
    assert _path() == 2
    zr = O.search(t, f, 2)
    assert int(np.argmax(z)) == int(np.argmax(zr))
    close_rel(z, zr)
    assert N.load().crimp_last_fixups() <= 4
    fd = np.array([-13.0, -12.0, -11.5])
    a = PeriodSearch(t, f[512:1536], 3, precision="nufft").twod_htest(fd)[0][:, 2]
    ar = O.search(t, f[512:1536], 3, freq_dot=fd, stat="h")
    assert int(np.argmax(a)) == int(np.argmax(ar))
    close_rel(a, ar)
    f2 = 7.123456789 + (np.arange(-2048, 2048) / (10 * 2.0e5))
    h = PeriodSearch(t, f2, 20, precision="nufft").htest()
    hr = O.search(t, f2, 20, stat="h")
    assert int(np.argmax(h)) == int(np.argmax(hr))
    close_rel(h, hr)


@pytest.mark.parametrize("spread", SPREADS)
def test_nufft_raw_powers_vs_f64(gpu, spread, monkeypatch):
    """The NUFFT itself (fix-up off) against the fp64 kernel on every trial: 1-D Z^2_2 and 2-D H_20 over 16 rows
    (two row passes), odd trial counts per row (h = nf // 2 with nf odd)."""
    from crimp_amd import ops, _native as N
    _spread(monkeypatch, spread)
    from crimp_amd.synth import pulsed_events
    t = pulsed_events(300000, 3.0e5, 3.3, pulsed_frac=0.05, fdot=-2e-11, seed=7)
    t0 = (t[0] + t[-1]) / 2
    f = 3.3 + (np.arange(-700, 701) / (10 * 3.0e5))
    ref = ops.search(t, t0, f, 2, 0, precision="f64")
    z = ops.search(t, t0, f, 2, 0, flags=N.FLAG_NO_FIXUP, precision="nufft")
    assert _path() == 2
    close_rel(z, ref, 1e-6)
    fd = np.linspace(-12.5, -10.0, 16)
    ref = ops.search(t, t0, f[:301], 20, 1, log10_negfdot=fd, precision="f64")
    h = ops.search(t, t0, f[:301], 20, 1, log10_negfdot=fd, flags=N.FLAG_NO_FIXUP, precision="nufft")
    assert _path() == 2
    close_rel(h, ref, 1e-6)


def test_nufft_deterministic_and_row_shards(gpu):
    """Repeat runs are bit-identical; a 2-D grid computed as row ranges (what each rank of a row-sharded search
    computes) equals the whole grid bit for bit. A range that cuts rows is planned on its own segment of the row
    (another n, centre and moment count), so it agrees with the whole grid within the plans' error, not bitwise."""
    from crimp_amd import ops
    from crimp_amd.synth import pulsed_events
    t = pulsed_events(100000, 1.0e5, 3.0, pulsed_frac=0.1, seed=9)
    f = 3.0 + np.arange(-300, 300) / 1.0e6
    fd = np.array([-12.0, -11.0, -10.5])
    t0 = (t[0] + t[-1]) / 2
    full = ops.search(t, t0, f, 2, 0, log10_negfdot=fd, precision="nufft")
    np.testing.assert_array_equal(ops.search(t, t0, f, 2, 0, log10_negfdot=fd, precision="nufft"), full)
    rows = [ops.search(t, t0, f, 2, 0, log10_negfdot=fd, first=r * 600, count=600, precision="nufft") for r in range(3)]
    np.testing.assert_array_equal(np.concatenate(rows), full)
    parts = [ops.search(t, t0, f, 2, 0, log10_negfdot=fd, first=a, count=b - a, precision="nufft")
             for a, b in ((0, 333), (333, 901), (901, 1800))]
    cut = np.concatenate(parts)
    close_rel(cut, full, 1e-6)
    assert np.median(np.abs(cut - full) / np.abs(full)) <= 1e-12


@pytest.mark.parametrize("precision", [None, "nufft"])
def test_nufft_unsorted_photons_take_default_path(gpu, precision):
    """Unsorted photons: the NUFFT declines and the exact rule runs -- the exact kernel on a 512-trial progression,
    the fp64 kernel on a 128-trial one (rows of < 256 trials never take the exact kernel, whichever precision was
    asked for; bit-identical to precision="f64")."""
    from crimp_amd import ops
    from crimp_amd.periodsearch import PeriodSearch
    from crimp_amd.synth import pulsed_events
    t = pulsed_events(50000, 5.0e4, 2.5, pulsed_frac=0.2, seed=3)
    f = 2.5 + np.arange(-256, 256) / (10 * 5.0e4)
    rng = np.random.default_rng(0)
    tp = t[rng.permutation(t.size)]
    tp[0], tp[-1] = t[0], t[-1]  # same t0
    z = PeriodSearch(tp, f, 2, precision=precision).ztest()
    assert _path() == 1
    close_rel(z, O.search(tp, f, 2))
    z = PeriodSearch(tp, f[:128], 2, precision=precision).ztest()
    assert _path() == 0
    t0 = (tp[0] + tp[-1]) / 2
    np.testing.assert_array_equal(z, ops.search(tp, t0, f[:128], 2, 0, precision="f64"))
    close_rel(z, O.search(tp, f[:128], 2))


@pytest.mark.parametrize("precision", [None, "nufft"])
def test_nufft_declines_descending_grid(gpu, precision):
    """A descending progression (delta < 0, accepted by the progression check) would size the NUFFT's cell tables
    negative: the plan declines it and the exact kernel runs, within 1e-6 of the oracle on every trial (1-D Z^2_2
    and 2-D H_3)."""
    from crimp_amd.periodsearch import PeriodSearch
    from crimp_amd.synth import pulsed_events
    t = pulsed_events(100000, 1.0e5, 3.0, pulsed_frac=0.1, seed=19)
    f = np.flip(3.0 + np.arange(-512, 512) / 1.0e6)
    z = PeriodSearch(t, f, 2, precision=precision).ztest()
    assert _path() == 1
    zr = O.search(t, f, 2)
    assert int(np.argmax(z)) == int(np.argmax(zr))
    close_rel(z, zr)
    fd = np.array([-12.0, -11.0])
    a = PeriodSearch(t, f[256:768], 3, precision=precision).twod_htest(fd)[0][:, 2]
    assert _path() == 1
    close_rel(a, O.search(t, f[256:768], 3, freq_dot=fd, stat="h"))


def test_nufft_declines_cells_beyond_32_bits(gpu):
    """The kernels convert cells with 32-bit rint: a reference time far from the photons (t0 = 0 for photons near
    5e9 s) puts the cells of a 4096-trial grid at 2e-4 Hz steps past 2^31 although the photons span only 3 wraps of
    the FFT. The plan declines (the exact kernel runs, bit-identical to precision="exact" with the same t0); with
    the photons' midpoint as t0 the same grid takes the NUFFT. (1-D Z^2 does not depend on t0.)"""
    from crimp_amd import ops
    rng = np.random.default_rng(23)
    t = np.sort(5.0e9 + rng.uniform(0.0, 1.0e4, 20000))
    f = 1.0 + np.arange(4096) * 2.0e-4
    z0 = ops.search(t, 0.0, f, 2, 0)
    assert _path() == 1
    np.testing.assert_array_equal(z0, ops.search(t, 0.0, f, 2, 0, precision="exact"))
    tm = (t[0] + t[-1]) / 2
    zm = ops.search(t, tm, f, 2, 0)
    assert _path() == 2
    close_rel(zm, ops.search(t, tm, f, 2, 0, precision="f64"))


def test_nufft_fused_pass2_equals_separate_combine(gpu, monkeypatch):
    """FFT pass 2 fused with the moments' Horner sum against pass 2 and k_nu_combine as two kernels
    (CRIMP_NUFFT_FUSED=0), both with the radix-16 row transform (CRIMP_NUFFT_R8=0): the same arithmetic, so
    bit-identical powers; the default (512-thread radix-8 row pass, k_nu_rows_iw) and the 4096-row / 256-row-column
    kernels (k_nu_rows4096_combine, k_nu_rows_combine8, k_nu_cols256; k_nu_cols512 with 2048-element rows at n = 2^20) against
    the generic ones (CRIMP_NUFFT_ROWS4096=0) to rounding -- single-pass (n <= 4096) and four-step FFTs, 1-D and 2-D
    grids."""
    from crimp_amd import ops, _native as N
    from crimp_amd.synth import pulsed_events
    t = pulsed_events(200000, 2.0e5, 3.3, pulsed_frac=0.05, fdot=-2e-11, seed=8)
    t0 = (t[0] + t[-1]) / 2
    fd = np.array([-12.0, -11.0, -10.5])

    def run(**env):
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        z = ops.search(t, t0, f, m, 1, log10_negfdot=fdv, precision="nufft", flags=N.FLAG_NO_FIXUP)
        for k in env:
            monkeypatch.delenv(k)
        return z

    def close(x, y):
        rel = np.abs(x - y) / np.abs(y)
        assert rel.max() <= 1e-10 and np.median(rel) <= 1e-13, (rel.max(), np.median(rel))

    for f, m, fdv in ((3.3 + np.arange(-700, 701) / 2.0e6, 2, None), (3.3 + np.arange(-40000, 40000) / 2.0e6, 3, None),
                      (3.3 + np.arange(-1500, 1500) / 2.0e6, 5, fd),
                      (3.3 + np.arange(-300000, 300000) / 2.0e7, 2, None)):  # n = 2^20: 256-row columns
        r16 = run(CRIMP_NUFFT_R8="0")
        np.testing.assert_array_equal(r16, run(CRIMP_NUFFT_R8="0", CRIMP_NUFFT_FUSED="0"))
        generic = run(CRIMP_NUFFT_ROWS4096="0")
        close(r16, generic)
        close(run(), generic)
        close(run(CRIMP_NUFFT_P2_IW="0"), generic)  # three block-wide exchanges per moment (k_nu_rows_combine8<12>)
        if len(f) == 600000:  # n = 2^20 as 512 x 2048 (k_nu_cols512, k_nu_rows_combine8<11>)
            close(run(CRIMP_NUFFT_ROW2048="1"), generic)


def test_nufft_gather_lane_splits(gpu, monkeypatch):
    """The cell gather with 1, 2, 4 and 8 lanes per cell (CRIMP_NUFFT_LANES; the default picks from photons per
    cell): each against the fp64 kernel at the per-trial contract with fix-up off, and against each other to
    summation-order rounding -- a dense 1-D grid (many photons per cell) and a 2-row 2-D grid."""
    from crimp_amd import ops, _native as N
    from crimp_amd.synth import pulsed_events
    monkeypatch.setenv("CRIMP_NUFFT_SPREAD", "gather")
    t = pulsed_events(400000, 2.0e5, 3.3, pulsed_frac=0.05, fdot=-2e-11, seed=11)
    t0 = (t[0] + t[-1]) / 2
    f = 3.3 + np.arange(-600, 600) / 2.0e6
    fd = np.array([-12.0, -10.5])
    for m, fdv in ((3, None), (2, fd)):
        ref = ops.search(t, t0, f, m, 1, log10_negfdot=fdv, precision="f64")
        got = []
        for lanes in ("1", "2", "4", "8"):
            monkeypatch.setenv("CRIMP_NUFFT_LANES", lanes)
            got.append(ops.search(t, t0, f, m, 1, log10_negfdot=fdv, precision="nufft", flags=N.FLAG_NO_FIXUP))
            assert _path() == 2
            close_rel(got[-1], ref, 1e-6)
        for g in got[1:]:
            assert np.median(np.abs(g - got[0]) / np.abs(got[0])) <= 1e-12
    monkeypatch.setenv("CRIMP_NUFFT_LANES", "3")
    with pytest.raises(Exception):
        ops.search(t, t0, f, 2, 1, precision="nufft")


def test_nufft_moment_chunks_agree(gpu, monkeypatch):
    """The radix-8 row path runs the moments in chunks (CRIMP_NUFFT_PCHUNK, default 4: pass 1 and pass 2 of one chunk
    in turn, each chunk adding its part of the moment sum to the trials' harmonic sums): chunks of 1, 3, 4 and all P
    moments agree to rounding (the chunks restart the Bessel recurrence from their own series values) -- a 1-D
    2^20-point plan (256-row columns) and a 2-D 2^17-point plan (generic columns), raw powers (fix-up off)."""
    from crimp_amd import ops, _native as N
    from crimp_amd.synth import pulsed_events
    t = pulsed_events(300_000, 2.0e5, 3.3, pulsed_frac=0.05, fdot=-2e-11, seed=13)
    t0 = (t[0] + t[-1]) / 2
    cases = ((3.3 + np.arange(-300000, 300000) / 2.0e7, 2, None), (3.3 + np.arange(-40000, 40000) / 2.0e6, 3,
                                                                    np.array([-12.0, -11.0, -10.5])))
    for f, m, fdv in cases:
        got = {}
        for pc in ("0", "1", "3", "4"):
            monkeypatch.setenv("CRIMP_NUFFT_PCHUNK", pc)
            got[pc] = ops.search(t, t0, f, m, 1, log10_negfdot=fdv, flags=N.FLAG_NO_FIXUP)
            assert _path() == 2
        for pc in ("1", "3", "4"):
            rel = np.abs(got[pc] - got["0"]) / np.abs(got["0"])
            assert rel.max() <= 1e-10 and np.median(rel) <= 1e-13, (pc, rel.max(), np.median(rel))
        close_rel(got["4"], ops.search(t, t0, f, m, 1, log10_negfdot=fdv, precision="f64"), 1e-6)


@pytest.mark.parametrize("rows", [1, 3])
def test_nufft_plan_cache_revalidated_on_device(gpu, rows, monkeypatch):
    """A repeated search over the same device buffers reuses its last plan without reading the plan's scalars back
    (the device re-checks them, k_ap_final). Changing the buffers in place between calls -- the photons shifted,
    the grid rescaled, two photons swapped (unsorted), the grid made non-uniform -- must give exactly what a search
    without the cache gives (CRIMP_NUFFT_PLAN_CACHE=0), kernel family included: the cell-gather form (1 row) and the
    MFMA-slot form (3 rows)."""
    import torch
    from crimp_amd import ops
    from crimp_amd.synth import pulsed_events
    t_h = pulsed_events(200_000, 2.0e5, 3.3, pulsed_frac=0.05, fdot=-2e-11, seed=17)
    f_h = 3.3 + np.arange(-1000, 1000) / 2.0e6
    fd = None if rows == 1 else torch.as_tensor(np.linspace(-12.0, -10.5, rows), device=gpu)
    t = torch.as_tensor(t_h, device=gpu)
    f = torch.as_tensor(f_h, device=gpu)
    t0 = (t_h[0] + t_h[-1]) / 2

    def run(cache):
        if cache:
            monkeypatch.delenv("CRIMP_NUFFT_PLAN_CACHE", raising=False)
        else:
            monkeypatch.setenv("CRIMP_NUFFT_PLAN_CACHE", "0")
        z = ops.search(t, t0, f, 3, 1, log10_negfdot=fd).cpu().numpy()
        return z, _path()

    first, p1 = run(True)
    again, p2 = run(True)        # the cached plan, revalidated on the device
    assert p1 == p2 == 2
    np.testing.assert_array_equal(again, first)
    edits = [("shift photons", lambda: t.add_(0.37)),
             ("rescale grid", lambda: f.mul_(1.0 + 1e-7)),
             ("swap two photons", lambda: t.__setitem__(slice(1000, 1002), t[1000:1002].flip(0).clone())),
             ("restore order", lambda: t.copy_(torch.sort(t).values)),
             ("non-uniform grid", lambda: f.__setitem__(7, f[7] + 1e-9))]
    for name, edit in edits:
        run(True)                 # the plan of the current buffers is cached
        edit()
        got, pg = run(True)       # the stale plan: detected on the device, recomputed
        ref, pr = run(False)
        assert pg == pr, (name, pg, pr)
        np.testing.assert_array_equal(got, ref, err_msg=name)


def test_nufft_fused_finalize_identical(gpu, monkeypatch):
    """The last harmonic's row pass forms the powers, certificate and per-block best trials itself (NuFinal); the
    separate k_nu_finalize launch (CRIMP_NUFFT_FINAL=separate) gives the same powers bit for bit, the same fix-up count
    and the same best trial -- Z^2 and H, 1-D (cell gather) and 3-row 2-D (MFMA slots) grids, a forced fix-up of many
    trials included (CRIMP_FIXUP_REL in a child process)."""
    import os
    import subprocess
    import sys
    import tempfile
    from crimp_amd import ops, _native as N
    from crimp_amd.synth import pulsed_events
    from conftest import ROOT
    t = pulsed_events(300_000, 2.0e5, 3.3, pulsed_frac=0.05, fdot=-2e-11, seed=21)
    t0 = (t[0] + t[-1]) / 2
    for f, m, stat, fdv in ((3.3 + np.arange(-300000, 300000) / 2.0e7, 2, 0, None),
                            (3.3 + np.arange(-300000, 300000) / 2.0e7, 5, 1, None),
                            (3.3 + np.arange(-40000, 40000) / 2.0e6, 3, 1, np.array([-12.0, -11.0, -10.5]))):
        res = {}
        for mode in ("fused", "separate"):
            if mode == "separate":
                monkeypatch.setenv("CRIMP_NUFFT_FINAL", "separate")
            else:
                monkeypatch.delenv("CRIMP_NUFFT_FINAL", raising=False)
            z, bv, bi = ops.search_best(t, t0, f, m, stat, log10_negfdot=fdv)
            res[mode] = (z, bv, bi, N.load().crimp_last_fixups(), _path())
        a, b = res["fused"], res["separate"]
        np.testing.assert_array_equal(a[0], b[0])
        assert a[1:] == b[1:] and a[4] == 2
        assert a[2] == int(np.argmax(a[0])) and a[1] == a[0].max()
    code = ("import sys, os, numpy as np; sys.path.insert(0, %r); from crimp_amd import ops, _native as N; "
            "from crimp_amd.synth import pulsed_events; t = pulsed_events(300000, 2.0e5, 3.3, pulsed_frac=0.05, "
            "seed=21); f = 3.3 + np.arange(-300000, 300000) / 2.0e7; t0 = (t[0] + t[-1]) / 2; out = {}\n"
            "for mode in ('fused', 'separate'):\n"
            "    os.environ['CRIMP_NUFFT_FINAL'] = mode\n"
            "    z, bv, bi = ops.search_best(t, t0, f, 3, 1); out[mode] = (z, bv, bi, N.load().crimp_last_fixups())\n"
            "np.savez(sys.argv[1], za=out['fused'][0], zb=out['separate'][0], "
            "ma=np.array(out['fused'][1:]), mb=np.array(out['separate'][1:]))") % ROOT
    with tempfile.TemporaryDirectory() as d:
        outp = os.path.join(d, "f.npz")
        subprocess.run([sys.executable, "-c", code, outp], check=True, timeout=300,
                       env=dict(os.environ, CRIMP_FIXUP_REL="1e-9"))
        r = np.load(outp)
    np.testing.assert_array_equal(r["za"], r["zb"])
    np.testing.assert_array_equal(r["ma"], r["mb"])
    assert r["ma"][2] > 100  # fix-ups ran (the best trial was then recomputed after them)

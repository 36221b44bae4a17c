"""Thin typed wrappers over the C-ABI (one per entry point of include/crimp_hip.h).

Arrays are NumPy (host; staged by the library, synchronous) or torch CUDA tensors
(device; enqueued on torch's current stream). Outputs are allocated here when not
given. These are the only functions that touch the native library.
"""
import ctypes
import os

import numpy as np

from . import _native as N


def _modeltm(tm):
    """Pack a timing-model dict (values or {value, flag}) into crimp_timing_model."""
    def val(x):
        if isinstance(x, dict) and "value" in x and "flag" in x:  # readtimingmodel.py:309-321
            return x["value"]
        return x
    d = {k: val(v) for k, v in tm.items()}
    m = N.TimingModel()
    m.pepoch = float(d["PEPOCH"])
    for i in range(13):
        m.f[i] = float(d.get("F%d" % i, 0.0))
    ngl = sum(1 for k in d if k.startswith("GLEP_"))  # calcphase.py:94
    if ngl > N.MAX_GLITCH:
        raise ValueError("at most %d glitches supported" % N.MAX_GLITCH)
    m.n_glitch = ngl
    for j in range(1, ngl + 1):
        row = [d["GLEP_%d" % j]] + [d.get("%s_%d" % (b, j), 0.0) for b in ("GLPH", "GLF0", "GLF1", "GLF2", "GLF0D", "GLTD")]
        for c in range(7):
            m.glitch[j - 1][c] = float(row[c])
    nw = sum(1 for k in d if k.startswith("WAVE"))  # calcphase.py:135
    if nw:
        nharm = nw - 2  # calcphase.py:142 assumes WAVEEPOCH and WAVE_OM are present
        if nharm > N.MAX_WAVE:
            raise ValueError("at most %d wave harmonics supported" % N.MAX_WAVE)
        m.wave_epoch = float(d["WAVEEPOCH"])
        m.wave_om = float(d["WAVE_OM"])
        m.n_wave = max(nharm, 0)
        for j in range(1, nharm + 1):
            m.wave_ab[j - 1][0] = float(d["WAVE%d" % j]["A"])
            m.wave_ab[j - 1][1] = float(d["WAVE%d" % j]["B"])
    return m


def calcphase(t_mjd, timing_model_dict, parts=7, total=None, folded=None, want_folded=True, flags=0):
    L = N.load()
    b = N.Buffers()
    tp = b.arg(t_mjd, np.float64)
    n = int(t_mjd.numel() if N._is_torch(t_mjd) else np.size(t_mjd))
    if total is None:
        total = _empty_like_input(t_mjd, n, b)
    if folded is None and want_folded:
        folded = _empty_like_input(t_mjd, n, b)
    op = b.arg(total, np.float64, writable=True)
    fp = b.arg(folded, np.float64, writable=True) if folded is not None else None
    m = _modeltm(timing_model_dict)
    with b.device_guard():
        N.check(L.crimp_calcphase(tp, n, ctypes.byref(m), int(parts), op, fp, b.flags(flags), b.stream()))
    return total, folded


def _empty_like_input(a, n, b, dtype=np.float64):
    if b.device:
        import torch
        return torch.empty(n, dtype=torch.float64 if dtype == np.float64 else torch.int64, device=a.device)
    return np.empty(n, dtype=dtype)


def search_flags():
    """Extra search flags from the environment for unmodified callers: CRIMP_PRECISION=exact|nufft|f64, and
    CRIMP_SEARCH=mfma (fail unless a factorised kernel applies)."""
    f = 0
    prec = os.environ.get("CRIMP_PRECISION", "").lower()
    if prec == "f64":
        f |= N.FLAG_F64
    elif prec == "nufft":
        f |= N.FLAG_NUFFT
    elif prec == "exact":
        f |= N.FLAG_EXACT
    elif prec != "":
        raise ValueError("CRIMP_PRECISION must be exact, nufft or f64 (the fp32 'fast' path was retired)")
    if os.environ.get("CRIMP_SEARCH", "").lower() == "mfma":
        f |= N.FLAG_FORCE_MFMA
    return f


PRECISIONS = (None, "exact", "f64", "nufft")
_PRECISION_FLAGS = {None: 0, "nufft": N.FLAG_NUFFT, "exact": N.FLAG_EXACT, "f64": N.FLAG_F64}


def search(t, t0, freq, nharm, stat, log10_negfdot=None, first=0, count=None, out=None, flags=0, precision=None):
    """Z^2 / H over the fd-outer grid; computes flat trials [first, first+count).
    ``precision``: None or "nufft" (default: the non-uniform FFT wherever it applies -- an ascending progression of
    >= 64 trials per row segment and time-sorted photons --, otherwise the "exact" rule; every trial within 1e-6
    relative of the reference by its certificate and the fp64 fix-up), "exact" (no NUFFT: the exact-integer i8 MFMA
    kernel on progressions of >= 256 trials, fp64 otherwise; the default of rounds 1-5) or "f64" (fp64 kernel
    everywhere). A precision argument takes precedence over CRIMP_PRECISION."""
    return _search(t, t0, freq, nharm, stat, log10_negfdot, first, count, out, flags, precision, False)


def search_best(t, t0, freq, nharm, stat, log10_negfdot=None, first=0, count=None, out=None, flags=0,
                precision=None):
    """``search`` and the best trial of its powers in one call (crimp_search_best): (out, best power, index within
    the computed range), np.argmax semantics; a NUFFT search reads the best back with its fix-up count."""
    return _search(t, t0, freq, nharm, stat, log10_negfdot, first, count, out, flags, precision, True)


def _search(t, t0, freq, nharm, stat, log10_negfdot, first, count, out, flags, precision, want_best):
    if precision not in PRECISIONS:
        raise ValueError("precision must be one of %s (the fp32 'fast' path was retired)" % (PRECISIONS,))
    env = search_flags()
    if precision is not None:
        env &= ~(N.FLAG_F64 | N.FLAG_NUFFT | N.FLAG_EXACT)
    flags |= _PRECISION_FLAGS[precision] | env
    L = N.load()
    b = N.Buffers()
    tp = b.arg(t, np.float64)
    fp = b.arg(freq, np.float64)
    dp = b.arg(log10_negfdot, np.float64, allow_none=True)
    n = int(t.numel() if N._is_torch(t) else np.size(t))
    nf = int(freq.numel() if N._is_torch(freq) else np.size(freq))
    nfd = 0 if log10_negfdot is None else int(log10_negfdot.numel() if N._is_torch(log10_negfdot)
                                               else np.size(log10_negfdot))
    total = (nfd if nfd else 1) * nf
    if count is None:
        count = total - first
    if out is None:
        out = _empty_like_input(t, count, b)
    op = b.arg(out, np.float64, writable=True)
    if not want_best:
        with b.device_guard():
            N.check(L.crimp_search(tp, n, float(t0), fp, nf, dp, nfd, int(nharm), int(stat), int(first), int(count),
                                   op, b.flags(flags), b.stream()))
        return out
    res = np.zeros(2, dtype=np.float64)
    with b.device_guard():
        N.check(L.crimp_search_best(tp, n, float(t0), fp, nf, dp, nfd, int(nharm), int(stat), int(first), int(count),
                                    op, ctypes.c_void_p(res.ctypes.data), b.flags(flags), b.stream()))
    return out, float(res[0]), int(res[1])


def best(x):
    """(max, index) of a power array with np.argmax semantics (ties to the lowest index, NaN first), one small
    device reduction and one readback (crimp_best)."""
    n = int(x.numel() if N._is_torch(x) else np.size(x))
    if n == 0:
        raise ValueError("best of an empty array")
    L = N.load()
    b = N.Buffers()
    xp = b.arg(x, np.float64)
    res = np.zeros(2, dtype=np.float64)
    with b.device_guard():
        N.check(L.crimp_best(xp, n, ctypes.c_void_p(res.ctypes.data), b.flags(), b.stream()))
    return float(res[0]), int(res[1])


def search_sets(t, offsets, freq, nharm, stat, flags=0):
    """One-trial Z^2 / H of many photon sets (crimp_search_sets): set i = t[offsets[i]:offsets[i+1]] (seconds) at
    freq[i], each with its own t0 = (first + last)/2. fp64. ``flags`` N.FLAG_ASYNC (device tensors): returns with the
    kernel queued on the current stream; synchronise with it before reading the result."""
    L = N.load()
    b = N.Buffers()
    tp = b.arg(t, np.float64)
    op = b.arg(offsets, np.int64)
    fp = b.arg(freq, np.float64)
    nset = int((offsets.numel() if N._is_torch(offsets) else np.size(offsets)) - 1)
    out = _empty_like_input(t, nset, b)
    outp = b.arg(out, np.float64, writable=True)
    with b.device_guard():
        N.check(L.crimp_search_sets(tp, op, nset, fp, int(nharm), int(stat), outp, b.flags(flags), b.stream()))
    return out


def make_template(model, amps, locs, wids=None, amp_shift=1.0):
    """crimp_template from arrays (model in {'fourier','cauchy','vonmises'})."""
    from scipy.special import i0
    t = N.Template()
    t.model = N.MODEL_IDS[model]
    K = len(amps)
    if not 1 <= K <= N.MAX_COMP:
        raise ValueError("template needs 1..%d components" % N.MAX_COMP)
    t.ncomp = K
    for j in range(K):
        t.amp[j] = float(amps[j])
        t.loc[j] = float(locs[j])
        if wids is not None:
            t.wid[j] = float(wids[j])
            t.i0[j] = float(i0(1.0 / float(wids[j]) ** 2)) if model == "vonmises" else 1.0
    t.amp_shift = float(amp_shift)
    return t


def toa_points(x, offsets, tpl, pt_interval, pt_norm, pt_phi):
    """[npts, 8] sums (see crimp_toa_points) in fp64 on host."""
    L = N.load()
    b = N.Buffers()
    xp = b.arg(x, np.float64)
    op = b.arg(offsets, np.int64)
    ip = b.arg(pt_interval, np.int64)
    npp = b.arg(pt_norm, np.float64)
    pp = b.arg(pt_phi, np.float64)
    npts = int(pt_norm.numel() if N._is_torch(pt_norm) else np.size(pt_norm))
    nint = int((offsets.numel() if N._is_torch(offsets) else np.size(offsets)) - 1)
    out = _empty_like_input(x, npts * 8, b)
    outp = b.arg(out, np.float64, writable=True)
    with b.device_guard():
        N.check(L.crimp_toa_points(xp, op, nint, ctypes.byref(tpl), ip, npp, pp, npts, outp, b.flags(), b.stream()))
    return out.reshape(npts, 8)


def toa_shape_points(x, offsets, tpls, pt_interval, pt_norm, pt_phi, aux=None):
    """[npts, CRIMP_SHAPE_SUMS] extended-LL sums with template-shape gradients (crimp_toa_shape_points):
    point p = interval pt_interval[p] with its own template tpls[p]; aux[p, j] = I1/I0(1/wid_j^2) for
    von Mises templates. Templates, intervals and aux are host data; pt_norm/pt_phi follow x."""
    L = N.load()
    b = N.Buffers()
    xp = b.arg(x, np.float64)
    op = b.arg(offsets, np.int64)
    npts = len(tpls)
    arr = (N.Template * max(npts, 1))(*tpls)
    pint = np.ascontiguousarray(pt_interval, dtype=np.int64)
    if pint.size != npts:
        raise ValueError("one interval per point")
    if b.device:
        import torch
        pt_norm = torch.as_tensor(np.asarray(pt_norm, np.float64), device=x.device)
        pt_phi = torch.as_tensor(np.asarray(pt_phi, np.float64), device=x.device)
    npp = b.arg(pt_norm, np.float64)
    pp = b.arg(pt_phi, np.float64)
    auxa = None if aux is None else np.ascontiguousarray(aux, dtype=np.float64).reshape(npts, N.MAX_COMP)
    nint = int((offsets.numel() if N._is_torch(offsets) else np.size(offsets)) - 1)
    out = _empty_like_input(x, npts * N.SHAPE_SUMS, b)
    outp = b.arg(out, np.float64, writable=True)
    with b.device_guard():
        N.check(L.crimp_toa_shape_points(xp, op, nint, arr, None if auxa is None else auxa.ctypes.data,
                                         pint.ctypes.data, npp, pp, npts, outp, b.flags(), b.stream()))
    out = out.cpu().numpy() if N._is_torch(out) else out
    return out.reshape(npts, N.SHAPE_SUMS)


def toa_grid(x, offsets, tpl, norms, phis):
    """lnsum [nint, nnorm, nphi], hmin [nint, nphi] of the brute grid (fp64 accumulation)."""
    L = N.load()
    b = N.Buffers()
    xp = b.arg(x, np.float64)
    op = b.arg(offsets, np.int64)
    nint = int((offsets.numel() if N._is_torch(offsets) else np.size(offsets)) - 1)
    norms = np.asarray(norms, dtype=np.float64) if not N._is_torch(norms) else norms
    nnorm = int(norms.shape[-1])
    np_ = b.arg(norms, np.float64)
    pp = b.arg(phis, np.float64)
    nphi = int(phis.numel() if N._is_torch(phis) else np.size(phis))
    ln = _empty_like_input(x, nint * nnorm * nphi, b)
    hm = _empty_like_input(x, nint * nphi, b)
    lp = b.arg(ln, np.float64, writable=True)
    hp = b.arg(hm, np.float64, writable=True)
    with b.device_guard():
        N.check(L.crimp_toa_grid(xp, op, nint, ctypes.byref(tpl), np_, nnorm, pp, nphi, lp, hp, b.flags(), b.stream()))
    return ln.reshape(nint, nnorm, nphi), hm.reshape(nint, nphi)


TOA_BRUTE, TOA_VARY_AMPS = 1, 2


def toa_fit(x, offsets, tpl, exposure, norm0, ph_shift_res=1000, brutemin=False, vary_amps=False, flags=0):
    """Whole per-interval ToA fits on the device (crimp_toa_fit): [nint, 8] = norm, phShift, LLmax,
    phShift_LL, phShift_UL, likelihood evaluations, ampShift."""
    options = (TOA_BRUTE if brutemin else 0) | (TOA_VARY_AMPS if vary_amps else 0)
    L = N.load()
    b = N.Buffers()
    xp = b.arg(x, np.float64)
    op = b.arg(offsets, np.int64)
    ep = b.arg(exposure, np.float64)
    nint = int((offsets.numel() if N._is_torch(offsets) else np.size(offsets)) - 1)
    out = _empty_like_input(x, nint * 8, b)
    outp = b.arg(out, np.float64, writable=True)
    with b.device_guard():
        N.check(L.crimp_toa_fit(xp, op, nint, ctypes.byref(tpl), ep, float(norm0), int(ph_shift_res), options, outp,
                                b.flags(flags), b.stream()))
    return out.reshape(nint, 8)


def toa_fit_redchi2(x, offsets, tpl, exposure, norm0, ph_shift_res, brutemin, vary_amps, edges, centers, nfree,
                    flags=0, packed=False):
    """toa_fit and toa_redchi2 in one call (crimp_toa_fit_redchi2): ([nint, 8] records, [nint] redChi2), views of
    one buffer; ``packed``: that buffer itself ([9 nint]: the records, then redChi2), for a single readback."""
    options = (TOA_BRUTE if brutemin else 0) | (TOA_VARY_AMPS if vary_amps else 0)
    L = N.load()
    b = N.Buffers()
    xp = b.arg(x, np.float64)
    op = b.arg(offsets, np.int64)
    ep = b.arg(exposure, np.float64)
    eg = b.arg(edges, np.float64)
    cg = b.arg(centers, np.float64)
    nint = int((offsets.numel() if N._is_torch(offsets) else np.size(offsets)) - 1)
    nb = int((centers.numel() if N._is_torch(centers) else np.size(centers)))
    buf = _empty_like_input(x, nint * 9, b)
    out, red = buf[:nint * 8], buf[nint * 8:]
    outp = b.arg(out, np.float64, writable=True)
    redp = b.arg(red, np.float64, writable=True)
    with b.device_guard():
        N.check(L.crimp_toa_fit_redchi2(xp, op, nint, ctypes.byref(tpl), ep, float(norm0), int(ph_shift_res), options,
                                        eg, cg, nb, int(nfree), outp, redp, b.flags(flags), b.stream()))
    return buf if packed else (out.reshape(nint, 8), red)


def toa_redchi2(x, offsets, tpl, exposure, records, edges, centers, nfree):
    """redChi2 of every interval from its fit record (crimp_toa_redchi2: histogram + template curve + chi2 on the
    device, measureToAs.py:385-393); ``records`` [nint, 8] as toa_fit returns them."""
    L = N.load()
    b = N.Buffers()
    xp = b.arg(x, np.float64)
    op = b.arg(offsets, np.int64)
    ep = b.arg(exposure, np.float64)
    rp = b.arg(records, np.float64)
    eg = b.arg(edges, np.float64)
    cg = b.arg(centers, np.float64)
    nint = int((offsets.numel() if N._is_torch(offsets) else np.size(offsets)) - 1)
    nb = int((centers.numel() if N._is_torch(centers) else np.size(centers)))
    out = _empty_like_input(x, nint, b)
    outp = b.arg(out, np.float64, writable=True)
    with b.device_guard():
        N.check(L.crimp_toa_redchi2(xp, op, nint, ctypes.byref(tpl), ep, rp, eg, cg, nb, int(nfree), outp,
                                    b.flags(), b.stream()))
    return out


def binphases_counts(x, offsets, edges):
    L = N.load()
    b = N.Buffers()
    xp = b.arg(x, np.float64)
    op = b.arg(offsets, np.int64)
    ep = b.arg(edges, np.float64)
    nint = int((offsets.numel() if N._is_torch(offsets) else np.size(offsets)) - 1)
    nb = int((edges.numel() if N._is_torch(edges) else np.size(edges)) - 1)
    out = _empty_like_input(x, nint * nb, b, dtype=np.int64)
    cp = b.arg(out, np.int64, writable=True)
    with b.device_guard():
        N.check(L.crimp_binphases(xp, op, nint, ep, nb, cp, b.flags(), b.stream()))
    return out.reshape(nint, nb)


def is_sorted(t):
    """True when the times are non-decreasing (crimp_is_sorted; a NaN counts as out of order), as
    np.all(t[1:] >= t[:-1])."""
    L = N.load()
    b = N.Buffers()
    tp = b.arg(t, np.float64)
    n = int(t.numel() if N._is_torch(t) else np.size(t))
    flag = ctypes.c_int32(0)
    with b.device_guard():
        N.check(L.crimp_is_sorted(tp, n, ctypes.byref(flag), b.flags(), b.stream()))
    return flag.value == 0


def select_intervals(t, starts, ends):
    """(lo, count, first, last) per interval on time-sorted photons t (crimp_select_intervals): the photons
    t[lo : lo + count] are those of the reference's mask (t >= start) & (t <= end) (measureToAs.py:173-174), first /
    last their first and last time (NaN for an empty interval). Host NumPy arrays out; t stays where it is (a device
    tensor is searched on the device, the bounds go up with it)."""
    L = N.load()
    b = N.Buffers()
    tp = b.arg(t, np.float64)
    n = int(t.numel() if N._is_torch(t) else np.size(t))
    starts = np.ascontiguousarray(starts, dtype=np.float64).reshape(-1)
    ends = np.ascontiguousarray(ends, dtype=np.float64).reshape(-1)
    if starts.size != ends.size:
        raise ValueError("starts and ends differ in length")
    nint = int(starts.size)
    if b.device:
        import torch
        sd = torch.as_tensor(starts, device=t.device)
        ed = torch.as_tensor(ends, device=t.device)
        outi = torch.empty(2 * nint, dtype=torch.int64, device=t.device)
        outf = torch.empty(2 * nint, dtype=torch.float64, device=t.device)
        args = (b.arg(sd, np.float64), b.arg(ed, np.float64), b.arg(outi[:nint], np.int64, writable=True),
                b.arg(outi[nint:], np.int64, writable=True), b.arg(outf, np.float64, writable=True))
    else:
        outi = np.empty(2 * nint, dtype=np.int64)
        outf = np.empty(2 * nint, dtype=np.float64)
        args = (b.arg(starts, np.float64), b.arg(ends, np.float64), ctypes.c_void_p(outi.ctypes.data),
                ctypes.c_void_p(outi[nint:].ctypes.data), ctypes.c_void_p(outf.ctypes.data))
    with b.device_guard():
        N.check(L.crimp_select_intervals(tp, n, args[0], args[1], nint, args[2], args[3], args[4], b.flags(),
                                         b.stream()))
    if N._is_torch(outi):
        outi, outf = outi.cpu().numpy(), outf.cpu().numpy()
    return outi[:nint].copy(), outi[nint:].copy(), outf[0::2].copy(), outf[1::2].copy()


def gather_ranges(t, lo, offsets):
    """The photons t[lo[i] : lo[i] + (offsets[i+1] - offsets[i])] of every interval, concatenated (crimp_gather_ranges);
    same placement as t (a device tensor in, a device tensor out)."""
    L = N.load()
    b = N.Buffers()
    tp = b.arg(t, np.float64)
    n = int(t.numel() if N._is_torch(t) else np.size(t))
    lo = np.ascontiguousarray(lo, dtype=np.int64).reshape(-1)
    offsets = np.ascontiguousarray(offsets, dtype=np.int64).reshape(-1)
    nint = int(lo.size)
    if offsets.size != nint + 1:
        raise ValueError("offsets needs one entry more than lo")
    total = int(offsets[-1]) if nint else 0
    out = _empty_like_input(t, total, b)
    if b.device:
        import torch
        lp = b.arg(torch.as_tensor(lo, device=t.device), np.int64)
        op = b.arg(torch.as_tensor(offsets, device=t.device), np.int64)
    else:
        lp, op = b.arg(lo, np.int64), b.arg(offsets, np.int64)
    outp = b.arg(out, np.float64, writable=True)
    with b.device_guard():
        N.check(L.crimp_gather_ranges(tp, n, lp, op, nint, outp, b.flags(), b.stream()))
    return out

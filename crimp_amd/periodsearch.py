"""Drop-in ``PeriodSearch`` (Z^2_m and H-test) running on the MI355X.

Mirrors CRIMP v2.3.0 ``periodsearch.py`` (:20-125): the constructor keeps
``time``, ``freq``, ``nbrHarm`` and ``t0 = (time[0] + time[-1]) / 2`` (first and
last element, not min/max, :54); ``ztest()``/``htest()`` return fp64 arrays over
``freq``; ``twod_ztest(freq_dot)`` returns the (M_fd*M_f, 3) array ordered
fd-outer / f-inner with columns [Freq, Freq_dot (the log10 exponent as given),
Z2pow] plus the matching DataFrame, where ``freq_dot`` holds log10|fdot| of a
negative fdot (:95). ``twod_htest`` is this package's extension (H-test on the
same 2-D grid).

All statistics come from ``crimp_search`` (csrc/crimp_hip.hip section 4: the default
NUFFT in csrc/search_nufft.h, the exact kernel in csrc/search_exact.h, the fp64 kernel);
there is no NumPy fallback.
"""
import numpy as np

from . import ops
from ._native import STAT_H, STAT_Z2, _is_torch


class PeriodSearch:
    """``precision`` (keyword, not in the reference):

    * None (default) or "nufft": the non-uniform FFT (csrc/search_nufft.h) wherever it applies -- an ascending
      arithmetic-progression grid of >= 64 trials per row segment and time-sorted photons (the reference's own
      ``PeriodSearch(time, freq).ztest()`` on an event list and a ``np.arange``/``linspace`` grid): fp64 Chebyshev
      moments of the photons' sub-cell offsets, an fp64 FFT per moment and harmonic, O(N m P + M log M) instead of
      O(N M m); every trial certified within 1e-6 relative of the reference by a worst-case truncation bound, the
      uncertified ones recomputed in fp64. Where it declines, the "exact" rule below;
    * "exact": the exact-integer path -- on progressions of >= 256 trials per row the i8-MFMA kernel with exact
      integer sums of 2^30 fixed-point cos/sin (~1e-9 relative per trial), plus an fp64 recomputation of every trial
      that its 10-sigma error bound cannot place within 1e-6 relative; other grids take the fp64 kernel (the default
      of rounds 1-5);
    * "f64": every term in fp64 like the reference (~1e-9 relative on every trial, near-zero bins included).

    Per-trial contract of every precision: 1e-6 relative of the reference's fp64 value, except where the reference's
    own argument rounding is larger (noise-level H at config-4 arguments);
    ``crimp_last_search_path()`` tells which kernel ran."""

    def __init__(self, time, freq, nbrHarm: int = 2, *, precision=None):
        self.time = time
        self.freq = freq
        self.nbrHarm = nbrHarm
        self.precision = precision
        if _is_torch(time):
            self.t0 = float((time[0] + time[-1]).item()) / 2
        else:
            self.t0 = (self.time[0] + self.time[-1]) / 2

    def _arrays(self):
        if _is_torch(self.time):
            import torch
            t = self.time.reshape(-1).to(torch.float64).contiguous()
            f = self.freq if _is_torch(self.freq) else torch.as_tensor(np.atleast_1d(self.freq), dtype=torch.float64,
                                                                       device=t.device)
            return t, f.reshape(-1).to(torch.float64).contiguous()
        return (np.ascontiguousarray(np.ravel(self.time), dtype=np.float64),
                np.ascontiguousarray(np.atleast_1d(self.freq), dtype=np.float64).ravel())

    def _run(self, stat, freq_dot=None):
        t, f = self._arrays()
        m = int(self.nbrHarm)
        nrows = 1 if freq_dot is None else np.size(freq_dot)
        if f.shape[0] == 0 or nrows == 0:
            return np.zeros(0)
        if m <= 0:
            if stat == STAT_H:  # np.max over an empty harmonic axis (periodsearch.py:123)
                raise ValueError("zero-size array to reduction operation maximum which has no identity")
            return np.zeros(f.shape[0] * nrows)
        fd = None if freq_dot is None else np.ascontiguousarray(np.atleast_1d(freq_dot), dtype=np.float64)
        if fd is not None and _is_torch(t):
            import torch
            fd = torch.as_tensor(fd, device=t.device)
        return ops.search(t, self.t0, f, m, stat, log10_negfdot=fd, precision=self.precision)

    def ztest(self):
        """Z^2_m power at each frequency (periodsearch.py:57-71)."""
        return self._run(STAT_Z2)

    def htest(self):
        """H power at each frequency (periodsearch.py:109-125)."""
        return self._run(STAT_H)

    def _twod(self, freq_dot, stat, col):
        import pandas as pd
        fd = np.atleast_1d(np.asarray(freq_dot, dtype=np.float64))
        pw = self._run(stat, fd)
        if _is_torch(pw):
            pw = pw.cpu().numpy()
        fr = np.atleast_1d(self.freq.cpu().numpy() if _is_torch(self.freq) else np.asarray(self.freq, dtype=np.float64))
        out = np.zeros((fr.size * fd.size, 3))
        out[:, 0] = np.tile(fr, fd.size)
        out[:, 1] = np.repeat(fd, fr.size)
        out[:, 2] = pw
        return out, pd.DataFrame(out, columns=["Freq", "Freq_dot", col])

    def twod_ztest(self, freq_dot):
        """2-D Z^2 over (freq_dot outer, freq inner) (periodsearch.py:73-106)."""
        return self._twod(freq_dot, STAT_Z2, "Z2pow")

    def twod_htest(self, freq_dot):
        """2-D H-test on the twod_ztest grid (extension; same phase model as periodsearch.py:88-102)."""
        return self._twod(freq_dot, STAT_H, "Hpow")

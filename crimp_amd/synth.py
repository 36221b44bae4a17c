"""Seeded synthetic photon generators for the benchmark and test workloads.

These replace the reference's unseeded sinusoidal simulator
(`/root/reference/src/crimp/simulatemodulatedlc.py:19-96`, global RNG) with
deterministic generators whose shapes follow SURVEY.md §8(d):

* ``pulsed_events``: homogeneous Poisson arrival times over ``[0, T)`` thinned
  with acceptance ``(1 + p*cos(2*pi*phase(t) + phi0)) / (1 + p)``, where
  ``phase(t) = f0*t' + 0.5*fdot*t'**2`` and ``t'`` is measured from the middle
  of the span; returned sorted, in seconds, with an offset (default 5.0e9 s)
  that mimics MJD*86400 as ``measureToAs.py:211`` hands it to PeriodSearch.
* ``template_intervals``: ToA-interval photon phases drawn from a Fourier
  template (``templatemodels.py:64-82``) with a per-interval true shift.
"""
import numpy as np

__all__ = ["pulsed_events", "template_phases", "template_intervals"]


def pulsed_events(n, span, f0, pulsed_frac=0.1, fdot=0.0, seed=0, offset=5.0e9, phi0=0.0):
    """Return ``n`` sorted fp64 arrival times (s) of a pulsed Poisson process."""
    rng = np.random.default_rng(seed)
    n = int(n)
    out = np.empty(0, dtype=np.float64)
    mid = 0.5 * span
    while out.size < n:
        want = int((n - out.size) * (1.0 + pulsed_frac) * 1.05) + 16
        t = rng.uniform(0.0, span, size=want)
        tm = t - mid
        ph = f0 * tm + 0.5 * fdot * tm * tm
        acc = (1.0 + pulsed_frac * np.cos(2.0 * np.pi * ph + phi0)) / (1.0 + pulsed_frac)
        keep = rng.uniform(0.0, 1.0, size=want) < acc
        out = np.concatenate([out, t[keep]])
    out = out[:n]
    out.sort()
    return out + offset


def _fourier_curve(x, norm, amps, phs, shift=0.0):
    y = np.full_like(x, norm, dtype=np.float64)
    for j, (a, p) in enumerate(zip(amps, phs), start=1):
        y += a * np.cos(2.0 * np.pi * j * x + p - j * shift)
    return y


def template_phases(n, norm, amps, phs, shift, rng):
    """Draw ``n`` folded phases in [0,1) from a Fourier template shifted by ``shift`` rad."""
    amps = np.asarray(amps, dtype=np.float64)
    ymax = norm + np.sum(np.abs(amps))
    out = np.empty(0, dtype=np.float64)
    while out.size < n:
        want = int((n - out.size) * ymax / norm * 1.05) + 16
        x = rng.uniform(0.0, 1.0, size=want)
        y = rng.uniform(0.0, ymax, size=want)
        keep = y < _fourier_curve(x, norm, amps, phs, shift)
        out = np.concatenate([out, x[keep]])
    return out[:n]


def template_intervals(n_int, n_per, norm, amps, phs, seed=2):
    """Config-5 generator: ``n_int`` intervals of ``n_per`` phases each.

    Returns (x, offsets, exposure, true_shift): x is fp64 [n_int*n_per] with
    interval i occupying ``x[offsets[i]:offsets[i+1]]``; exposure = n_per/norm s
    (so the count rate matches the template norm).
    """
    rng = np.random.default_rng(seed)
    shifts = rng.uniform(-np.pi, np.pi, size=n_int)
    xs = [template_phases(n_per, norm, amps, phs, s, rng) for s in shifts]
    x = np.concatenate(xs) if xs else np.empty(0)
    offsets = np.arange(n_int + 1, dtype=np.int64) * n_per
    exposure = np.full(n_int, n_per / norm)
    return x, offsets, exposure, shifts

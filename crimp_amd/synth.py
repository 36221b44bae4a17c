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


def template_intervals_torch(n_int, n_per, norm, amps, phs, seed=2, device="cuda"):
    """Device-side version of ``template_intervals`` for large benchmark workloads (config 5):
    rejection sampling of every interval at once with torch; returns device tensors
    (x [n_int*n_per] fp64, offsets [n_int+1] int64) and host arrays (exposure, true shifts)."""
    import torch
    g = torch.Generator(device=device)
    g.manual_seed(int(seed))
    amps_t = torch.tensor(amps, dtype=torch.float64, device=device)
    phs_t = torch.tensor(phs, dtype=torch.float64, device=device)
    j = torch.arange(1, len(amps) + 1, dtype=torch.float64, device=device)
    shifts = (torch.rand(n_int, generator=g, device=device, dtype=torch.float64) * 2 - 1) * np.pi
    ymax = norm + float(np.sum(np.abs(amps)))
    out = torch.empty(n_int, n_per, dtype=torch.float64, device=device)
    step = max(1, int(2.0e8 // (2 * n_per * (len(amps) + 3))))  # bound the temporaries (~1.6 GB)
    for c0 in range(0, n_int, step):
        c1 = min(n_int, c0 + step)
        m = c1 - c0
        filled = torch.zeros(m, dtype=torch.int64, device=device)
        rows = torch.arange(m, device=device)
        sh = shifts[c0:c1]
        while int(filled.min()) < n_per:
            want = n_per * 2
            x = torch.rand(m, want, generator=g, device=device, dtype=torch.float64)
            y = torch.rand(m, want, generator=g, device=device, dtype=torch.float64) * ymax
            arg = 2 * np.pi * x[..., None] * j + phs_t - j * sh[:, None, None]
            curve = norm + (amps_t * torch.cos(arg)).sum(-1)
            keep = y < curve
            rank = torch.cumsum(keep, dim=1) - 1 + filled[:, None]
            ok = keep & (rank < n_per)
            r_idx = rows[:, None].expand(-1, want)[ok]
            out[c0:c1][r_idx, rank[ok]] = x[ok]
            filled = torch.clamp(filled + keep.sum(1), max=n_per)
            del x, y, arg, curve
    offsets = torch.arange(n_int + 1, dtype=torch.int64, device=device) * n_per
    return out.reshape(-1), offsets, np.full(n_int, n_per / norm), shifts.cpu().numpy()

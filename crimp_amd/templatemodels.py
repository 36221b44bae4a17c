"""Drop-in template models: ``Fourier``, ``WrappedCauchy``, ``VonMises``.

Mirrors CRIMP v2.3.0 ``templatemodels.py`` (:24-329). The unbinned extended
log-likelihoods -- the ToA-scan hot path -- run on the MI355X through
``crimp_toa_points`` (fp64 sums over the photons); the curve methods and the
binned Gaussian likelihoods (template building, outside the hot path, <=10^2
bins) are evaluated on the host.

``theta`` may be a plain dict or any mapping whose values convert with
``float()`` (e.g. lmfit Parameters), keyed norm, ampShift, phShift and amp_j with
ph_j (Fourier) or cen_j, wid_j (Cauchy / von Mises); components are counted from
the keys starting with ``amp_`` as the reference does (:71, :173, :278).
"""
import math

import numpy as np

from . import ops
from ._native import _is_torch

TWO_PI = 2.0 * math.pi


def _f(theta, key, default=None):
    if key not in theta:
        if default is None:
            raise KeyError(key)
        return default
    return float(theta[key])


def _ncomp(theta):
    return len([k for k in theta.keys() if k.startswith("amp_")])


def _sorted(xx):
    if _is_torch(xx):
        return xx.reshape(-1).sort().values
    return np.sort(np.asarray(xx))


def template_from_theta(model, theta):
    """crimp_template for a theta mapping (model in fourier/cauchy/vonmises)."""
    K = _ncomp(theta)
    amps = [_f(theta, "amp_%d" % j) for j in range(1, K + 1)]
    if model == "fourier":
        locs = [_f(theta, "ph_%d" % j) for j in range(1, K + 1)]
        wids = None
    else:
        locs = [_f(theta, "cen_%d" % j) for j in range(1, K + 1)]
        wids = [_f(theta, "wid_%d" % j) for j in range(1, K + 1)]
    return ops.make_template(model, amps, locs, wids, amp_shift=_f(theta, "ampShift", 1.0))


def _extended_ll(model, theta, xx, exposure):
    """Reference extended LL from the device sums at one (norm, phShift) point."""
    n = _f(theta, "norm")
    phi = _f(theta, "phShift", 0.0)
    tpl = template_from_theta(model, theta)
    if _is_torch(xx):
        import torch
        x = xx.reshape(-1).to(torch.float64).contiguous()
        dev = x.device
        off = torch.tensor([0, x.numel()], dtype=torch.int64, device=dev)
        s = ops.toa_points(x, off, tpl, torch.zeros(1, dtype=torch.int64, device=dev),
                           torch.tensor([n], dtype=torch.float64, device=dev),
                           torch.tensor([phi], dtype=torch.float64, device=dev)).cpu().numpy()[0]
    else:
        x = np.ascontiguousarray(np.ravel(xx), dtype=np.float64)
        s = ops.toa_points(x, np.array([0, x.size], dtype=np.int64), tpl, np.zeros(1, dtype=np.int64),
                           np.array([n]), np.array([phi]))[0]
    N = s[7]
    if model == "fourier":
        F = n
    else:
        F = TWO_PI * n + sum(tpl.amp[j] * tpl.amp_shift for j in range(tpl.ncomp))
    if not (s[6] / F > 0):  # min(model/normalisation) <= 0 -> -inf (:113-115, :220-222, :324-326)
        return -np.inf
    if model == "fourier":
        return -n * exposure + N * np.log(n * exposure) + (s[0] - N * np.log(n))
    return -F * exposure / TWO_PI + N * np.log(F * exposure / TWO_PI) + (s[0] - N * np.log(F))


def _gauss_ll(yy, model, yy_err):
    from scipy import stats
    return np.sum(stats.norm.logpdf(yy, loc=model, scale=yy_err))


class Fourier:
    """Fourier-series template (templatemodels.py:24-121)."""

    def __init__(self, theta, xx):
        self.theta = theta
        self.xx = _sorted(xx)

    def fourseries(self):
        x = np.asarray(self.xx.cpu().numpy() if _is_torch(self.xx) else self.xx)
        curve = _f(self.theta, "norm")
        a = _f(self.theta, "ampShift", 1.0)
        sh = _f(self.theta, "phShift", 0.0)
        for j in range(1, _ncomp(self.theta) + 1):
            curve = curve + (_f(self.theta, "amp_%d" % j) * a *
                             np.cos(j * 2 * np.pi * x + _f(self.theta, "ph_%d" % j) - j * sh))
        return curve

    def loglikelihoodFS(self, yy, yy_err):
        return _gauss_ll(yy, Fourier(self.theta, self.xx).fourseries(), yy_err)

    def loglikelihoodFSnormalized(self, exposure):
        return _extended_ll("fourier", self.theta, self.xx, float(exposure))


class WrappedCauchy:
    """Wrapped-Cauchy template, x in radians (templatemodels.py:124-226)."""

    def __init__(self, theta, xx):
        self.theta = theta
        self.xx = _sorted(xx)

    def wrapcauchy(self):
        x = np.asarray(self.xx.cpu().numpy() if _is_torch(self.xx) else self.xx)
        curve = _f(self.theta, "norm")
        a = _f(self.theta, "ampShift", 1.0)
        sh = _f(self.theta, "phShift", 0.0)
        for j in range(1, _ncomp(self.theta) + 1):
            w = _f(self.theta, "wid_%d" % j)
            curve = curve + ((_f(self.theta, "amp_%d" % j) * a) / (2 * np.pi)) * (
                np.sinh(w) / (np.cosh(w) - np.cos(x - _f(self.theta, "cen_%d" % j) - sh)))
        return curve

    def loglikelihoodCA(self, yy, yy_err):
        return _gauss_ll(yy, WrappedCauchy(self.theta, self.xx).wrapcauchy(), yy_err)

    def loglikelihoodCAnormalized(self, exposure):
        return _extended_ll("cauchy", self.theta, self.xx, float(exposure))


class VonMises:
    """von Mises template, x in radians (templatemodels.py:229-329)."""

    def __init__(self, theta, xx):
        self.theta = theta
        self.xx = _sorted(xx)

    def vonmises(self):
        from scipy.special import i0
        x = np.asarray(self.xx.cpu().numpy() if _is_torch(self.xx) else self.xx)
        curve = _f(self.theta, "norm")
        a = _f(self.theta, "ampShift", 1.0)
        sh = _f(self.theta, "phShift", 0.0)
        for j in range(1, _ncomp(self.theta) + 1):
            k = 1 / _f(self.theta, "wid_%d" % j) ** 2
            curve = curve + ((_f(self.theta, "amp_%d" % j) * a) / (2 * np.pi * i0(k))) * np.exp(
                k * np.cos(x - _f(self.theta, "cen_%d" % j) - sh))
        return curve

    def loglikelihoodVM(self, yy, yy_err):
        return _gauss_ll(yy, VonMises(self.theta, self.xx).vonmises(), yy_err)

    def loglikelihoodVMnormalized(self, exposure):
        return _extended_ll("vonmises", self.theta, self.xx, float(exposure))

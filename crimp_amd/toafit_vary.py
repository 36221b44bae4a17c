"""ToA fits with template parameters freed by their ``vary`` flags (``readvaryparam=True``).

Restates CRIMP v2.3.0 ``measureToAs.py:727-801`` (``defineinitialfitparam(readvaryparam=True)``)
with the drivers of ``:285-403`` / ``:437-548`` / ``:582-693``: norm in [norm/5, 5 norm] (free if
the template says so), every template parameter whose ``vary`` flag is True free within the
reference's bounds (Fourier amp [0, 1000], ph [-pi, pi]; Cauchy / von Mises amp [0, 5 amp],
cen +- 0.6, wid [0, 30 pi]), phShift free in [-pi, pi] (Fourier) or [-1.5 pi, 1.5 pi], ampShift 1.
As for the default fit, the optimum replaces lmfit's Nelder-Mead iterate: bounded L-BFGS-B on the
extended LL with its exact gradient, whose photon sums come from the device in one pass per
evaluation (``crimp_toa_shape_points``); the 1-sigma scan re-maximises every other free parameter
at each phShift step, starting from the best fit as the reference does (``initParam_forErrCalc``
is a copy of the best-fit parameters, :319), and redChi2 counts the free parameters the way
:733-748 does (norm and the freed template parameters -- not phShift).

Deviation: with ``brutemin`` the reference hands every free parameter to lmfit's brute grid (20
points per bounded parameter without a ``brute_step``: 20^k x 126 evaluations). Here the brute start
is the (norm, phShift) grid of the default path with the template's shape, then the full local
maximisation.
"""
import math

import numpy as np

from . import ops
from . import _native as N
from .toafit import CHI2_1SIG_1DOF, TWO_PI, ToAFitter


class VaryParamFitter(ToAFitter):
    """readvaryparam fits of every interval of one concatenated folded-phase array."""

    def __init__(self, x, offsets, exposure, tmpl, ph_shift_res=1000, nbr_bins=15, device=None):
        super().__init__(x, offsets, exposure, tmpl, ph_shift_res, nbr_bins, device)
        K, m = self.K, self.model
        names, val, lo, hi, vary = ["norm"], [self.norm0], [self.norm0 / 5], [self.norm0 * 5], [bool(tmpl["norm"]["vary"])]
        for k in range(1, K + 1):
            a = float(tmpl["amp_%d" % k]["value"])
            if m == "fourier":
                rows = [("amp_%d" % k, a, 0.0, 1000.0), ("ph_%d" % k, float(tmpl["ph_%d" % k]["value"]), -math.pi, math.pi)]
            else:
                c = float(tmpl["cen_%d" % k]["value"])
                rows = [("amp_%d" % k, a, 0.0, 5 * a), ("cen_%d" % k, c, -0.6 + c, 0.6 + c),
                        ("wid_%d" % k, float(tmpl["wid_%d" % k]["value"]), 0.0, 30 * math.pi)]
            for nm, v, l, h in rows:
                names.append(nm)
                val.append(v)
                lo.append(l)
                hi.append(h)
                vary.append(bool(tmpl[nm]["vary"]))
        names.append("phShift")
        val.append(0.0)
        lo.append(-self.pb)
        hi.append(self.pb)
        vary.append(True)
        self.names = names
        self.blo, self.bhi = np.array(lo), np.array(hi)
        self.theta0 = np.clip(np.array(val), self.blo, self.bhi)   # lmfit clips values into their bounds
        self.vary = np.array(vary)
        # redChi2 dof (:733-748): norm if free + the freed template parameters; phShift is not counted
        self.nfree = int(self.vary[:-1].sum())
        self.evals = np.zeros(self.nint, dtype=np.int64)

    # ------------------------------------------------------------------ one batch of evaluations
    def _template(self, th):
        K = self.K
        if self.model == "fourier":
            amps, locs, wids = th[1:1 + 2 * K:2], th[2:2 + 2 * K:2], None
        else:
            amps, locs, wids = th[1:1 + 3 * K:3], th[2:2 + 3 * K:3], th[3:3 + 3 * K:3]
        return ops.make_template(self.model, amps, locs, wids, 1.0), amps, wids

    def evaluate_theta(self, iv, thetas):
        """LL and its gradient over the full parameter vector at (interval, theta) points."""
        iv = np.asarray(iv, dtype=np.int64).reshape(-1)
        thetas = np.asarray(thetas, dtype=np.float64).reshape(iv.size, -1)
        K = self.K
        tpls, amp_sum, aux = [], np.zeros(iv.size), None
        if self.model == "vonmises":
            from scipy.special import i0e, i1e
            aux = np.zeros((iv.size, N.MAX_COMP))
        for p, th in enumerate(thetas):
            t, amps, wids = self._template(th)
            tpls.append(t)
            amp_sum[p] = np.sum(amps)
            if aux is not None:
                kap = 1.0 / np.asarray(wids) ** 2
                aux[p, :K] = i1e(kap) / i0e(kap)
        n, phi = thetas[:, 0], thetas[:, -1]
        s = ops.toa_shape_points(self.x, self.offsets, tpls, iv, n, phi, aux)
        np.add.at(self.evals, iv, 1)
        Np, E = self.N[iv], self.E[iv]
        g = np.zeros_like(thetas)
        g[:, 0] = -E + s[:, 2]
        g[:, -1] = s[:, 3]
        step = 2 if self.model == "fourier" else 3
        for j in range(K):
            for c in range(step):
                g[:, 1 + step * j + c] = s[:, 4 + 3 * j + c]
        with np.errstate(divide="ignore", invalid="ignore"):
            if self.model == "fourier":
                ll = -n * E + Np * np.log(n * E) + (s[:, 0] - Np * np.log(n))
                ok = s[:, 1] / n > 0
            else:
                F = TWO_PI * n + amp_sum
                ll = -F * E / TWO_PI + Np * np.log(F * E / TWO_PI) + (s[:, 0] - Np * np.log(F))
                ok = s[:, 1] / F > 0
                g[:, 1:1 + 3 * K:3] -= (E / TWO_PI)[:, None]   # dF/damp_j = 1 (ampShift 1)
        ll = np.where(ok, ll, -np.inf)
        return ll, g

    # ------------------------------------------------------------------ maximisation
    def _maximise(self, i, theta_start, free, max_iter=200):
        """Bounded maximum over the ``free`` mask for interval i: projected Newton ascent with the exact
        gradient and a forward-difference Hessian of it (all n+1 points in one device launch),
        eigenvalue-shifted when not negative definite, backtracking line search on the LL."""
        th = theta_start.copy()
        idx = np.nonzero(free)[0]
        lo, hi = self.blo[idx], self.bhi[idx]
        z = np.clip(th[idx], lo, hi)
        nz = idx.size

        def at(zz):
            t = th.copy()
            t[idx] = zz
            return t

        if nz == 0:
            ll, _ = self.evaluate_theta([i], th[None, :])
            return th, float(ll[0])
        ll0, g0 = self.evaluate_theta([i], at(z)[None, :])
        f, g = float(ll0[0]), g0[0, idx]
        if not np.isfinite(f):
            raise FloatingPointError("readvaryparam: the starting template gives a non-positive model")
        small = 0
        for _ in range(max_iter):
            h = 1e-6 * np.maximum(1.0, np.abs(z))
            # step inward at an upper bound so that the difference stays inside the box
            h = np.where(z + h > hi, -h, h)
            pts = np.repeat(at(z)[None, :], nz, axis=0)
            pts[np.arange(nz), idx] += h
            _, gp = self.evaluate_theta(np.full(nz, i), pts)
            H = (gp[:, idx] - g[None, :]) / h[:, None]
            H = 0.5 * (H + H.T)
            # active bounds (maximisation): at lo with g < 0, or at hi with g > 0
            act = ((z <= lo) & (g < 0)) | ((z >= hi) & (g > 0))
            fr = ~act
            d = np.zeros(nz)
            if fr.any():
                Hf = H[np.ix_(fr, fr)]
                w = np.linalg.eigvalsh(Hf)
                if w.max() >= 0:
                    Hf = Hf - (w.max() + 1e-8 * max(1.0, abs(w.min()))) * np.eye(fr.sum())
                d[fr] = -np.linalg.solve(Hf, g[fr])
            slope = float(g @ d)
            t, accepted = 1.0, False
            for _ls in range(60):
                zn = np.clip(z + t * d, lo, hi)
                lln, gn = self.evaluate_theta([i], at(zn)[None, :])
                if np.isfinite(lln[0]) and lln[0] >= f + 1e-4 * t * max(slope, 0.0):
                    accepted = True
                    break
                t *= 0.5
            if not accepted:
                break
            df = float(lln[0]) - f
            z, f, g = zn, float(lln[0]), gn[0, idx]
            step = np.max(np.abs(t * d) / np.maximum(1.0, np.abs(z)))
            small = small + 1 if (df <= 1e-11 * max(1.0, abs(f)) and step < 1e-9) else 0
            if small >= 2 or step < 1e-14:
                break
        th[idx] = z
        return th, f

    def fit(self, brutemin=False):
        if brutemin:
            n0, p0 = self.brute()
        else:
            n0, p0 = np.full(self.nint, self.norm0), np.zeros(self.nint)
        theta_hat = np.tile(self.theta0, (self.nint, 1))
        ll_max = np.zeros(self.nint)
        for i in range(self.nint):
            start = self.theta0.copy()
            start[0], start[-1] = np.clip(n0[i], self.blo[0], self.bhi[0]), p0[i]
            theta_hat[i], ll_max[i] = self._maximise(i, start, self.vary)
        lo_err, up_err = self._scan(theta_hat, ll_max)
        rchi2 = self._reduced_chi2_theta(theta_hat)
        return {"phShi": theta_hat[:, -1].copy(), "phShi_LL": lo_err, "phShi_UL": up_err, "reducedChi2": rchi2,
                "norm": theta_hat[:, 0].copy(), "LLmax": ll_max, "theta": theta_hat, "names": list(self.names),
                "evaluations": self.evals.copy(), "ampShift": np.ones(self.nint)}

    # ------------------------------------------------------------------ 1-sigma scan
    def _scan(self, theta_hat, ll_max):
        step = TWO_PI / self.res
        kcap = self.res / 2.0
        free = self.vary.copy()
        free[-1] = False
        out = {}
        for side in (-1, 1):
            res = np.zeros(self.nint)
            for i in range(self.nint):
                passed = np.zeros(1, dtype=bool)
                k = 1
                while True:
                    ks = np.array([k])
                    phi = self._scan_phases(theta_hat[i:i + 1, -1], side, ks, passed)[0, 0]
                    tg = theta_hat[i, -1] + side * k * step
                    passed |= (tg <= -math.pi) if side < 0 else (tg >= math.pi)
                    start = theta_hat[i].copy()
                    start[-1] = phi          # fixed (phShift is not among the re-maximised parameters)
                    _, llk = self._maximise(i, start, free)
                    k += 1
                    if ll_max[i] - llk > CHI2_1SIG_1DOF or k > kcap:
                        break
                res[i] = k * step + step / 2
            out[side] = res
        return out[-1], out[1]

    # ------------------------------------------------------------------ redChi2
    def _reduced_chi2_theta(self, theta_hat):
        upper = 1.0 if self.model == "fourier" else TWO_PI
        edges = np.linspace(0, upper, self.nbins + 1, endpoint=True)
        cts = ops.binphases_counts(self.x, self.offsets, self._arr(edges, np.float64))
        cts = np.asarray(cts.cpu().numpy() if hasattr(cts, "cpu") else cts, dtype=np.float64)
        pp = np.linspace(0, upper, self.nbins, endpoint=False) + (upper / self.nbins) / 2
        out = np.zeros(self.nint)
        saved = self.tpl
        for i in range(self.nint):
            self.tpl = self._template(theta_hat[i])[0]
            model = self.curve(theta_hat[i, 0], theta_hat[i, -1], pp)
            rate = cts[i] / (self.E[i] / self.nbins)
            err = np.sqrt(cts[i]) / (self.E[i] / self.nbins)
            with np.errstate(divide="ignore", invalid="ignore"):
                out[i] = np.divide(np.sum(np.divide((model - rate) ** 2, err ** 2)), self.nbins - self.nfree)
        self.tpl = saved
        return out

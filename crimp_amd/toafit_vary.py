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

``varyAmps`` together with ``readvaryparam`` (:306-312 after :727-801): once the freed parameters are fitted,
ampShift (a common factor on every template amplitude) is freed from 1 within its model's bounds (Fourier
[0.01, 100] :308, Cauchy [0, inf) :461, von Mises [0, 500] :605) and everything free is
maximised again; the 1-sigma scan then re-maximises ampShift too, and redChi2 counts one more free parameter.
The parameter vector is then [norm, template..., ampShift, phShift].

``brutemin`` (:292-295): lmfit's brute over every free parameter -- 20 points on [min, max] for each bounded
parameter without a ``brute_step`` (norm, amp_k, ph_k, wid_k), steps of 0.05 for cen_k and phShift -- and its first
maximum in C order of the parameters (norm, template parameters in insertion order, phShift). Each template of the
lattice is one device brute-grid launch (``crimp_toa_grid``: every norm x phShift of every interval), so up to
``BRUTE_MAX_TEMPLATE_PARAMS`` = 2 freed template parameters (<= 625 templates) are covered exactly; with more the
start is the (norm, phShift) lattice at the template's values (a documented deviation). Lattice points whose LL is
not finite (a von Mises width of 0) are skipped. Parity unpinned: lmfit (absent) aborts brute after
max_nfev = 1e4 evaluations (:294), which any lattice with a freed template parameter exceeds, and the point it then
hands to Nelder-Mead depends on the lmfit version; the oracle restates the lattice maximum (oracle.readvary_brute).
"""
import math

import numpy as np

from . import ops
from . import _native as N
from ._native import _is_torch
from .toafit import CHI2_1SIG_1DOF, TWO_PI, ToAFitter

# ampShift bounds when varyAmps frees it: measureToAs.py:308 (Fourier), :461 (Cauchy), :605 (von Mises)
AMP_SHIFT_BOUNDS = {"fourier": (0.01, 100.0), "cauchy": (0.0, math.inf), "vonmises": (0.0, 500.0)}
BRUTE_MAX_TEMPLATE_PARAMS = 2   # freed template parameters the full brute lattice covers (20^k templates)


def mgrid_axis(lo, hi, step=None, ns=20):
    """One axis of lmfit's brute lattice as scipy.optimize.brute builds it with np.mgrid: ``slice(lo, hi, step)``
    (arange semantics, hi excluded) for a parameter with a ``brute_step``, ``slice(lo, hi, complex(Ns))`` (Ns
    points, both bounds included) otherwise (lmfit Minimizer.brute, Ns = 20)."""
    if step is None:
        return np.mgrid[slice(lo, hi, complex(ns))]
    return np.mgrid[slice(lo, hi, step)]


class VaryParamFitter(ToAFitter):
    """readvaryparam fits of every interval of one concatenated folded-phase array."""

    def __init__(self, x, offsets, exposure, tmpl, ph_shift_res=1000, nbr_bins=15, device=None, vary_amps=False):
        super().__init__(x, offsets, exposure, tmpl, ph_shift_res, nbr_bins, device)
        self.vary_amps = bool(vary_amps)
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
        if self.vary_amps:  # measureToAs.py:308, :461, :605: ampShift 1 in its model's bounds, freed after the first fit
            alo, ahi = AMP_SHIFT_BOUNDS[m]
            names.append("ampShift")
            val.append(1.0)
            lo.append(alo)
            hi.append(ahi)
            vary.append(False)
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
    def _amp_shift(self, th):
        return float(th[-2]) if self.vary_amps else 1.0

    def _template(self, th):
        """Device template of a parameter vector (amplitudes times ampShift), its amplitudes and widths."""
        K = self.K
        if self.model == "fourier":
            amps, locs, wids = th[1:1 + 2 * K:2], th[2:2 + 2 * K:2], None
        else:
            amps, locs, wids = th[1:1 + 3 * K:3], th[2:2 + 3 * K:3], th[3:3 + 3 * K:3]
        A = self._amp_shift(th)
        return ops.make_template(self.model, np.asarray(amps) * A, locs, wids, 1.0), amps, wids

    def evaluate_theta(self, iv, thetas):
        """LL and its gradient over the full parameter vector at (interval, theta) points."""
        iv = np.asarray(iv, dtype=np.int64).reshape(-1)
        thetas = np.asarray(thetas, dtype=np.float64).reshape(iv.size, -1)
        K = self.K
        tpls, amp_sum, aux = [], np.zeros(iv.size), None
        if self.model == "vonmises":
            from scipy.special import i0e, i1e
            aux = np.zeros((iv.size, N.MAX_COMP))
        A = np.array([self._amp_shift(th) for th in thetas])
        for p, th in enumerate(thetas):
            t, amps, wids = self._template(th)
            tpls.append(t)
            amp_sum[p] = np.sum(amps) * A[p]
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
        # the device sums are gradients in the effective amplitudes amp_j * ampShift
        ga = g[:, 1:1 + step * K:step].copy()
        if self.model != "fourier":
            ga -= (E / TWO_PI)[:, None]                     # dF/d(amp_j ampShift) = 1
        with np.errstate(divide="ignore", invalid="ignore"):
            if self.model == "fourier":
                ll = -n * E + Np * np.log(n * E) + (s[:, 0] - Np * np.log(n))
                ok = s[:, 1] / n > 0
            else:
                F = TWO_PI * n + amp_sum
                ll = -F * E / TWO_PI + Np * np.log(F * E / TWO_PI) + (s[:, 0] - Np * np.log(F))
                ok = s[:, 1] / F > 0
        g[:, 1:1 + step * K:step] = ga * A[:, None]
        if self.vary_amps:
            g[:, -2] = np.sum(ga * thetas[:, 1:1 + step * K:step], axis=1)
        ll = np.where(ok, ll, -np.inf)
        return ll, g

    # ------------------------------------------------------------------ maximisation
    def _maximise(self, i, theta_start, free, max_iter=200):
        """Bounded maximum over the ``free`` mask for interval i (one-interval form of _maximise_batch)."""
        th, ll = self._maximise_batch(np.array([i]), theta_start[None, :], free, max_iter)
        return th[0], float(ll[0])

    def _maximise_batch(self, ivs, starts, free, max_iter=200):
        """Bounded maxima over the ``free`` mask, one per (interval, start) row: projected Newton ascent with
        the exact gradient and a forward-difference Hessian of it, eigenvalue-shifted when not negative
        definite, backtracking line search on the LL. The intervals iterate in lockstep so that every
        Hessian stage and every line-search trial of all still-active intervals is one device launch; each
        interval's own sequence of evaluation points (hence its result) is the one-interval iteration's."""
        ivs = np.asarray(ivs, dtype=np.int64).reshape(-1)
        th = np.array(starts, dtype=np.float64).reshape(ivs.size, -1)
        B = ivs.size
        idx = np.nonzero(free)[0]
        nz = idx.size
        if nz == 0:
            ll, _ = self.evaluate_theta(ivs, th)
            return th, ll
        lo, hi = self.blo[idx], self.bhi[idx]
        Z = np.clip(th[:, idx], lo, hi)

        def at(rows, zz):
            t = th[rows].copy()
            t[:, idx] = zz
            return t

        ll0, g0 = self.evaluate_theta(ivs, at(np.arange(B), Z))
        F, G = ll0.astype(np.float64), g0[:, idx]
        if not np.all(np.isfinite(F)):
            raise FloatingPointError("readvaryparam: the starting template gives a non-positive model")
        small = np.zeros(B, dtype=np.int64)
        active = np.ones(B, dtype=bool)
        for _ in range(max_iter):
            A = np.nonzero(active)[0]
            if A.size == 0:
                break
            # forward-difference Hessian points of every active interval, one launch
            hs = np.empty((A.size, nz))
            pts = np.empty((A.size * nz, th.shape[1]))
            for p, b in enumerate(A):
                h = 1e-6 * np.maximum(1.0, np.abs(Z[b]))
                h = np.where(Z[b] + h > hi, -h, h)   # step inward at an upper bound
                P = np.repeat(at([b], Z[b][None, :]), nz, axis=0)
                P[np.arange(nz), idx] += h
                pts[p * nz:(p + 1) * nz] = P
                hs[p] = h
            _, gp = self.evaluate_theta(np.repeat(ivs[A], nz), pts)
            Dm = np.zeros((A.size, nz))
            slope = np.zeros(A.size)
            for p, b in enumerate(A):
                z, g = Z[b], G[b]
                H = (gp[p * nz:(p + 1) * nz][:, idx] - g[None, :]) / hs[p][:, None]
                H = 0.5 * (H + H.T)
                # active bounds (maximisation): at lo with g < 0, or at hi with g > 0
                act = ((z <= lo) & (g < 0)) | ((z >= hi) & (g > 0))
                fr = ~act
                if fr.any():
                    Hf = H[np.ix_(fr, fr)]
                    w = np.linalg.eigvalsh(Hf)
                    if w.max() >= 0:
                        Hf = Hf - (w.max() + 1e-8 * max(1.0, abs(w.min()))) * np.eye(fr.sum())
                    Dm[p, fr] = -np.linalg.solve(Hf, g[fr])
                slope[p] = float(g @ Dm[p])
            # backtracking line search, all pending intervals' trial points in one launch
            t = np.ones(A.size)
            accepted = np.zeros(A.size, dtype=bool)
            ZN, LLN, GN = np.empty((A.size, nz)), np.empty(A.size), np.empty((A.size, nz))
            for _ls in range(60):
                Pn = np.nonzero(~accepted)[0]
                if Pn.size == 0:
                    break
                zn = np.clip(Z[A[Pn]] + t[Pn, None] * Dm[Pn], lo, hi)
                lln, gn = self.evaluate_theta(ivs[A[Pn]], at(A[Pn], zn))
                ok = np.isfinite(lln) & (lln >= F[A[Pn]] + 1e-4 * t[Pn] * np.maximum(slope[Pn], 0.0))
                for k, p in enumerate(Pn):
                    if ok[k]:
                        accepted[p] = True
                        ZN[p], LLN[p], GN[p] = zn[k], lln[k], gn[k, idx]
                    else:
                        t[p] *= 0.5
            for p, b in enumerate(A):
                if not accepted[p]:
                    active[b] = False
                    continue
                df = float(LLN[p]) - F[b]
                Z[b], F[b], G[b] = ZN[p], LLN[p], GN[p]
                step = np.max(np.abs(t[p] * Dm[p]) / np.maximum(1.0, np.abs(Z[b])))
                small[b] = small[b] + 1 if (df <= 1e-11 * max(1.0, abs(F[b])) and step < 1e-9) else 0
                if small[b] >= 2 or step < 1e-14:
                    active[b] = False
        th[:, idx] = Z
        return th, F

    def brute_lattice(self):
        """Start vectors [nint, len(theta)] from lmfit's brute lattice over every free parameter (module docstring),
        or None when more than BRUTE_MAX_TEMPLATE_PARAMS template parameters are free."""
        import itertools
        names, th0 = self.names, self.theta0
        tp = [i for i in range(1, len(names) - 1) if self.vary[i] and names[i] != "ampShift"]
        if len(tp) > BRUTE_MAX_TEMPLATE_PARAMS:
            return None
        axes = [mgrid_axis(self.blo[i], self.bhi[i], 0.05 if names[i].startswith("cen_") else None) for i in tp]
        norms = mgrid_axis(self.blo[0], self.bhi[0]) if self.vary[0] else np.array([th0[0]])
        phis = mgrid_axis(-self.pb, self.pb, 0.05)
        combos = list(itertools.product(*axes))
        nn, nc, nphi = norms.size, len(combos), phis.size
        ll = np.full((self.nint, nn, nc, nphi), -np.inf)
        Np, E = self.N[:, None, None], self.E[:, None, None]
        nv = norms[None, :, None]
        step = 2 if self.model == "fourier" else 3
        for c, combo in enumerate(combos):
            th = th0.copy()
            th[tp] = combo
            if self.model == "vonmises" and np.any(th[3:3 + 3 * self.K:3] <= 0):
                continue                      # width 0: I0(1/w^2) overflows, the reference's LL is NaN there
            tpl, amps, _ = self._template(th)
            ln, hmin = ops.toa_grid(self.x, self.offsets, tpl, self._arr(np.tile(norms, (self.nint, 1)), np.float64),
                                    self._arr(phis, np.float64))
            if _is_torch(ln):
                ln, hmin = ln.cpu().numpy(), hmin.cpu().numpy()
            with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
                if self.model == "fourier":
                    v = -nv * E + Np * np.log(nv * E) + (ln - Np * np.log(nv))
                else:
                    F = TWO_PI * nv + float(np.sum(th[1:1 + step * self.K:step]))
                    v = -F * E / TWO_PI + Np * np.log(F * E / TWO_PI) + (ln - Np * np.log(F))
                valid = (hmin[:, None, :] + nv) > 0
            ll[:, :, c, :] = np.where(valid & np.isfinite(v), v, -np.inf)
        flat = ll.reshape(self.nint, -1)
        idx = np.argmax(flat, axis=1)                                 # first maximum in C order (np.argmin of -LL)
        a, c, b = np.unravel_index(idx, (nn, nc, nphi))
        starts = np.tile(th0, (self.nint, 1))
        starts[:, 0] = norms[a]
        for i in range(self.nint):
            starts[i, tp] = combos[c[i]]
        starts[:, -1] = phis[b]
        return starts

    def fit(self, brutemin=False):
        if self.vary_amps:  # ampShift is fixed at 1 for the first fit
            self.vary[-2] = False
        self.nfree = int(self.vary[:-1].sum())
        starts = self.brute_lattice() if brutemin else None
        if starts is None:
            if brutemin:    # more free template parameters than the lattice covers: the (norm, phShift) lattice
                n0, p0 = self.brute()
            else:
                n0, p0 = np.full(self.nint, self.norm0), np.zeros(self.nint)
            starts = np.tile(self.theta0, (self.nint, 1))
            starts[:, 0] = np.clip(n0, self.blo[0], self.bhi[0])
            starts[:, -1] = p0
        theta_hat, ll_max = self._maximise_batch(np.arange(self.nint), starts, self.vary)
        if self.vary_amps:  # measureToAs.py:306-312: free ampShift from 1 and refit everything free
            self.vary[-2] = True
            self.nfree += 1
            theta_hat[:, -2] = 1.0
            theta_hat, ll_max = self._maximise_batch(np.arange(self.nint), theta_hat, self.vary)
        lo_err, up_err = self._scan(theta_hat, ll_max)
        rchi2 = self._reduced_chi2_theta(theta_hat)
        return {"phShi": theta_hat[:, -1].copy(), "phShi_LL": lo_err, "phShi_UL": up_err, "reducedChi2": rchi2,
                "norm": theta_hat[:, 0].copy(), "LLmax": ll_max, "theta": theta_hat, "names": list(self.names),
                "evaluations": self.evals.copy(),
                "ampShift": theta_hat[:, -2].copy() if self.vary_amps else np.ones(self.nint)}

    # ------------------------------------------------------------------ 1-sigma scan
    def _scan(self, theta_hat, ll_max):
        step = TWO_PI / self.res
        kcap = self.res / 2.0
        free = self.vary.copy()
        free[-1] = False
        out = {}
        for side in (-1, 1):
            # every interval steps k = 1, 2, ... in lockstep; each step's re-maximisations are one batch
            res = np.zeros(self.nint)
            k = np.ones(self.nint, dtype=np.int64)
            passed = np.zeros(self.nint, dtype=bool)
            going = np.ones(self.nint, dtype=bool)
            while going.any():
                A = np.nonzero(going)[0]
                starts = theta_hat[A].copy()
                for p, i in enumerate(A):
                    pa = passed[i:i + 1].copy()
                    starts[p, -1] = self._scan_phases(theta_hat[i:i + 1, -1], side, k[i:i + 1], pa)[0, 0]
                    tg = theta_hat[i, -1] + side * k[i] * step
                    passed[i] |= (tg <= -math.pi) if side < 0 else (tg >= math.pi)
                # phShift fixed (not among the re-maximised parameters)
                _, llk = self._maximise_batch(A, starts, free)
                k[A] += 1
                stop = (ll_max[A] - llk > CHI2_1SIG_1DOF) | (k[A] > kcap)
                going[A[stop]] = False
            res[:] = k * step + step / 2
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

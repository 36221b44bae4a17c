"""Batched ToA phase-shift fits on the MI355X (the measureToA_* driver).

Restates, for every ToA interval at once, what CRIMP v2.3.0
``measureToAs.py:254-403`` (Fourier), ``:406-548`` (Cauchy) and ``:551-693``
(von Mises) do with lmfit, targeting the same optimum rather than lmfit's
iterates:

1. optional brute grid (``-bm``): lmfit's ``brute`` over norm x phShift with
   scipy's ``mgrid`` lattices -- 20 norms on [norm0/100, 500] and phShift =
   k*0.05 - bound (126 points for Fourier, 189 for Cauchy / von Mises), LL on the
   device (``crimp_toa_grid``, fp32 model/log, fp64 sums), first maximum in
   norm-outer order as scipy.optimize.brute picks it;
2. the local maximum of the extended LL in (norm, phShift) from the brute point
   (or from (norm0, 0) without ``-bm``, where lmfit starts Nelder-Mead): a damped
   2-D Newton ascent on fp64 device sums (``crimp_toa_points``: LL, gradient and
   Hessian in one pass over the photons);
3. the 1-sigma scan: phShift = best -/+ k*2*pi/phShiftRes with lmfit's clip-to-
   bound behaviour, norm re-profiled (1-D Newton) at every step, stop at the first
   LLmax - LL > 0.5*chi2.ppf(0.6827, 1); sigma = (k+1)*step + step/2, capped at
   phShiftRes/2 steps (:330-376);
4. redChi2 from the ``binphases`` profile (numpy.histogram edge semantics) against
   the best-fit curve, dof = nbrBins - 2 (:385-393), on the device from the fit
   records (``crimp_toa_redchi2``).

``varyAmps`` (a free ampShift, :305-312) runs on the device too (``k_toa_fit_amp``: (norm, ampShift)
re-profiled at every scan step); ``readvaryparam`` (free template parameters, :727-801) is driven from
``toafit_vary.py`` on device likelihood/gradient sums.
"""
import math

import numpy as np

from . import ops
from ._native import _is_torch

CHI2_1SIG_1DOF = 0.500021713558733  # 0.5 * scipy.stats.chi2.ppf(0.6827, 1)   (measureToAs.py:324)
TWO_PI = 2.0 * math.pi
MODEL_STEP = 1e-6  # ascent: final plain Newton step below this (rad; relative in the norm) taken by the quadratic model


def scan_capped(sigma, ph_shift_res):
    """True where a 1-sigma bound came from the phShiftRes/2 cap rather than the chi2 crossing: the reference loop
    stops once its counter kk exceeds phShiftRes/2 and logs 'Could not estimate lower/upper-bound uncertainty'
    (measureToAs.py:348-350, :373-375); the bound is kk*step + step/2, so kk is read back from it."""
    step = TWO_PI / int(ph_shift_res)
    kk = np.rint((np.asarray(sigma, dtype=np.float64) - step / 2) / step)
    return kk > int(ph_shift_res) / 2


def warn_capped(res, ph_shift_res, names, log):
    """The reference's warnings for every interval whose scan hit the cap (one call per fit batch)."""
    for side, key in (("lower", "phShi_LL"), ("upper", "phShi_UL")):
        for i in np.nonzero(scan_capped(res[key], ph_shift_res))[0]:
            log.warning('Could not estimate {}-bound uncertainty on {}'.format(side, names[i]))


def _vals(tmpl, prefix, K):
    out = []
    for j in range(1, K + 1):
        v = tmpl["%s_%d" % (prefix, j)]
        out.append(float(v["value"] if isinstance(v, dict) else v))
    return out


class ToAFitter:
    """Fits all intervals of one concatenated folded-phase array together."""

    def __init__(self, x, offsets, exposure, tmpl, ph_shift_res=1000, nbr_bins=15, device=None):
        self.model = str(tmpl["model"]).lower()
        if self.model not in ("fourier", "cauchy", "vonmises"):
            raise ValueError("Unknown template model. Only fourier, cauchy, or vonmises are supported")
        K = len([k for k in tmpl if k.startswith("amp_")])
        self.K = K
        amps = _vals(tmpl, "amp", K)
        if self.model == "fourier":
            locs, wids = _vals(tmpl, "ph", K), None
        else:
            locs, wids = _vals(tmpl, "cen", K), _vals(tmpl, "wid", K)
        self.amps = np.array(amps)
        self.tpl = ops.make_template(self.model, amps, locs, wids, 1.0)
        self.tmpl = tmpl
        nv = tmpl["norm"]
        self.norm0 = float(nv["value"] if isinstance(nv, dict) else nv)
        self.lo, self.hi = self.norm0 / 100.0, 500.0                          # measureToAs.py:715-716, :757-758
        self.pb = math.pi if self.model == "fourier" else 1.5 * math.pi       # :722, :767
        self.res = int(ph_shift_res)
        self.nbins = int(nbr_bins)
        self.E = np.asarray(exposure, dtype=np.float64).reshape(-1)
        off = np.asarray(offsets.cpu().numpy() if _is_torch(offsets) else offsets, dtype=np.int64)
        self.offsets_h = off
        self.nint = off.size - 1
        if self.E.size != self.nint:
            raise ValueError("one exposure per interval required")
        self.N = np.diff(off).astype(np.float64)
        if np.any(self.N <= 0):
            raise IndexError("a ToA interval holds no photons (measureToAs.py:182 would fail on TIME_toa[-1])")
        self.x_h = None if _is_torch(x) else np.ascontiguousarray(x, dtype=np.float64)
        self.x, self.offsets = self._to_device(x, off, device)

    # ------------------------------------------------------------------ device plumbing
    def _to_device(self, x, off, device):
        if _is_torch(x):
            import torch
            return x.reshape(-1).to(torch.float64).contiguous(), torch.as_tensor(off, device=x.device)
        try:
            import torch
            if torch.cuda.is_available():
                dev = torch.device(device if device is not None else "cuda")
                return (torch.as_tensor(np.ascontiguousarray(x, dtype=np.float64), device=dev),
                        torch.as_tensor(off, device=dev))
        except ImportError:  # pragma: no cover
            pass
        return np.ascontiguousarray(x, dtype=np.float64), off

    def _arr(self, a, dtype):
        if _is_torch(self.x):
            import torch
            return torch.as_tensor(np.ascontiguousarray(a, dtype=dtype), device=self.x.device)
        return np.ascontiguousarray(a, dtype=dtype)

    # ------------------------------------------------------------------ evaluations
    def _F(self, n):
        return n if self.model == "fourier" else TWO_PI * n + self.amps.sum()

    def evaluate(self, iv, n, phi):
        """LL, gradient (2) and Hessian (3) of the reference extended LL at points."""
        iv = np.asarray(iv, dtype=np.int64)
        n = np.asarray(n, dtype=np.float64)
        phi = np.asarray(phi, dtype=np.float64)
        s = ops.toa_points(self.x, self.offsets, self.tpl, self._arr(iv, np.int64), self._arr(n, np.float64),
                           self._arr(phi, np.float64))
        if _is_torch(s):
            s = s.cpu().numpy()
        s = np.asarray(s)
        N, E = s[:, 7], self.E[iv]
        F = self._F(n)
        with np.errstate(divide="ignore", invalid="ignore"):
            if self.model == "fourier":
                ll = -n * E + N * np.log(n * E) + (s[:, 0] - N * np.log(n))
            else:
                ll = -F * E / TWO_PI + N * np.log(F * E / TWO_PI) + (s[:, 0] - N * np.log(F))
        ll = np.where(s[:, 6] / F > 0, ll, -np.inf)
        g = np.stack([-E + s[:, 1], s[:, 2]], axis=1)
        H = np.stack([s[:, 3], s[:, 4], s[:, 5]], axis=1)
        return ll, g, H

    # ------------------------------------------------------------------ step 1: brute grid
    def brute(self, with_hmin=False):
        nphi = int(math.ceil((2 * self.pb) / (0.05 * 1.0)))
        phis = np.arange(nphi) * 0.05 + (-self.pb)                            # numpy mgrid lattice
        norms = np.arange(20) * ((self.hi - self.lo) / float(20 - 1)) + self.lo
        ln, hmin = ops.toa_grid(self.x, self.offsets, self.tpl, self._arr(np.tile(norms, (self.nint, 1)), np.float64),
                                self._arr(phis, np.float64))
        if _is_torch(ln):
            ln, hmin = ln.cpu().numpy(), hmin.cpu().numpy()
        N = self.N[:, None, None]
        E = self.E[:, None, None]
        nn = norms[None, :, None]
        F = self._F(nn)
        with np.errstate(divide="ignore", invalid="ignore"):
            if self.model == "fourier":
                ll = -nn * E + N * np.log(nn * E) + (ln - N * np.log(nn))
            else:
                ll = -F * E / TWO_PI + N * np.log(F * E / TWO_PI) + (ln - N * np.log(F))
        valid = (hmin[:, None, :] + nn) > 0
        ll = np.where(valid & np.isfinite(ll), ll, -np.inf)
        ll = ll.reshape(self.nint, 20, nphi)
        flat = ll.reshape(self.nint, -1)
        idx = np.argmax(flat, axis=1)                                          # first maximum, norm-outer
        a, b = np.unravel_index(idx, (20, nphi))
        if with_hmin:
            return norms[a], phis[b], hmin[np.arange(self.nint), b], ll, a, b
        return norms[a], phis[b]

    # ------------------------------------------------------------------ step 2: 2-D ascent
    def maximise(self, n0, phi0, max_iter=60):
        n = np.array(n0, dtype=np.float64)
        phi = np.array(phi0, dtype=np.float64)
        iv_all = np.arange(self.nint)
        ll, g, H = self.evaluate(iv_all, n, phi)
        active = np.ones(self.nint, dtype=bool)
        for _ in range(max_iter):
            act = np.nonzero(active)[0]
            if act.size == 0:
                break
            dn, dp, pure = self._newton_step(n[act], g[act], H[act], with_pure=True, phi=phi[act])
            # converged: even the full step moves less than the stopping tolerance (no confirming pass)
            fn = np.clip(n[act] + dn, self.lo, self.hi)
            fp = np.clip(phi[act] + dp, -self.pb, self.pb)
            pre = np.isfinite(ll[act]) & (np.abs(fp - phi[act]) < 1e-12) & (
                np.abs(fn - n[act]) < 1e-12 * np.maximum(1.0, np.abs(fn)))
            # final step by the local quadratic model (k_toa_fit's kFitModelStep): the plain Newton step of a
            # negative definite Hessian below MODEL_STEP, inside the bounds, is taken without a likelihood pass
            ia = act
            mod = ~pre & pure & np.isfinite(ll[ia]) & (fn == n[ia] + dn) & (fp == phi[ia] + dp) & (
                np.abs(dp) < MODEL_STEP) & (np.abs(dn) < MODEL_STEP * np.maximum(1.0, np.abs(n[ia])))
            if mod.any():
                im = ia[mod]
                Hm, gm, dnm, dpm = H[im], g[im], dn[mod], dp[mod]
                q = Hm[:, 0] * dnm * dnm + 2.0 * Hm[:, 1] * dnm * dpm + Hm[:, 2] * dpm * dpm
                ll[im] = ll[im] + (gm[:, 0] * dnm + gm[:, 1] * dpm + 0.5 * q)
                n[im], phi[im] = fn[mod], fp[mod]
            pre |= mod
            if pre.any():
                active[act[pre]] = False
                keep = ~pre
                act, dn, dp = act[keep], dn[keep], dp[keep]
                if act.size == 0:
                    break
            t = np.ones(act.size)
            pending = np.ones(act.size, dtype=bool)
            new_n, new_p = n[act].copy(), phi[act].copy()
            new_ll, new_g, new_H = ll[act].copy(), g[act].copy(), H[act].copy()
            for _ls in range(40):
                idx = np.nonzero(pending)[0]
                if idx.size == 0:
                    break
                tn = np.clip(n[act][idx] + t[idx] * dn[idx], self.lo, self.hi)
                tp = np.clip(phi[act][idx] + t[idx] * dp[idx], -self.pb, self.pb)
                l2, g2, H2 = self.evaluate(act[idx], tn, tp)
                ok = np.isfinite(l2) & (l2 >= ll[act][idx] - 1e-12 * np.abs(ll[act][idx]))
                acc = idx[ok]
                new_n[acc], new_p[acc] = tn[ok], tp[ok]
                new_ll[acc], new_g[acc], new_H[acc] = l2[ok], g2[ok], H2[ok]
                pending[acc] = False
                t[idx[~ok]] *= 0.5
            moved_n = np.abs(new_n - n[act])
            moved_p = np.abs(new_p - phi[act])
            n[act], phi[act] = new_n, new_p
            ll[act], g[act], H[act] = new_ll, new_g, new_H
            done = (moved_p < 1e-12) & (moved_n < 1e-12 * np.maximum(1.0, np.abs(new_n)))
            done |= pending  # line search exhausted: at the (numerical) optimum
            active[act[done]] = False
        return n, phi, ll

    def _newton_step(self, n, g, H, with_pure=False, phi=None):
        """Levenberg-shifted Newton step with a trust region; projected (k_toa_fit's fit_newton_dir): a coordinate on
        its bound whose gradient points out is held and the other takes its own 1-D Newton step."""
        hnn, hnp, hpp = H[:, 0], H[:, 1], H[:, 2]
        if phi is not None:
            pfix = ((phi <= -self.pb) & (g[:, 1] < 0)) | ((phi >= self.pb) & (g[:, 1] > 0))
            nfix = ((n <= self.lo) & (g[:, 0] < 0)) | ((n >= self.hi) & (g[:, 0] > 0))
            proj = pfix | nfix
        else:
            proj = np.zeros(n.size, dtype=bool)
        # shift the Hessian to be negative definite (Levenberg damping), then solve
        tr = hnn + hpp
        det = hnn * hpp - hnp * hnp
        lam_max = 0.5 * tr + np.sqrt(np.maximum(0.25 * tr * tr - det, 0.0))   # largest eigenvalue
        shift = np.where(lam_max < 0, 0.0, lam_max * 1.5 + 1e-6 * (np.abs(hnn) + np.abs(hpp)) + 1e-12)
        a, c = hnn - shift, hpp - shift
        det2 = a * c - hnp * hnp
        dn = -(c * g[:, 0] - hnp * g[:, 1]) / det2
        dp = -(a * g[:, 1] - hnp * g[:, 0]) / det2
        # trust region: at most 0.05 rad in phShift and half the norm per step
        pure = shift == 0.0
        if proj.any():
            with np.errstate(divide="ignore", invalid="ignore"):
                dn1 = np.where(hnn < 0, -g[:, 0] / np.where(hnn < 0, hnn, -1.0), np.where(g[:, 0] > 0, 0.1, -0.1) * np.abs(n))
                dp1 = np.where(hpp < 0, -g[:, 1] / np.where(hpp < 0, hpp, -1.0), np.where(g[:, 1] > 0, 0.05, -0.05))
            dn = np.where(proj, np.where(nfix, 0.0, dn1), dn)
            dp = np.where(proj, np.where(pfix, 0.0, dp1), dp)
            pure = np.where(proj, (nfix | (hnn < 0)) & (pfix | (hpp < 0)), pure)
        sc = np.minimum(1.0, 0.05 / np.maximum(np.abs(dp), 1e-300))
        sc = np.minimum(sc, 0.5 * np.abs(n) / np.maximum(np.abs(dn), 1e-300))
        if with_pure:
            return dn * sc, dp * sc, pure & (sc == 1.0)
        return dn * sc, dp * sc

    def profile_norm(self, iv, phi, n_start, max_iter=30):
        """max over norm in [lo, hi] of LL(norm, phi) at fixed phi (1-D Newton, concave)."""
        iv = np.asarray(iv)
        n = np.clip(np.array(n_start, dtype=np.float64), self.lo, self.hi)
        ll, g, H = self.evaluate(iv, n, phi)
        converged = np.zeros(n.size, dtype=bool)
        for _ in range(max_iter):
            bad = ~np.isfinite(ll)
            step = np.where(H[:, 0] < 0, -g[:, 0] / np.where(H[:, 0] < 0, H[:, 0], -1.0), 0.1 * n)
            step = np.clip(step, -0.5 * n, 0.5 * n)
            step = np.where(bad, 0.5 * n, step)  # infeasible: model <= 0 somewhere, raise the norm
            nn = np.clip(n + step, self.lo, self.hi)
            # converged: the next pass would move the norm by <= 1e-13 of it (no confirming pass)
            done = np.isfinite(ll) & (np.abs(nn - n) <= 1e-13 * np.maximum(1.0, n)) | converged
            converged = done
            if np.all(done):
                break
            w = np.nonzero(~done)[0]
            l2, g2, H2 = self.evaluate(iv[w], nn[w], phi[w])
            worse = np.isfinite(ll[w]) & (~np.isfinite(l2) | (l2 < ll[w] - 1e-12 * np.abs(ll[w])))
            if np.any(worse):  # damp the few overshoots
                ww = w[worse]
                nn[ww] = np.clip(n[ww] + 0.25 * step[ww], self.lo, self.hi)
                l3, g3, H3 = self.evaluate(iv[ww], nn[ww], phi[ww])
                l2[worse], g2[worse], H2[worse] = l3, g3, H3
            conv = np.abs(nn[w] - n[w]) <= 1e-13 * np.maximum(1.0, n[w])
            n[w], ll[w], g[w], H[w] = nn[w], l2, g2, H2
            converged[w[conv]] = True
            if np.all(converged):
                break
        return n, ll

    # ------------------------------------------------------------------ step 3: error scan
    def _scan_phases(self, phi_hat, side, ks, passed=None):
        """phShift values the lmfit loop evaluates at steps ks (clip-to-bound semantics); ``passed`` marks
        intervals whose scan already crossed the bound in an earlier batch of steps."""
        step = TWO_PI / self.res
        target = phi_hat[:, None] + side * ks[None, :] * step
        if self.model == "fourier":
            # the first step past +-pi is clipped to the bound; later steps move the bound (:332-334, :357-359)
            past = (target <= -math.pi) if side < 0 else (target >= math.pi)
            first = np.where(past.any(axis=1), past.argmax(axis=1), -1)
            if passed is not None:
                first = np.where(passed, -1, first)
            cur = target.copy()
            rows = np.nonzero(first >= 0)[0]
            cur[rows, first[rows]] = -math.pi if side < 0 else math.pi
            return cur
        return np.clip(target, -self.pb, self.pb)

    def error_scan(self, phi_hat, n_hat, ll_max):
        step = TWO_PI / self.res
        kcap = self.res / 2.0
        out = {}
        for side in (-1, 1):
            kk_final = np.full(self.nint, -1, dtype=np.int64)
            passed = np.zeros(self.nint, dtype=bool)
            k0 = 1
            batch = 12
            while True:
                todo = np.nonzero(kk_final < 0)[0]
                if todo.size == 0:
                    break
                ks = np.arange(k0, k0 + batch)
                phis = self._scan_phases(phi_hat[todo], side, ks, passed[todo])
                tg = phi_hat[todo][:, None] + side * ks[None, :] * step
                passed[todo] |= ((tg <= -math.pi) if side < 0 else (tg >= math.pi)).any(axis=1)
                iv = np.repeat(todo, ks.size)
                nprof, llk = self.profile_norm(iv, phis.reshape(-1), np.repeat(n_hat[todo], ks.size))
                diff = (ll_max[todo][:, None] - llk.reshape(todo.size, ks.size))
                cross = diff > CHI2_1SIG_1DOF
                # the loop stops at the first crossing, or once kk (= k+1) exceeds phShiftRes/2
                stop = cross | ((ks[None, :] + 1) > kcap)
                hit = stop.any(axis=1)
                first = stop.argmax(axis=1)
                kk_final[todo[hit]] = ks[first[hit]] + 1
                k0 += batch
                batch = min(batch * 2, 256)
            out[side] = kk_final * step + step / 2
        return out[-1], out[1]

    # ------------------------------------------------------------------ step 4: redChi2
    def _bins(self):
        """numpy.linspace edges and the bin centres of binphases (binphases.py:9-39, measureToAs.py:385-387)."""
        upper = 1.0 if self.model == "fourier" else TWO_PI
        edges = np.linspace(0, upper, self.nbins + 1, endpoint=True)
        pp = np.linspace(0, upper, self.nbins, endpoint=False) + (upper / self.nbins) / 2
        return edges, pp

    def reduced_chi2(self, n_hat, phi_hat, nfree=2, amp_shift=None, records=None):
        """redChi2 per interval (measureToAs.py:385-393) on the device (crimp_toa_redchi2: the binned profile against
        the best-fit curve). ``records``: crimp_toa_fit's [nint, 8] records where they are at hand (device-resident,
        no host round trip); else built from the arguments."""
        edges, pp = self._bins()
        if records is None:
            rec = np.zeros((self.nint, 8))
            rec[:, 0], rec[:, 1] = n_hat, phi_hat
            rec[:, 6] = 1.0 if amp_shift is None else np.asarray(amp_shift, dtype=np.float64)
            records = self._arr(rec, np.float64)
        rc = ops.toa_redchi2(self.x, self.offsets, self.tpl, self._arr(self.E, np.float64), records,
                             self._arr(edges, np.float64), self._arr(pp, np.float64), nfree)
        return rc.cpu().numpy() if _is_torch(rc) else np.asarray(rc)

    def curve(self, n, phi, xx, amp_shift=1.0):
        """fourseries / wrapcauchy / vonmises at xx (templatemodels.py:64-82, :166-185, :271-290)."""
        y = np.zeros(np.broadcast(n, xx).shape) + n
        t = self.tpl
        a = amp_shift
        for j in range(self.K):
            if self.model == "fourier":
                # cos(A - B) with A = (j+1) 2 pi xx + loc_j, B = (j+1) phi by angle subtraction: the cos/sin run on
                # the bin centres and on the intervals' phShifts (no (intervals x bins) cos), the terms differ from
                # np.cos(A - B) by ~1e-16
                ang = (j + 1) * 2 * np.pi * xx + t.loc[j]
                bph = (j + 1) * phi
                y = y + t.amp[j] * a * (np.cos(ang) * np.cos(bph) + np.sin(ang) * np.sin(bph))
            elif self.model == "cauchy":
                y = y + ((t.amp[j] * a) / (2 * np.pi)) * (np.sinh(t.wid[j]) / (np.cosh(t.wid[j]) - np.cos(xx - t.loc[j] - phi)))
            else:
                y = y + ((t.amp[j] * a) / (2 * np.pi * t.i0[j])) * np.exp((1 / t.wid[j] ** 2) * np.cos(xx - t.loc[j] - phi))
        return y

    # ------------------------------------------------------------------ drivers
    def fit(self, brutemin=False, vary_amps=False):
        """Every interval's fit and redChi2 in one device call (crimp_toa_fit_redchi2: one workgroup per interval runs
        steps 1-3, the histogram of step 4 beside them). ``vary_amps``: ampShift free (Fourier [0.01, 100], Cauchy [0, inf), von Mises [0, 500]) after the (norm, phShift) fit,
        re-profiled with the norm in the 1-sigma scan, one more free parameter in redChi2 (:305-312)."""
        edges, pp = self._bins()
        n = self.nint
        small = self._arr(np.concatenate([self.E, edges, pp]), np.float64)  # one upload
        buf = ops.toa_fit_redchi2(self.x, self.offsets, self.tpl, small[:n], self.norm0, self.res, brutemin, vary_amps,
                                  small[n:n + edges.size], small[n + edges.size:], 3 if vary_amps else 2, packed=True)
        buf = np.asarray(buf.cpu().numpy() if _is_torch(buf) else buf)           # one readback
        r, rchi2 = buf[:8 * n].reshape(n, 8), buf[8 * n:].copy()
        n_hat, phi_hat, amp = r[:, 0].copy(), r[:, 1].copy(), r[:, 6].copy()
        return {"phShi": phi_hat, "phShi_LL": r[:, 3].copy(), "phShi_UL": r[:, 4].copy(), "reducedChi2": rchi2,
                "norm": n_hat, "LLmax": r[:, 2].copy(), "evaluations": r[:, 5].copy(), "ampShift": amp,
                "cached_evaluations": r[:, 7].copy()}

    def fit_host(self, brutemin=False):
        """The same fit driven from the host, one batched likelihood launch per iteration (cross-check of fit)."""
        if brutemin:
            n0, p0, hm, ll, a, b = self.brute(with_hmin=True)
            # the ascent's start (k_toa_grid_best does the same): the norm at the photon rate N/E where it is inside
            # the bounds and keeps the model positive at the lattice phShift; there, if the model stays well positive,
            # the phShift at the vertex of the parabola through the maximum and its lattice neighbours
            rate = self.N / self.E
            use = (rate >= self.lo) & (rate <= self.hi) & (hm + rate > 0)
            n0 = np.where(use, rate, n0)
            nphi = ll.shape[2]
            phis = np.arange(nphi) * 0.05 + (-self.pb)
            iv = np.arange(self.nint)
            inner = use & (hm + rate > 0.5 * rate) & (b >= 1) & (b + 1 < nphi)
            bm, bp = np.clip(b - 1, 0, nphi - 1), np.clip(b + 1, 0, nphi - 1)
            lm, l0, lp = ll[iv, a, bm], ll[iv, a, b], ll[iv, a, bp]
            den = lm - 2.0 * l0 + lp
            with np.errstate(invalid="ignore", divide="ignore"):
                d = np.clip(0.5 * (lm - lp) / den, -0.5, 0.5)
            ok = inner & np.isfinite(lm) & np.isfinite(lp) & (den < 0)
            p0 = np.where(ok, phis[b] + d * (phis[bp] - phis[b]), p0)
        else:
            n0, p0 = np.full(self.nint, self.norm0), np.zeros(self.nint)
        n_hat, phi_hat, ll_max = self.maximise(n0, p0)
        lo_err, up_err = self.error_scan(phi_hat, n_hat, ll_max)
        rchi2 = self.reduced_chi2(n_hat, phi_hat)
        return {"phShi": phi_hat, "phShi_LL": lo_err, "phShi_UL": up_err, "reducedChi2": rchi2, "norm": n_hat,
                "LLmax": ll_max}

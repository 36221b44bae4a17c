"""Template building: a high-S/N pulse profile and its best-fit template model.

Drop-in for CRIMP v2.3.0 ``pulseprofile.py`` (:57-800): ``PulseProfileFromEventFile``
(``createpulseprofile`` :109-139, ``fitpulseprofile`` :142-260), ``ModelPulseProfile`` (Fourier
:294-383, wrapped Cauchy :385-475, von Mises :477-563), ``measurechi2`` (:568-591),
``calcpulseproperties`` (:596-630), ``calcuncertaintypulseproperties`` (:633-668),
``plotpulseprofile`` (:671-720), ``writetemplatefile`` (:723-752) and the
``templatepulseprofile`` CLI (:755-796).

The photon-scale part -- phases of every event (``crimp_calcphase``) and their histogram
(``crimp_binphases``, numpy.histogram edge semantics) -- runs on the MI355X; the fit of the binned
profile (10^1-10^2 bins) is host work. The reference fits with lmfit's ``minimize(method='BFGS')``;
lmfit is not importable here, so ``_bfgs`` restates what that call does: lmfit's bounded-parameter
transforms (MINUIT style, ``lmfit/parameter.py`` ``setup_bounds``/``from_internal``) and
``scipy.optimize.minimize(penalty, x_internal, method='BFGS', options={'maxiter': 2*max_nfev})`` on
the negative binned Gaussian log likelihood.
"""
import argparse
import copy
import logging
import math

import numpy as np

from .binphases import binphases as _binphases_host  # noqa: F401  (reference-compatible helper)
from .calcphase import calcphase
from .eventfile import EvtFileOps
from .logging_utils import configure_logging, get_logger
from .readPPtemplate import readPPtemplate
from .templatemodels import Fourier, VonMises, WrappedCauchy

logger = get_logger(__name__)

_TINY = 1.0e-15  # lmfit parameter.py: internal values below this are set to 0


class _Par:
    """One lmfit Parameter as the BFGS call sees it (value clipped into [min, max])."""

    def __init__(self, name, value, vary=True, min=-np.inf, max=np.inf):  # noqa: A002
        self.name, self.vary, self.min, self.max = name, bool(vary), float(min), float(max)
        self.value = float(np.clip(float(value), self.min, self.max))

    def to_internal(self):
        lo, hi, v = self.min, self.max, self.value
        if lo == -np.inf and hi == np.inf:
            x = v
        elif hi == np.inf:
            x = math.sqrt((v - lo + 1.0) ** 2 - 1)
        elif lo == -np.inf:
            x = math.sqrt((hi - v + 1.0) ** 2 - 1)
        else:
            x = math.asin(2 * (v - lo) / (hi - lo) - 1)
        return 0.0 if abs(x) < _TINY else x

    def from_internal(self, x):
        lo, hi = self.min, self.max
        if lo == -np.inf and hi == np.inf:
            return x
        if hi == np.inf:
            return lo - 1.0 + math.sqrt(x * x + 1)
        if lo == -np.inf:
            return hi + 1 - math.sqrt(x * x + 1)
        return lo + (math.sin(x) + 1) * (hi - lo) / 2.0


class _Params(dict):
    def add(self, name, value, vary=True, min=-np.inf, max=np.inf):  # noqa: A002
        self[name] = _Par(name, value, vary, min, max)


def _bfgs(nll, params, args, nan_policy="raise", max_nfev=1.0e6):
    """lmfit ``minimize(nll, params, args, method='BFGS', max_nfev, nan_policy)``: returns the
    ``valuesdict()`` of the result (insertion order) and scipy's OptimizeResult."""
    from scipy.optimize import minimize

    free = [p for p in params.values() if p.vary]
    vals = {k: p.value for k, p in params.items()}
    nfev = [0]

    def penalty(x):
        nfev[0] += 1
        if nfev[0] > max_nfev:
            raise RuntimeError("fit aborted: number of function evaluations > %d" % max_nfev)
        for p, xi in zip(free, x):
            vals[p.name] = p.from_internal(float(xi))
        r = nll(vals, *args)
        if nan_policy == "raise" and np.isnan(r):
            raise ValueError("The model function generated NaN values and the fit aborted! Please check your "
                             "model function and/or set boundaries on parameters where applicable.")
        return r

    x0 = np.array([p.to_internal() for p in free], dtype=np.float64)
    res = minimize(penalty, x0, method="BFGS", options={"maxiter": 2 * max_nfev})
    for p, xi in zip(free, res.x):
        vals[p.name] = p.from_internal(float(xi))
    return dict(vals), res


class PulseProfileFromEventFile:
    """Build and model a pulse profile from an event file (pulseprofile.py:57-260)."""

    def __init__(self, evtFile: str, timMod: str, eneLow: float = 0.5, eneHigh: float = 10., nbrBins: int = 30):
        self.evtFile = evtFile
        self.timMod = timMod
        self.eneLow = eneLow
        self.eneHigh = eneHigh
        self.nbrBins = nbrBins

    def createpulseprofile(self):
        """pulseprofile.py:109-139: LIVETIME from the GTIs, energy-filtered photon phases on the device,
        their histogram on the device; count rates per bin."""
        from . import ops

        EF = EvtFileOps(self.evtFile)
        _, gtiList = EF.readGTI()
        LIVETIME = np.sum(gtiList[:, 1] - gtiList[:, 0]) * 86400
        ef = EF.build_time_energy_df().filtenergy(eneLow=self.eneLow, eneHigh=self.eneHigh)
        timeMJD = ef.time_energy_df["TIME"].to_numpy()
        _, folded = calcphase(timeMJD, self.timMod)
        folded = np.asarray(folded, dtype=np.float64)
        if not (((folded >= 0) & (folded <= 1)).all()):
            raise Exception('Array in not cycle folded between [0,1) or [0, 2*pi)')
        nb = int(self.nbrBins)
        edges = np.linspace(0, 1, nb + 1, endpoint=True)
        cts = np.asarray(ops.binphases_counts(folded, np.array([0, folded.size], np.int64), edges)).reshape(-1)
        ppBins = np.linspace(0, 1, nb, endpoint=False) + (1 / nb) / 2
        ctRate = cts / (LIVETIME / nb)
        ctRateErr = np.sqrt(cts) / (LIVETIME / nb)
        return {'ppBins': ppBins, 'ppBinsRange': (1 / nb) / 2, 'countRate': ctRate, 'countRateErr': ctRateErr}

    def fitpulseprofile(self, ppmodel: str = 'fourier', nbrComp: int = 2, initTemplateMod: str = None,
                        fixPhases: bool = False, figure: str = None, templateFile: str = None,
                        calcPulsedFraction: bool = False):
        """pulseprofile.py:142-260. Returns (fitResultsDict, bestFitModel, pulsedProperties)."""
        logger.info('\n Running method fitpulseprofile with input parameters: \n evtFile: %s\n Timing model: %s'
                    '\n eneLow: %s\n eneHigh: %s\n nbrBins: %s\n ppmodel: %s\n nbrComp: %s\n initTemplateMod: %s'
                    '\n fixPhases: %s\n figure: %s(.pdf)\n templateFile: %s(.txt)\n calcPulsedFraction: %s\n',
                    self.evtFile, self.timMod, self.eneLow, self.eneHigh, self.nbrBins, ppmodel, nbrComp,
                    initTemplateMod, fixPhases, figure, templateFile, calcPulsedFraction)
        pulseProfile = self.createpulseprofile()
        if initTemplateMod is not None:
            logger.info('\n Initial template file provided : %s\n Using these model parameters as starting point.'
                        ' \n Ignoring input keywords ppmodel = %s and nbrComp = %s', initTemplateMod, ppmodel,
                        nbrComp)
            tmpl = readPPtemplate(initTemplateMod)
            ppmodel, nbrComp = tmpl["model"], tmpl["nbrComp"]
        else:
            logger.info('\n No initial template file provided\n Fitting to user chosen model : %s'
                        '\n using number of components : %s', ppmodel, nbrComp)
        kind = ppmodel.casefold()
        mp = ModelPulseProfile(pulseProfile, nbrComp, initTemplateMod, fixPhases)
        if kind == 'fourier':
            fitResultsDict, bestFitModel = mp.fouriermodel()
        elif kind in ('cauchy', 'vonmises'):
            pulseProfile["ppBins"] *= 2 * np.pi  # radians for the peaked models (:183-188)
            fitResultsDict, bestFitModel = mp.cauchymodel() if kind == 'cauchy' else mp.vonmisesmodel()
        else:
            logger.error('Model {} is not supported yet; fourier, vonmises, cauchy are supported'.format(ppmodel))
            raise ValueError('Model {} is not supported yet; fourier, vonmises, cauchy are supported'.format(ppmodel))

        if templateFile is not None:
            writetemplatefile(templateFile, fitResultsDict)
            logger.info('\n chi2 = %s\n dof = %s\n redchi2 = %s\n', fitResultsDict["chi2"], fitResultsDict["dof"],
                        fitResultsDict["redchi2"])
            logger.info('\n Created best fit template file : %s.txt \n', templateFile)
        else:
            logger.info('\n No template file created: templateFile is None\n')

        pulsedProperties = None
        if calcPulsedFraction and kind == 'fourier':
            pulsedProperties = calcpulseproperties(pulseProfile, nbrComp)
            pulsedProperties.update(calcuncertaintypulseproperties(pulseProfile, nbrComp))
        elif calcPulsedFraction:
            logger.warning('Cannot calculate rms pulsed fraction for ' + kind + '\n Setting pulsedProperties to None')

        if figure is not None:
            plotpulseprofile(pulseProfile, outFile=figure, fittedModel=bestFitModel)
            logger.info('\n Created figure of pulse profile and best-fit template : %s.pdf \n', figure)
        else:
            logger.info('\n No figure file provided/created\n')
        return fitResultsDict, bestFitModel, pulsedProperties


def _nll_fourier(theta, xx, yy, yyErr):
    return -Fourier(theta, xx).loglikelihoodFS(yy, yyErr)


def _nll_cauchy(theta, xx, yy, yyErr):
    return -WrappedCauchy(theta, xx).loglikelihoodCA(yy, yyErr)


def _nll_vonmises(theta, xx, yy, yyErr):
    return -VonMises(theta, xx).loglikelihoodVM(yy, yyErr)


class ModelPulseProfile:
    """Fit a binned pulse profile {ppBins, countRate, countRateErr} (pulseprofile.py:263-563)."""

    def __init__(self, pulseProfile: dict, nbrComp: int = 2, initTemplateMod: str = None, fixPhases: bool = False):
        self.pulseProfile = pulseProfile
        self.nbrComp = nbrComp
        self.initTemplateMod = initTemplateMod
        self.fixPhases = fixPhases

    def _run(self, template, params, nbrFreeParams, nll, curve, nan_policy):
        pp = self.pulseProfile
        vals, _ = _bfgs(nll, params, (pp["ppBins"], pp["countRate"], pp["countRateErr"]), nan_policy=nan_policy)
        bfModel = curve(vals, pp["ppBins"])
        chi2Results = measurechi2(pp, bfModel, nbrFreeParams)
        print('Template {} best fit statistics\n chi2 = {} for dof = {}\n Reduced chi2 = {}'.format(
            template, chi2Results["chi2"], chi2Results["dof"], chi2Results["redchi2"]))
        fitResultsDict = dict(vals)
        fitResultsDict.update(chi2Results)
        fitResultsDict.update({'model': template})
        return fitResultsDict, bfModel

    def fouriermodel(self):
        """pulseprofile.py:294-383."""
        ctRate = self.pulseProfile["countRate"]
        P = _Params()
        if self.initTemplateMod is None:
            P.add('norm', np.mean(ctRate), min=0.0, max=1.0e6)
            for kk in range(1, self.nbrComp + 1):
                P.add('amp_%d' % kk, 0.1 * np.mean(ctRate))
                P.add('ph_%d' % kk, 0)
            nbrFreeParams = 2 * self.nbrComp + 1
        else:
            t = readPPtemplate(self.initTemplateMod)
            self.nbrComp = t["nbrComp"]
            P.add('norm', t['norm']['value'], min=0.0, max=1.0e6, vary=t['norm']['vary'])
            nbrFreeParams = 1 if t['norm']['vary'] else 0
            for kk in range(1, self.nbrComp + 1):
                P.add('amp_%d' % kk, t['amp_%d' % kk]['value'], vary=t['amp_%d' % kk]['vary'])
                P.add('ph_%d' % kk, t['ph_%d' % kk]['value'], vary=t['ph_%d' % kk]['vary'])
                if self.fixPhases:
                    P['ph_%d' % kk].vary = False
                nbrFreeParams += sum(1 for key in ('amp_%d' % kk, 'ph_%d' % kk) if t[key]['vary'])
        P.add('phShift', 0, vary=False)
        P.add('ampShift', 1, vary=False)
        return self._run('fourier', P, nbrFreeParams, _nll_fourier,
                         lambda v, x: Fourier(v, x).fourseries(), "raise")

    def _peaked_params(self):
        """Parameters of the Cauchy / von Mises fits (:401-451, :493-538)."""
        ctRate = self.pulseProfile["countRate"]
        P = _Params()
        if self.initTemplateMod is None:
            P.add('norm', np.min(ctRate), min=0.0, max=np.max(ctRate))
            for kk in range(1, self.nbrComp + 1):
                P.add('amp_%d' % kk, 1.3 * np.min(ctRate), min=0.0, max=np.inf)
                P.add('cen_%d' % kk, np.pi, min=0.0, max=2 * np.pi)
                P.add('wid_%d' % kk, 1, min=0.0, max=np.inf)
            nbrFreeParams = 2 * self.nbrComp + 1  # as the reference counts it (:413, :505)
        else:
            t = readPPtemplate(self.initTemplateMod)
            self.nbrComp = t["nbrComp"]
            P.add('norm', t['norm']['value'], min=0.0, max=np.max(ctRate), vary=t['norm']['vary'])
            nbrFreeParams = 1 if t['norm']['vary'] else 0
            for kk in range(1, self.nbrComp + 1):
                P.add('amp_%d' % kk, t['amp_%d' % kk]['value'], min=0.0, max=np.inf, vary=t['amp_%d' % kk]['vary'])
                P.add('cen_%d' % kk, t['cen_%d' % kk]['value'], min=0.0, max=2 * np.pi,
                      vary=t['cen_%d' % kk]['vary'])
                P.add('wid_%d' % kk, t['wid_%d' % kk]['value'], min=0.0, max=np.inf, vary=t['wid_%d' % kk]['vary'])
                if self.fixPhases:
                    P['cen_%d' % kk].vary = False
                nbrFreeParams += sum(1 for key in ('amp_%d' % kk, 'cen_%d' % kk, 'wid_%d' % kk) if t[key]['vary'])
        P.add('phShift', 0, vary=False)
        P.add('ampShift', 1, vary=False)
        return P, nbrFreeParams

    def cauchymodel(self):
        """pulseprofile.py:385-475."""
        P, nfree = self._peaked_params()
        return self._run('cauchy', P, nfree, _nll_cauchy, lambda v, x: WrappedCauchy(v, x).wrapcauchy(),
                         "propagate")

    def vonmisesmodel(self):
        """pulseprofile.py:477-563."""
        P, nfree = self._peaked_params()
        return self._run('vonmises', P, nfree, _nll_vonmises, lambda v, x: VonMises(v, x).vonmises(), "propagate")


def measurechi2(pulseProfile, model, nbrFreeParam):
    """pulseprofile.py:568-591."""
    ctRate = pulseProfile["countRate"]
    ctRateErr = pulseProfile["countRateErr"]
    chi2 = np.sum(((ctRate - model) ** 2) / (ctRateErr ** 2))
    dof = len(ctRate) - nbrFreeParam
    return {'chi2': chi2, 'dof': dof, 'redchi2': chi2 / dof}


def calcpulseproperties(pulseProfile, nbrComp):
    """rms pulsed flux / fraction and per-harmonic terms, formulas as pulseprofile.py:596-630
    (including its subtraction of the squared variance terms)."""
    ppBins = pulseProfile["ppBins"]
    ctRate = pulseProfile["countRate"]
    ctRateErr = pulseProfile["countRateErr"]
    N = len(ppBins)
    FrmsHarms = np.zeros(nbrComp)
    for kk in range(1, nbrComp + 1):
        c = np.cos(kk * 2 * np.pi * ppBins)
        s = np.sin(kk * 2 * np.pi * ppBins)
        ak = (1 / N) * np.sum(ctRate * c)
        sak = (1 / N ** 2) * np.sum(ctRateErr ** 2 * c ** 2)
        bk = (1 / N) * np.sum(ctRate * s)
        sbk = (1 / N ** 2) * np.sum(ctRateErr ** 2 * s ** 2)
        FrmsHarms[kk - 1] = (ak ** 2 + bk ** 2) - (sak ** 2 + sbk ** 2)
    Frms = np.sqrt(np.sum(FrmsHarms) * 2)
    return {'pulsedFlux': Frms, 'pulsedFraction': Frms / np.mean(ctRate), 'harmonicPulsedFractions': FrmsHarms}


def calcuncertaintypulseproperties(pulseProfile, nbrComp, nbrOfSimulations=1000, rng=None):
    """Monte Carlo 1-sigma of the pulsed properties (pulseprofile.py:633-668): 1000 profiles drawn
    from N(countRate, countRateErr), a normal fitted to each property. ``rng`` defaults to numpy's
    global generator, as the reference draws from it."""
    from scipy.stats import norm

    draw = np.random.normal if rng is None else rng.normal
    sim = copy.deepcopy(pulseProfile)
    flux = np.zeros(nbrOfSimulations)
    frac = np.zeros(nbrOfSimulations)
    harm = np.zeros((nbrOfSimulations, nbrComp))
    for jj in range(nbrOfSimulations):
        sim["countRate"] = draw(pulseProfile["countRate"], pulseProfile["countRateErr"], size=None)
        p = calcpulseproperties(sim, nbrComp)
        flux[jj], frac[jj], harm[jj, :] = p["pulsedFlux"], p["pulsedFraction"], p["harmonicPulsedFractions"]
    _, FrmsErr = norm.fit(flux)
    _, PFrmsErr = norm.fit(frac)
    FrmsHarmsErr = np.array([norm.fit(harm[:, kk])[1] for kk in range(nbrComp)])
    return {'pulsedFluxErr': FrmsErr, 'pulsedFractionErr': PFrmsErr, 'harmonicPulsedFractionsErr': FrmsHarmsErr}


def plotpulseprofile(pulseProfile, outFile='pulseprof', fittedModel=None):
    """Two cycles of the binned profile and the best-fit model, ``outFile``.pdf (pulseprofile.py:671-720)."""
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt

    ppBins = pulseProfile["ppBins"]
    cycle = 2 * np.pi if np.max(ppBins) > 1 else 1
    x = np.append(ppBins, ppBins + cycle)
    y = np.append(pulseProfile["countRate"], pulseProfile["countRate"])
    ye = np.append(pulseProfile["countRateErr"], pulseProfile["countRateErr"])
    fig, ax = plt.subplots(1, figsize=(6, 4.0), dpi=80)
    ax.set_xlabel(r'$\,\mathrm{Phase\,(cycles)}$', fontsize=12)
    ax.set_ylabel(r'$\,\mathrm{Rate\,(counts\,s^{-1})}$', fontsize=12)
    ax.step(x, y, 'k+-', where='mid')
    ax.errorbar(x, y, yerr=ye, fmt='ok')
    if fittedModel is not None:
        ax.plot(x, np.append(fittedModel, fittedModel), 'r-', linewidth=2.0)
    fig.tight_layout()
    fig.savefig(outFile + '.pdf', format='pdf')
    plt.close(fig)


def writetemplatefile(templateFile, fitResultsDict):
    """``templateFile``.txt in the format readPPtemplate reads (pulseprofile.py:723-752)."""
    nbrComp = len([k for k in fitResultsDict if k.startswith('amp_')])
    kind = fitResultsDict["model"].casefold()
    lines = ['model ' + str(fitResultsDict["model"]) + '\n',
             'norm ' + str(fitResultsDict["norm"]) + ' vary True \n']
    for nn in range(1, nbrComp + 1):
        lines.append('amp_%d ' % nn + str(fitResultsDict["amp_%d" % nn]) + ' vary True \n')
        if kind == 'fourier':
            lines.append('ph_%d ' % nn + str(fitResultsDict["ph_%d" % nn]) + ' vary True \n')
        if kind in ('vonmises', 'cauchy'):
            lines.append('cen_%d ' % nn + str(fitResultsDict["cen_%d" % nn]) + ' vary True \n')
            lines.append('wid_%d ' % nn + str(fitResultsDict["wid_%d" % nn]) + ' vary True \n')
    lines += ['chi2 ' + str(fitResultsDict["chi2"]) + '\n', 'dof ' + str(fitResultsDict["dof"]) + '\n',
              'redchi2 ' + str(fitResultsDict["redchi2"]) + '\n']
    with open(templateFile + '.txt', 'w+') as fh:
        fh.writelines(lines)


def main(argv=None):
    """``templatepulseprofile`` CLI (pulseprofile.py:755-796)."""
    parser = argparse.ArgumentParser(description="Build and fit pulse profile from event file")
    parser.add_argument("evtFile", help="Event file", type=str)
    parser.add_argument("timMod", help="Timing model (.par file)", type=str)
    parser.add_argument("-el", "--eneLow", help="lower energy cut, default=0.5 keV", type=float, default=0.5)
    parser.add_argument("-eh", "--eneHigh", help="high energy cut, default=10 keV", type=float, default=10)
    parser.add_argument("-nb", "--nbrBins", help="Number of bins, default = 15", type=int, default=15)
    parser.add_argument("-pm", "--ppmodel", help="fourier (default), vonmises or cauchy", type=str,
                        default='fourier')
    parser.add_argument("-nc", "--nbrComp", help="Number of components, default = 2", type=int, default=2)
    parser.add_argument("-it", "--initTemplateMod", help="Initial template model parameters", type=str,
                        default=None)
    parser.add_argument("-fp", "--fixPhases", help="Fix phases of the initial template", default=False,
                        action=argparse.BooleanOptionalAction)
    parser.add_argument("-fg", "--figure", help="Plot of the pulse profile, 'figure'.pdf", type=str, default=None)
    parser.add_argument("-tf", "--templateFile", help="Output .txt file for the best-fit model", type=str,
                        default=None)
    parser.add_argument("-v", "--verbose", action="count", default=0, help="WARNING if absent, -v: INFO, -vv: DEBUG")
    args = parser.parse_args(argv)
    console_level = ("WARNING", "INFO", "DEBUG")[min(args.verbose, 2)]
    logfile = 'logfile_buildtemplate' if args.templateFile is None else args.templateFile
    configure_logging(console_level=console_level, file_path=logfile + ".log", file_level="INFO", force=True)
    logging.getLogger(__name__).info("\nCLI starting")
    pp = PulseProfileFromEventFile(args.evtFile, args.timMod, args.eneLow, args.eneHigh, args.nbrBins)
    pp.fitpulseprofile(args.ppmodel, args.nbrComp, args.initTemplateMod, args.fixPhases, args.figure,
                       args.templateFile)


if __name__ == '__main__':
    main()

"""Earliest MJD at or before ``Tmjd`` with an integer number of rotations since PEPOCH
(Taylor + glitch terms), with the spin frequency there -- CRIMP v2.3.0
``ephemIntegerRotation.py:25-86``. A per-ToA scalar used only by the .tim writer; the
phase is evaluated on the host with the reference's own NumPy expression
(calcphase.py:80-126) so the written ToAs match CRIMP's digits."""
import argparse
from math import factorial

import numpy as np

from .ephemTmjd import ephemTmjd
from .readtimingmodel import ReadTimingModel


def _model(timMod):
    return ReadTimingModel(timMod).readfulltimingmodel()[0] if isinstance(timMod, str) else timMod


def phase_no_waves(t, timMod):
    """Taylor + glitch phase of one MJD (calcphase.py:73-126 evaluated on a 1-element array)."""
    p = _model(timMod)
    tt = np.atleast_1d(t).astype(float).reshape(-1)
    dt = (tt - p["PEPOCH"]) * 86400.0
    te = 0.0
    for nn in range(1, 14):
        te += (1.0 / factorial(nn)) * p["F%d" % (nn - 1)] * (dt ** nn)
    gl = np.zeros(tt.size)
    ngl = sum(1 for k in p if k.startswith("GLEP_"))
    for jj in range(1, ngl + 1):
        glep = float(p["GLEP_%d" % jj])
        mask = tt >= glep
        if not np.any(mask):
            continue
        g = {b: float(p.get("%s_%d" % (b, jj), 0.0)) for b in ("GLPH", "GLF0", "GLF1", "GLF2", "GLF0D", "GLTD")}
        ta = tt[mask]
        dts = (ta - glep) * 86400.0
        ex = 0.0 if g["GLTD"] == 0.0 else (g["GLTD"] * 86400.0) * (1.0 - np.exp(-(ta - glep) / g["GLTD"]))
        gl[mask] += (g["GLPH"] + g["GLF0"] * dts + 0.5 * g["GLF1"] * dts ** 2 + (1.0 / 6.0) * g["GLF2"] * dts ** 3
                     + g["GLF0D"] * ex)
    return float(np.atleast_1d(te + gl)[0])


def ephemIntegerRotation(Tmjd, timMod, printOutput=False, tol_phase=1e-10, max_iter=10):
    ph0 = phase_no_waves(Tmjd, timMod)
    target = np.floor(ph0)
    t = Tmjd
    for _ in range(max_iter):  # Newton on the phase (ephemIntegerRotation.py:52-59)
        err = phase_no_waves(t, timMod) - target
        if abs(err) < tol_phase:
            break
        t -= (err / ephemTmjd(t, timMod)["freqAtTmjd"]) / 86400.0
    eph = ephemTmjd(t, timMod)
    ph = phase_no_waves(t, timMod)
    out = {"Tmjd_intRotation": t, "freq_intRotation": eph["freqAtTmjd"], "freqdot_intRotation": eph["freqdotAtTmjd"],
           "ph_intRotation": ph, "phase_residual_from_integer": ph - np.round(ph)}
    if printOutput:
        print(f"Input Tmjd = {Tmjd} days. Corresponding phase = {ph0}\n Earliest Tmjd with integer number of "
              f"rotation = {t}. Corresponding frequency = {eph['freqAtTmjd']}. Corresponding phase = {ph}\n "
              f"Phase residual from integer = {out['phase_residual_from_integer']}")
    return out


def main(argv=None):
    """ephemintegerrotation CLI (ephemIntegerRotation.py:89-99)."""
    parser = argparse.ArgumentParser(description="Calculate earliest MJD (and corresponding spin frequency and "
                                                 "rotational phase) that results in an integer number of rotations")
    parser.add_argument("tMJD", help="Time in MJD at which to derive frequency and rotational phase", type=float)
    parser.add_argument("timMod", help="Timing model in text format. A tempo2 .par file should work", type=str)
    parser.add_argument("-po", "--printOutput", help="Print output", default=False,
                        action=argparse.BooleanOptionalAction)
    args = parser.parse_args(argv)
    ephemIntegerRotation(args.tMJD, args.timMod, args.printOutput)


if __name__ == "__main__":
    main()

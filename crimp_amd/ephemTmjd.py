"""Spin frequency and its derivative at an MJD (host; sets the H-test trial frequency of measureToAs,
measureToAs.py:210). Same result dict as CRIMP v2.3.0 ``ephemTmjd.py:19-77``: Taylor terms F0..F12 plus every
glitch with Tmjd >= GLEP (GLF0, GLF1, GLF2 and a GLF0D/GLTD decay). ``Tmjd`` may be an array (element-wise, as
the reference's expressions are) and ``timMod`` an already parsed model dict (values or {value, flag}) as well
as a .par path, so that a ToA loop parses the model once."""
from math import factorial

import numpy as np

from .readtimingmodel import ReadTimingModel, get_parameter_value


def _model(timMod):
    if isinstance(timMod, dict):
        p = {k: get_parameter_value(v) for k, v in timMod.items()}
        for k in range(13):
            p.setdefault("F%d" % k, 0.0)  # absent Taylor terms are 0 (readtimingmodel.py:64-65)
        return p
    return ReadTimingModel(timMod).readfulltimingmodel()[0]


def ephemTmjd(Tmjd, timMod):
    p = _model(timMod)
    dts = (Tmjd - p["PEPOCH"]) * 86400
    f = p["F0"]
    for k in range(1, 13):
        f += (1 / factorial(k)) * p["F%d" % k] * dts ** k
    fd = p["F1"]
    for k in range(2, 13):
        fd += (1 / factorial(k - 1)) * p["F%d" % k] * dts ** (k - 1)
    f_gl, fd_gl = 0, 0
    ngl = len([k for k in p if k.startswith("GLEP_")])
    for j in range(1, ngl + 1):
        ep = p["GLEP_%d" % j]
        after = Tmjd >= ep
        if np.any(after):
            g0, g1, g2 = p["GLF0_%d" % j], p["GLF1_%d" % j], p["GLF2_%d" % j]
            g0d, td = p["GLF0D_%d" % j], p["GLTD_%d" % j]
            d = (Tmjd - ep) * 86400
            f_gl += (g0 + (g1 * d) + (0.5 * g2 * d ** 2) + (g0d * np.exp(-(Tmjd - ep) / td))) * after
            fd_gl += ((g1 + (g2 * d) + (-(g0d / (td * 86400)) * np.exp(-d / (td * 86400)))) * after)
    return {"Tmjd": Tmjd, "freqAtTmjd": f + f_gl, "freqdotAtTmjd": fd + fd_gl}

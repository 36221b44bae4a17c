"""Pulse-profile template reader (input format of the ToA likelihood scan).

Same dictionary as CRIMP's ``readPPtemplate.py`` (v2.3.0, :15-166):
``{'model', 'norm': {'value', 'vary'}, 'nbrComp', 'amp_j': {...}, 'ph_j' | 'cen_j', 'wid_j': {...}}``.
A parameter line is ``<name> <value> vary <True|False>``; 'model' and 'norm' are required, and so
are the first component's parameters.
"""
import numpy as np


def _param(tokens):
    # "<name> <value> vary <bool>": the third token is the vary flag (readPPtemplate.py:64-66)
    return {"value": np.float64(tokens[1]), "vary": tokens[3].lower() == "true"}


def readPPtemplate(tempModPP):
    with open(tempModPP) as fh:
        lines = [ln.strip().split() for ln in fh]
    model = None
    for tok in lines:
        if tok and tok[0].startswith("model"):
            model = tok[1] if tok[0] == "model" else tok[0][len("model"):]
    if model is None:
        raise Exception('The "model" parameter must exist in template file')
    kind = model.casefold()
    if kind not in ("fourier", "vonmises", "cauchy"):
        raise Exception("Model {} is not supported yet; fourier, vonmises, cauchy are supported".format(model))
    out = {"model": model}
    norm = None
    comps = []
    for tok in lines:
        if tok and tok[0] == "norm":
            norm = _param(tok)
        elif tok and tok[0].startswith("amp_"):
            comps.append(int(tok[0].split("_")[1]))
    if norm is None:
        raise Exception('The "norm" parameter must exist in template file')
    out["norm"] = norm
    out["nbrComp"] = np.int64(max(comps)) if comps else np.int64(0)
    names = ("amp", "ph") if kind == "fourier" else ("amp", "cen", "wid")
    for j in range(1, int(out["nbrComp"]) + 1):
        for nm in names:
            key = "%s_%d" % (nm, j)
            for tok in lines:
                if tok and tok[0] == key:
                    out[key] = _param(tok)
    required = ["%s_1" % nm for nm in names]
    if any(out.get(k) is None for k in required):
        raise Exception("Parameters of the first component, %s, must exist in template file" % ", ".join(required))
    return out

""".par timing-model reader (host side of the calcphase boundary).

Restates the behaviour of CRIMP's ``readtimingmodel.py`` (v2.3.0):
  * Taylor terms PEPOCH, F0..F12, absent ones 0.0                 (:56-83)
  * glitches keyed by the suffix of every ``GLEP_<id>`` line; GLPH/GLF0/GLF1/
    GLF2/GLF0D default 0, GLTD default 1                          (:86-149)
  * WAVEEPOCH, WAVE_OM (+flag) and WAVEj A/B pairs                (:152-209)
  * readfulltimingmodel() -> (values, flags, both), adding TRACK=-2 when present (:212-233, :324-335)
  * a value token goes through complex(tok).real, a flag is 0/1 or 0 (:38-53)
"""
import re

import numpy as np

_TAYLOR = ["PEPOCH"] + ["F%d" % i for i in range(13)]
_GLITCH = (("GLEP_", 0.0), ("GLPH_", 0.0), ("GLF0_", 0.0), ("GLF1_", 0.0), ("GLF2_", 0.0), ("GLF0D_", 0.0),
           ("GLTD_", 1.0))


def _value_flag(tokens):
    value = complex(tokens[0]).real
    flag = 0
    if len(tokens) > 1:
        try:
            f = int(float(tokens[1]))
            flag = f if f in (0, 1) else 0
        except (ValueError, OverflowError):
            flag = 0
    return value, flag


class ReadTimingModel:
    """Reads a .par file into (values, flags, {value, flag}) dictionaries."""

    def __init__(self, timMod):
        self.timMod = timMod

    def _lines(self):
        with open(self.timMod) as fh:
            return [ln.lstrip() for ln in fh]

    def readtaylorexpansion(self):
        vals = {k: np.float64(0) for k in _TAYLOR}
        flags = {k: 0 for k in _TAYLOR}
        both = {k: {"value": np.float64(0), "flag": 0} for k in _TAYLOR}
        for ln in self._lines():
            tok = ln.split()
            if len(tok) >= 2 and tok[0] in vals:
                v, f = _value_flag(tok[1:])
                vals[tok[0]], flags[tok[0]] = v, f
                both[tok[0]] = {"value": v, "flag": f}
        return vals, flags, both

    def readglitches(self):
        lines = self._lines()
        ids = []
        for ln in lines:
            if ln.startswith("GLEP_"):
                m = re.match(r"GLEP_(\S+)", ln)
                if m:
                    ids.append(m.group(1))
        vals, flags, both = {}, {}, {}
        for gid in ids:
            for base, dv in _GLITCH:
                key = base + gid
                vals[key] = np.float64(dv)
                flags[key] = 0
                both[key] = {"value": np.float64(dv), "flag": 0}
        keys = set(vals)
        for ln in lines:
            tok = ln.split()
            if len(tok) >= 2 and tok[0] in keys:
                v, f = _value_flag(tok[1:])
                vals[tok[0]], flags[tok[0]] = v, f
                both[tok[0]] = {"value": v, "flag": f}
        return vals, flags, both

    def readwaves(self):
        lines = self._lines()
        vals, flags, both = {}, {}, {}
        harmonics = set()
        for ln in lines:
            tok = ln.split()
            if tok and tok[0].startswith("WAVE"):
                m = re.match(r"WAVE(\d+)$", tok[0])
                if m:
                    harmonics.add(int(m.group(1)))
        for ln in lines:
            tok = ln.split()
            if len(tok) >= 2 and tok[0] == "WAVEEPOCH":
                vals["WAVEEPOCH"] = complex(tok[1]).real
                both["WAVEEPOCH"] = {"value": vals["WAVEEPOCH"], "flag": None}
            elif len(tok) >= 2 and tok[0] == "WAVE_OM":
                v, f = _value_flag(tok[1:])
                vals["WAVE_OM"], flags["WAVE_OM"] = v, f
                both["WAVE_OM"] = {"value": v, "flag": f}
        for j in sorted(harmonics):
            for ln in lines:
                if ln.startswith("WAVE%d " % j) or ln.startswith("WAVE%d\t" % j):
                    tok = ln.split()
                    if len(tok) >= 3:
                        ab = {"A": complex(tok[1]).real, "B": complex(tok[2]).real}
                        vals["WAVE%d" % j] = ab
                        both["WAVE%d" % j] = {"value": dict(ab), "flag": None}
                    break
        return vals, flags, both

    def readfulltimingmodel(self):
        te = self.readtaylorexpansion()
        gl = self.readglitches()
        wv = self.readwaves()
        vals = {**te[0], **gl[0], **wv[0]}
        flags = {**te[1], **gl[1], **wv[1]}
        both = {**te[2], **gl[2], **wv[2]}
        if self.readmiscellaneous().get("TRACK") == -2:
            vals["TRACK"] = -2.0
            both["TRACK"] = {"value": -2.0, "flag": 0}
        return vals, flags, both

    def readstatistics(self):
        out = {"CHI2R": None, "CHI2R_DOF": None, "NTOA": None, "TRES": None}
        for ln in self._lines():
            tok = ln.strip().split()
            if not tok:
                continue
            key = tok[0].upper()
            try:
                if key == "CHI2R":
                    out["CHI2R"] = float(tok[1])
                    if len(tok) > 2:
                        out["CHI2R_DOF"] = int(tok[2])
                elif key == "NTOA":
                    out["NTOA"] = int(tok[1])
                elif key == "TRES":
                    out["TRES"] = float(tok[1])
            except (ValueError, IndexError):
                pass
        return out

    def readmiscellaneous(self):
        schema = {"PSR": str, "RAJ": str, "DECJ": str, "POSEPOCH": float, "DMEPOCH": float, "START": float,
                  "FINISH": float, "TZRMJD": float, "TZRFRQ": float, "TZRSITE": str, "CLK": str, "UNITS": str,
                  "EPHEM": str, "TRACK": float}
        out = {k: None for k in schema}
        for ln in self._lines():
            tok = ln.strip().split()
            if tok and tok[0].upper() in schema:
                try:
                    out[tok[0].upper()] = schema[tok[0].upper()](tok[1])
                except (IndexError, ValueError):
                    pass
        return out


def get_parameter_value(entry):
    """Plain numbers pass through; a {'value', 'flag'} dict yields its value (readtimingmodel.py:309-321)."""
    if isinstance(entry, dict) and {"value", "flag"} <= set(entry.keys()):
        return entry.get("value")
    return entry

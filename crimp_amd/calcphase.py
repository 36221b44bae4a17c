"""Drop-in ``calcphase`` / ``Phases`` running on the MI355X.

Mirrors CRIMP v2.3.0 ``calcphase.py`` (:20-176): same signatures, same return
shapes (input shape restored, Python floats for a scalar input), same
``TypeError`` for a timing model that is neither a dict nor a path. The phase
evaluation itself is the fp64 HIP kernel behind ``crimp_calcphase``
(csrc/crimp_hip.hip, section 3); there is no NumPy fallback.

Accepts a torch CUDA tensor as ``timeMJD`` too; the result then stays on the
device (tensors of the input shape).
"""
import os

import numpy as np

from . import ops
from ._native import _is_torch
from .readtimingmodel import ReadTimingModel, get_parameter_value

PART_TAYLOR, PART_GLITCH, PART_WAVES = 1, 2, 4


class Phases:
    """Phases of an array of MJD times under a .par model (calcphase.py:20-149)."""

    def __init__(self, timeMJD, timMod):
        self._orig_shape = tuple(timeMJD.shape) if _is_torch(timeMJD) else np.shape(timeMJD)
        if _is_torch(timeMJD):
            import torch
            self.timeMJD = timeMJD.reshape(-1).to(torch.float64).contiguous()
        else:
            self.timeMJD = np.atleast_1d(timeMJD).astype(float).reshape(-1)
        if isinstance(timMod, dict):
            self.timModParam = self._normalize_timdict(timMod)
        elif isinstance(timMod, (str, os.PathLike)):
            self.timModParam = ReadTimingModel(str(timMod)).readfulltimingmodel()[0]
        else:
            raise TypeError("timMod must be a dict or path to a .par file")

    @staticmethod
    def _normalize_timdict(d):
        return {k: get_parameter_value(v) for k, v in d.items()}

    def _run(self, parts):
        total, _ = ops.calcphase(self.timeMJD, self.timModParam, parts=parts, want_folded=False)
        return total

    def taylorexpansion(self):
        return self._run(PART_TAYLOR)

    def glitches(self):
        return self._run(PART_GLITCH)

    def waves(self):
        # calcphase.py:135-149: the harmonics are WAVE1 .. WAVE(n-2) of the n WAVE* keys (WAVEEPOCH and WAVE_OM
        # among them); with none -- no WAVE* key at all, or only the epoch and OM -- the loop adds nothing and the
        # reference returns the scalar 0 * F0 (KeyError without F0, as there)
        nharm = sum(1 for k in self.timModParam if k.startswith("WAVE")) - 2
        if nharm <= 0:
            return 0 * self.timModParam["F0"]
        return self._run(PART_WAVES)


def calcphase(timeMJD, timMod):
    """(total phase, cycle-folded phase in [0,1)) -- calcphase.py:152-176."""
    ph = Phases(timeMJD, timMod)
    total, folded = ops.calcphase(ph.timeMJD, ph.timModParam, parts=PART_TAYLOR | PART_GLITCH | PART_WAVES)
    if ph._orig_shape == ():
        return float(total[0]), float(folded[0])
    return total.reshape(ph._orig_shape), folded.reshape(ph._orig_shape)

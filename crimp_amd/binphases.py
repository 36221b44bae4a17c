"""Folded-phase histogram (binphases.py:9-39 of CRIMP v2.3.0): bins over [0,1) or [0,2pi),
numpy.histogram edge semantics. Host version for one array; measureToAs bins every interval
at once on the device (ops.binphases_counts)."""
import numpy as np


def binphases(phases, nbrBins=15):
    ph = np.asarray(phases)
    if ((ph >= 0) & (ph <= 1)).all():
        upper = 1
    elif ((ph >= 0) & (ph <= 2 * np.pi)).all():
        upper = 2 * np.pi
    else:
        raise Exception('Array in not cycle folded between [0,1) or [0, 2*pi)')
    centres = np.linspace(0, upper, nbrBins, endpoint=False) + (upper / nbrBins) / 2
    cts = np.histogram(ph, bins=np.linspace(0, upper, nbrBins + 1, endpoint=True))[0]
    return {'ppBins': centres, 'ppBinsRange': (upper / nbrBins) / 2, 'ctsBins': cts, 'ctsBinsErr': np.sqrt(cts)}

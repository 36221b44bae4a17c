"""Fixture generator for the config-4 parity windows (tests/test_gpu_fullsize.py::test_config4_windows_vs_oracle).

Config 4: 1e8 photons (T = 1e7 s, p = 0.05, f0 = 7.123456789 Hz, fdot = -1e-12, seed 1),
2-D H-test m = 20 over 1e5 f (step 1/(10 T)) x 100 log10|fdot| rows np.linspace(-13.5, -11.5, 100). Contiguous
windows of trials are evaluated over ALL 1e8 photons by the oracle twice:

* ``ref``:  the reference's operation order (crimp_oracle.c trial_sums: a = 2 pi (k+1) (f dt + c2 dt^2) rounded in
            fp64 exactly as periodsearch.py:93-98, :118-123 builds it) -- what CRIMP's NumPy path returns;
* ``true``: the same formula with the argument carried exactly (trial_sums_true, double-double phase in cycles) --
            the value of the formula on these inputs, which measures the reference's own argument rounding.

The oracle needs ~16 s of 8 CPU cores per trial and variant at 1e8 photons x 20 harmonics, too slow for a GPU test,
so the values are committed (tests/golden/config4_windows.npz, ~3 KB) together with checksums of the photon times,
which the GPU test regenerates with the same seeded generator and checks before comparing.

usage: python tests/golden/gen_config4_windows.py [threads]   (~40 min on 8 cores)
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from crimp_amd.synth import pulsed_events  # noqa: E402
from oracle import oracle as O  # noqa: E402

N, SPAN, F0, FDOT, M = 100_000_000, 1.0e7, 7.123456789, -1.0e-12, 100_000
FD = np.linspace(-13.5, -11.5, 100)
FREQ = F0 + (np.arange(M) - M // 2) / (10.0 * SPAN)
# (fd row, first f index, count): a far row at the grid's start, 32 noise trials beside the peak in the row closest
# to the injected fdot (log10 1e-12 = -12: row 74 = -12.005), and the peak itself with its neighbours
WINDOWS = [(0, 0, 32), (74, M // 2 + 4, 32), (74, M // 2 - 2, 4)]


def photon_checksums(t):
    return np.array([t[0], t[-1], t[N // 3], t[2 * N // 3], float(np.sum(t - t[0]))])


def main():
    threads = int(sys.argv[1]) if len(sys.argv) > 1 else (os.cpu_count() or 1)
    O.set_threads(threads)
    t1 = time.time()
    t = pulsed_events(N, SPAN, F0, pulsed_frac=0.05, fdot=FDOT, seed=1)
    print("photons generated in %.1f s" % (time.time() - t1), flush=True)
    rows, cols, ref, true = [], [], [], []
    for r, j0, cnt in WINDOWS:
        f = FREQ[j0:j0 + cnt]
        fd = FD[r:r + 1]
        for exact, dst in ((False, ref), (True, true)):
            t1 = time.time()
            dst.append(O.search(t, f, 20, freq_dot=fd, stat="h", exact_argument=exact))
            print("row %d f[%d:%d] %s: %.1f s" % (r, j0, j0 + cnt, "true" if exact else "ref", time.time() - t1),
                  flush=True)
        rows.append(np.full(cnt, r))
        cols.append(np.arange(j0, j0 + cnt))
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "config4_windows.npz")
    np.savez(out, row=np.concatenate(rows), col=np.concatenate(cols), ref=np.concatenate(ref),
             true=np.concatenate(true), fd=FD, checksums=photon_checksums(t), n=N, span=SPAN, f0=F0, fdot=FDOT, m=M)
    print("wrote", out)


if __name__ == "__main__":
    main()

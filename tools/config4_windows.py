"""Config-4 parity windows on the GPU: the exact (default) and fp64 paths over the trial windows of
tests/golden/config4_windows.npz, against the oracle's reference-order values (``ref``) and exact-argument values
(``true``) committed there. Prints the error distributions as JSON (one line) for DESIGN.md section 8.
usage: python tools/config4_windows.py"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
from crimp_amd import ops, _native as N  # noqa: E402
from crimp_amd.synth import pulsed_events  # noqa: E402
from gen_config4_windows import FD, FREQ, M, N as NPH, SPAN, F0, FDOT, WINDOWS, photon_checksums  # noqa: E402


def stats(e):
    return {"max": float(e.max()), "median": float(np.median(e)), "n_over_1e-6": int((e > 1e-6).sum())}


def main():
    fx = np.load(os.path.join(ROOT, "tests", "golden", "config4_windows.npz"))
    t_h = pulsed_events(NPH, SPAN, F0, pulsed_frac=0.05, fdot=FDOT, seed=1)
    same = bool(np.array_equal(photon_checksums(t_h), fx["checksums"]))
    dev = torch.device("cuda", 0)
    t = torch.as_tensor(t_h, device=dev)
    t0 = (t_h[0] + t_h[-1]) / 2
    f = torch.as_tensor(FREQ, device=dev)
    fd = torch.as_tensor(FD, device=dev)
    got, got64, nfix = [], [], 0
    for r, j0, cnt in WINDOWS:
        got.append(ops.search(t, t0, f, 20, 1, log10_negfdot=fd, first=r * M + j0, count=cnt).cpu().numpy())
        nfix += N.load().crimp_last_fixups()
        got64.append(ops.search(t, t0, f, 20, 1, log10_negfdot=fd, first=r * M + j0, count=cnt,
                                precision="f64").cpu().numpy())
    h, h64, ref, tru = np.concatenate(got), np.concatenate(got64), fx["ref"], fx["true"]
    rel = lambda a, b: np.abs(a - b) / np.abs(b)  # noqa: E731
    out = {"photons_identical": same, "trials": int(h.size), "fixups": int(nfix),
           "exact_vs_ref": stats(rel(h, ref)), "exact_vs_true": stats(rel(h, tru)),
           "f64_vs_ref": stats(rel(h64, ref)), "f64_vs_true": stats(rel(h64, tru)),
           "ref_vs_true": stats(rel(ref, tru)), "H_range": [float(ref.min()), float(ref.max())],
           "rows": [[int(a), float(b), float(c), float(d), float(e)] for a, b, c, d, e in
                    zip(range(h.size), ref, tru, h, h64)]}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

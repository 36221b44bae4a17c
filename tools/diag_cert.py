"""Diagnostic of the exact path's certificate on correlated inputs (tests/test_gpu_certificate.py): for each input,
the worst trials of the default result against the fp64 path, with the raw kernel value, the fix-up flag and the
oracle's reference-order and exact-argument values. Prints one JSON line.
usage: python tools/diag_cert.py [nharm stat [precision [input]]]  (precision: default | exact)"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from crimp_amd import ops, _native as N  # noqa: E402
from oracle import oracle as O  # noqa: E402
from test_gpu_certificate import _correlated_inputs  # noqa: E402


def main():
    nharm = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    stat = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    prec = sys.argv[3] if len(sys.argv) > 3 else "exact"
    prec = None if prec == "default" else prec
    only = sys.argv[4] if len(sys.argv) > 4 else None
    O.set_threads(16)
    dev = torch.device("cuda", 0)
    f0, inputs = _correlated_inputs()
    f_h = f0 + (np.arange(8192) - 4096) / 1.0e7
    f = torch.as_tensor(f_h, device=dev)
    out = {}
    for name, t_h in inputs.items():
        if only and name != only:
            continue
        t = torch.as_tensor(t_h, device=dev)
        t0 = (t_h[0] + t_h[-1]) / 2
        z = ops.search(t, t0, f, nharm, stat, precision=prec).cpu().numpy()
        nfix = N.load().crimp_last_fixups()
        path = N.load().crimp_last_search_path()
        raw = ops.search(t, t0, f, nharm, stat, flags=N.FLAG_NO_FIXUP, precision=prec).cpu().numpy()
        z64 = ops.search(t, t0, f, nharm, stat, precision="f64").cpu().numpy()
        e = np.abs(z - z64) / np.abs(z64)
        er = np.abs(raw - z64) / np.abs(z64)
        worst = np.argsort(-np.maximum(e, er))[:8]
        sh = "h" if stat else "z2"
        ref = O.search(t_h, f_h[worst], nharm, stat=sh)
        tru = O.search(t_h, f_h[worst], nharm, stat=sh, exact_argument=True)
        out[name] = {"path": path, "nfix": int(nfix), "max_e": float(e.max()), "max_raw": float(er.max()),
                     "n_raw_over": int((er > 1e-6).sum()), "z64_min": float(np.abs(z64).min()),
                     "worst": [[int(i), float(z[i]), float(raw[i]), float(z64[i]), float(r), float(q)]
                               for i, r, q in zip(worst, ref, tru)]}
        print(name, json.dumps(out[name]), flush=True)


if __name__ == "__main__":
    main()

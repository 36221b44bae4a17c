"""Per-harmonic error of the NUFFT on the certificate test's duplicated-photon input (tests/test_gpu_certificate.py):
Z^2_m of one trial for m = 1..M by the NUFFT (raw, fix-up off) under spread/lane variants, the fp64 kernel, and the
oracle in the reference's operation order and with the argument carried exactly. Prints one line per m.
usage: python tools/diag_nufft_harm.py [trial [M [input]]]"""
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

trial = int(sys.argv[1]) if len(sys.argv) > 1 else 7429
M = int(sys.argv[2]) if len(sys.argv) > 2 else 20
name = sys.argv[3] if len(sys.argv) > 3 else "duplicated"
O.set_threads(16)
f0, inputs = _correlated_inputs()
t_h = inputs[name]
f_h = f0 + (np.arange(8192) - 4096) / 1.0e7
dev = torch.device("cuda", 0)
t = torch.as_tensor(t_h, device=dev)
f = torch.as_tensor(f_h, device=dev)
t0 = (t_h[0] + t_h[-1]) / 2
variants = {"auto": {}, "mfma": {"CRIMP_NUFFT_SPREAD": "mfma"}, "lanes1": {"CRIMP_NUFFT_LANES": "1"},
            "nofused": {"CRIMP_NUFFT_FUSED": "0"}, "generic": {"CRIMP_NUFFT_ROWS4096": "0"}}
print("plan", N.last_nufft_plan() if False else "", flush=True)
for m in range(1, M + 1):
    row = []
    for v, env in variants.items():
        for k in ("CRIMP_NUFFT_SPREAD", "CRIMP_NUFFT_LANES", "CRIMP_NUFFT_FUSED", "CRIMP_NUFFT_ROWS4096"):
            os.environ.pop(k, None)
        os.environ.update(env)
        z = ops.search(t, t0, f, m, 0, flags=N.FLAG_NO_FIXUP).cpu().numpy()[trial]
        row.append((v, z))
        if m == 1 and v == "auto":
            print("plan", N.last_nufft_plan(), flush=True)
    for k in ("CRIMP_NUFFT_SPREAD", "CRIMP_NUFFT_LANES", "CRIMP_NUFFT_FUSED", "CRIMP_NUFFT_ROWS4096"):
        os.environ.pop(k, None)
    z64 = ops.search(t, t0, f, m, 0, precision="f64").cpu().numpy()[trial]
    zx = ops.search(t, t0, f, m, 0, precision="exact").cpu().numpy()[trial]
    ref = O.search(t_h, f_h[trial:trial + 1], m)[0]
    tru = O.search(t_h, f_h[trial:trial + 1], m, exact_argument=True)[0]
    print("m=%2d true %.12f ref %+.2e f64 %+.2e exact %+.2e | %s" % (
        m, tru, (ref - tru) / tru, (z64 - tru) / tru, (zx - tru) / tru,
        " ".join("%s %+.2e" % (v, (z - tru) / tru) for v, z in row)), flush=True)

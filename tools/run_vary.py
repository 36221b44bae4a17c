"""readvaryparam fit time (7 golden intervals, amplitudes 1-2 freed with the norm): the interval-batched
host driver vs the one-interval-at-a-time driver (tools/_old_toafit_vary.py, if present)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from test_gpu_parity import _golden_rows, _vary_template, gpath  # noqa: E402
from crimp_amd.readPPtemplate import readPPtemplate  # noqa: E402
from crimp_amd import toafit_vary  # noqa: E402

g, iv, _ = _golden_rows()
E = iv["ToA_exposure"].to_numpy()[g["ids"]]
tm = _vary_template(readPPtemplate(gpath("1e2259_template.txt")), {"norm", "amp_1", "amp_2"})
mods = [("batched", toafit_vary)]
try:
    import _old_toafit_vary
    mods.append(("per-interval", _old_toafit_vary))
except ImportError:
    pass
res = {}
for rep in range(2):
    for name, m in mods:
        t = time.perf_counter()
        r = m.VaryParamFitter(g["folded"], g["offsets"], E, tm).fit()
        dt = time.perf_counter() - t
        res[name] = r
        print("%-13s %d intervals: %.3f s, %d evaluations" % (name, len(r["phShi"]), dt, int(np.sum(r["evaluations"]))), flush=True)
if len(res) == 2:
    a, b = res["batched"], res["per-interval"]
    print("identical phShi/LL/UL/theta:", all(np.array_equal(a[k], b[k]) for k in ("phShi", "phShi_LL", "phShi_UL", "theta", "LLmax")))

"""HBM bytes per launch of each NUFFT kernel from tools/pmc_nufft.sh's FETCH_SIZE / WRITE_SIZE passes (config 3 over
tools/run_search.py with CRIMP_PRECISION=nufft): bytes = (2 x FETCH_SIZE + WRITE_SIZE) x 1024 per dispatch (the
guide's gfx950 FETCH_SIZE correction). Prints the JSON record bench.py reads (profiles/r05/pmc_nufft_traffic.json).
usage: python tools/pmc_nufft_json.py <pmc output dir, e.g. gpurun_out/pmc_nufft>"""
import csv
import glob
import json
import sys
from collections import defaultdict

root = sys.argv[1]
val = defaultdict(lambda: defaultdict(float))
disp = defaultdict(lambda: defaultdict(set))
for fn in glob.glob(root + "/p*/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(fn)):
        c = row["Counter_Name"]
        if c not in ("FETCH_SIZE", "WRITE_SIZE"):
            continue
        name = row.get("Kernel_Name", "").split("(")[0].replace("void ", "").split("<")[0]
        if not name.startswith("k_nu_"):
            continue
        val[name][c] += float(row["Counter_Value"])
        disp[name][c].add((fn, row.get("Dispatch_Id", "")))
out = {}
for name, cs in val.items():
    nf, nw = len(disp[name]["FETCH_SIZE"]), len(disp[name]["WRITE_SIZE"])
    if nf and nw:
        out[name] = {"fetch_kb_per_launch": cs["FETCH_SIZE"] / nf, "write_kb_per_launch": cs["WRITE_SIZE"] / nw,
                     "bytes_per_launch": (2 * cs["FETCH_SIZE"] / nf + cs["WRITE_SIZE"] / nw) * 1024.0}
print(json.dumps({"photons": 10000000, "trials": 1000000, "nharm": 2, "kernels": out,
                  "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes, tools/pmc_nufft.sh) over "
                            "tools/run_search.py with CRIMP_PRECISION=nufft; bytes per launch = (2 x FETCH_SIZE + "
                            "WRITE_SIZE) x 1024 (gfx950 FETCH_SIZE correction)"}, indent=1))

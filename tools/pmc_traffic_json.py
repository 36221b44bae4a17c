"""HBM bytes per config-3 search from the FETCH_SIZE / WRITE_SIZE passes of tools/pmc_traffic_quick.sh (sums over
the k_search_exact launches of one search, kB): bytes = (2 x FETCH_SIZE + WRITE_SIZE) x 1024 (the guide's gfx950
FETCH_SIZE correction). Prints the JSON record bench.py reads (profiles/<round>/pmc_traffic.json).
usage: python tools/pmc_traffic_json.py <gpurun_out dir>"""
import csv
import glob
import json
import sys


def total(root, counter):
    v, disp = 0.0, set()
    for fn in glob.glob("%s/tr_%s/**/*counter_collection.csv" % (root, counter), recursive=True):
        for row in csv.DictReader(open(fn)):
            if "k_search_exact" in row.get("Kernel_Name", "") and row["Counter_Name"] == counter:
                v += float(row["Counter_Value"])
                disp.add(row.get("Dispatch_Id", ""))
    return v, len(disp)


root = sys.argv[1]
f, nf = total(root, "FETCH_SIZE")
w, nw = total(root, "WRITE_SIZE")
if nf == 0 or nw == 0:
    sys.exit("no k_search_exact counter rows found")
print(json.dumps({"photons": 10000000, "trials": 1000000, "nharm": 2, "launches": nf, "fetch_size_kb": f,
                  "write_size_kb": w, "bytes_per_search": (2 * f + w) * 1024.0,
                  "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes, tools/pmc_traffic_quick.sh) over "
                            "tools/run_search.py, k_search_exact launches of one search; bytes = (2 x FETCH_SIZE + "
                            "WRITE_SIZE) x 1024 (gfx950 FETCH_SIZE correction; 8-byte loads and 64-bit atomics are "
                            "outside the guide's calibrated widths)"}, indent=1))

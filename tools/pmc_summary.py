"""Sum rocprofv3 counter_collection CSVs per counter for one kernel-name pattern, with per-dispatch means.
usage: python tools/pmc_summary.py <rocprof output dir> [kernel-name substring]"""
import csv
import glob
import sys
from collections import defaultdict

root, pat = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "k_search_exact"
tot, durs = defaultdict(float), {}
disp = defaultdict(set)
for fn in glob.glob(root + "/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(fn)):
        if pat in row.get("Kernel_Name", ""):
            tot[row["Counter_Name"]] += float(row["Counter_Value"])
            disp[row["Counter_Name"]].add((fn, row.get("Dispatch_Id", row.get("Correlation_Id", ""))))
ndisp = defaultdict(int)
for fn in glob.glob(root + "/**/*kernel_trace.csv", recursive=True):
    for row in csv.DictReader(open(fn)):
        if pat in row.get("Kernel_Name", ""):
            durs[fn] = durs.get(fn, 0) + (int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
            ndisp[fn] += 1
for k in sorted(tot):
    n = max(1, len(disp[k]))
    print("%-28s %.4g" % (k, tot[k]))
    print("%-28s %.4g  (per dispatch, %d dispatches)" % (k + "/disp", tot[k] / n, n))
print("kernel ns per pass:", sorted(durs.values()))
print("dispatches per pass:", sorted(ndisp.values()))

"""Sum rocprofv3 counter_collection CSVs per counter for one kernel-name pattern."""
import csv
import glob
import sys
from collections import defaultdict

root, pat = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "k_search_exact"
tot, durs = defaultdict(float), {}
for fn in glob.glob(root + "/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(fn)):
        if pat in row.get("Kernel_Name", ""):
            tot[row["Counter_Name"]] += float(row["Counter_Value"])
for fn in glob.glob(root + "/**/*kernel_trace.csv", recursive=True):
    for row in csv.DictReader(open(fn)):
        if pat in row.get("Kernel_Name", ""):
            durs[fn] = durs.get(fn, 0) + (int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
for k in sorted(tot):
    print("%-28s %.4g" % (k, tot[k]))
print("kernel ns per pass:", sorted(durs.values()))

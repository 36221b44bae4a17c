"""Timeline of one call from a rocprofv3 trace directory (kernel + HIP API + memory copies, CSV output): prints every
event (start relative to the window, duration, name) in the window around the Nth-from-last kernel whose name contains
PAT. usage: python tools/trace_timeline.py <dir> <PAT> [N=2] [before_us=1500] [after_us=4500]"""
import csv
import glob
import sys

d, pat = sys.argv[1], sys.argv[2]
nth = int(sys.argv[3]) if len(sys.argv) > 3 else 2
before = float(sys.argv[4]) if len(sys.argv) > 4 else 1500.0
after = float(sys.argv[5]) if len(sys.argv) > 5 else 4500.0
skip = ("hipGetLastError", "hipGetDevice", "__hipPush", "__hipPop", "hipSetDevice", "hipStreamGetCaptureInfo",
        "hipPeekAtLastError")
ev = []
for fn in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(fn)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K " + r["Kernel_Name"][:60]))
for fn in glob.glob(d + "/**/*hip_api_trace.csv", recursive=True):
    for r in csv.DictReader(open(fn)):
        if not r["Function"].startswith(skip):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "A " + r["Function"]))
for fn in glob.glob(d + "/**/*memory_copy_trace.csv", recursive=True):
    for r in csv.DictReader(open(fn)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "C " + r.get("Direction", "copy")))
ev.sort()
hits = [e for e in ev if e[2].startswith("K") and pat in e[2]]
g = hits[-nth]
start, end = g[0] - before * 1e3, g[1] + after * 1e3
for e in ev:
    if start <= e[0] <= end:
        print("%9.1f %8.1f  %s" % ((e[0] - start) / 1e3, (e[1] - e[0]) / 1e3, e[2]))

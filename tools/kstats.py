"""Print a rocprofv3 kernel_stats.csv as a short table: name, calls, average and total microseconds."""
import csv
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof_nufft/run_kernel_stats.csv"
for r in csv.DictReader(open(path)):
    print("%-44s calls=%-5s avg=%9.1f us  tot=%10.1f us" % (r["Name"][:44], r["Calls"], float(r["AverageNs"]) / 1e3,
                                                         float(r["TotalDurationNs"]) / 1e3))

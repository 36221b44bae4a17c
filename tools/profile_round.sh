#!/bin/bash
# Round evidence on one GPU: (1) the default bench under rocprofv3 kernel-trace stats, (2) FETCH_SIZE and
# WRITE_SIZE of one config-3 search (tools/run_search.py) in separate PMC passes, (3) the traffic record for
# bench.py (2 x FETCH_SIZE + WRITE_SIZE of the k_search_exact launches, MI355X_MICROARCH.md HBM section).
# Output under gpurun_out/$TAG; copy what is judged into profiles/$TAG.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r02}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
step() { echo "[$1] rc=$2"; [ "$2" -ne 0 ] && exit "$2"; return 0; }
timeout -k 10 ${BENCH_TIMEOUT:-420} rocprofv3 --kernel-trace --stats -d "$OUT/bench_trace" -o bench --output-format csv \
    -- python3 bench.py ${BENCH_ARGS:-} > "$OUT/bench_traced.log" 2>&1
step bench-trace $?
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c --kernel-trace -d "$OUT/pmc_$c" -o pmc --output-format csv \
      -- python3 tools/run_search.py > "$OUT/pmc_$c.log" 2>&1
  step "pmc $c" $?
done
python3 - "$OUT" <<'EOF'
import csv, glob, json, os, sys
out = sys.argv[1]
def total(counter, pat="k_search_exact"):
    s, n = 0.0, 0
    for fn in glob.glob(os.path.join(out, "pmc_" + counter, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(fn)):
            if pat in row.get("Kernel_Name", "") and row["Counter_Name"] == counter:
                s += float(row["Counter_Value"]); n += 1
    return s, n
fetch, nf = total("FETCH_SIZE")
write, nw = total("WRITE_SIZE")
# FETCH_SIZE/WRITE_SIZE are in KB (rocprofv3 derived metrics); FETCH_SIZE x 2 on gfx950 (guide, HBM section)
rec = {"photons": int(os.environ.get("NPH", 10_000_000)), "trials": int(os.environ.get("NTR", 1_000_000)),
       "nharm": int(os.environ.get("NHARM", 2)), "launches": nf,
       "fetch_size_kb": fetch, "write_size_kb": write,
       "bytes_per_search": (2.0 * fetch + write) * 1024.0,
       "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) over tools/run_search.py, k_search_exact "
                 "launches of one search; bytes = (2 x FETCH_SIZE + WRITE_SIZE) x 1024 (gfx950 FETCH_SIZE correction; "
                 "8-byte loads and 64-bit atomics are outside the guide's calibrated widths)"}
json.dump(rec, open(os.path.join(out, "pmc_traffic.json"), "w"), indent=1)
print(json.dumps(rec))
EOF
step summary $?

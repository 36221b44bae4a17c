#!/bin/bash
# rocprofv3 evidence for the dominant kernels: kernel-trace stats + separate PMC passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_${TAG:-r1}
mkdir -p "$OUT"
ARGS=${PROF_ARGS:---steps 2 --warmup 1 --no-cpu}
chk() { local rc=$1; echo "[$2] rc=$rc"; if [ "$rc" -ne 0 ]; then echo "stop after $2"; exit "$rc"; fi; }
timeout -k 10 120 rocprofv3 -L > "$OUT/counters.txt" 2>&1; echo "[list] rc=$?"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o trace --output-format csv -- python bench.py $ARGS > "$OUT/trace.log" 2>&1
chk $? trace
for set in "${PMC1:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU}" \
           "${PMC2:-GRBM_GUI_ACTIVE GRBM_COUNT}" "${PMC3:-FETCH_SIZE}" "${PMC4:-WRITE_SIZE}"; do
  name=$(echo $set | tr ' ' '_' | cut -c1-40)
  timeout -k 10 600 rocprofv3 --pmc $set --kernel-trace -d "$OUT/pmc_$name" -o pmc --output-format csv -- python bench.py --steps 1 --warmup 0 --no-cpu > "$OUT/pmc_$name.log" 2>&1
  chk $? "pmc $set"
done
find "$OUT" -name "*.csv" | head -40

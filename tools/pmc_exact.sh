#!/bin/bash
# rocprofv3 evidence over one workload (RUN, default tools/run_search.py: one config-3 search):
# kernel-trace stats, then one PMC pass per counter set (PMC_SETS, one line each; each under its own time limit),
# summed for the kernels matching PAT (space-separated substrings).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_${TAG:-x}
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o trace --output-format csv -- python3 ${RUN:-tools/run_search.py} > "$OUT/trace.log" 2>&1
rc=$?; echo "[trace] rc=$rc"; [ $rc -ne 0 ] && exit $rc
i=0
while read -r set; do
  [ -z "$set" ] && continue
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $set --kernel-trace -d "$OUT/p$i" -o pmc --output-format csv -- python3 ${RUN:-tools/run_search.py} > "$OUT/p$i.log" 2>&1
  rc=$?; echo "[pass $i: $set] rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done <<SETS
${PMC_SETS:-SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA
SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_LDS
GRBM_GUI_ACTIVE GRBM_COUNT}
SETS
for p in ${PAT:-k_search_exact}; do
  python3 tools/pmc_summary.py "$OUT" "$p" > "$OUT/summary_$p.txt" 2>&1; echo "== $p"; cat "$OUT/summary_$p.txt"
done

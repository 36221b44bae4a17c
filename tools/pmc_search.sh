#!/bin/bash
# PMC passes over one config-3 search (tools/run_search.py); one rocprofv3 run per counter set.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_${TAG:-x}
mkdir -p "$OUT"
timeout -k 10 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1
i=0
while read -r set; do
  [ -z "$set" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace -d "$OUT/p$i" -o pmc --output-format csv -- python3 tools/run_search.py > "$OUT/p$i.log" 2>&1
  rc=$?; echo "[pass $i: $set] rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done <<SETS
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS
SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM
GRBM_GUI_ACTIVE GRBM_COUNT
SETS

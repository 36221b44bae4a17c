#!/bin/bash
# A/B of search-kernel builds (CRIMP_LIB_VARIANT): timing on config 3 and accuracy vs the oracle (cmp_mfma2.py).
# VARIANTS / ACC pick the builds ("default" = libcrimp_hip.so). Each GPU step has its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
chk() { local rc=$1; echo "[$2] rc=$rc" | tee -a "$OUT/ab2_steps.log"; if [ "$rc" -ne 0 ]; then exit "$rc"; fi; }
for v in ${VARIANTS:-default nofract cos6 default nofract cos6}; do
  [ "$v" = default ] && v=""
  REPS=3 CRIMP_LIB_VARIANT=$v timeout -k 10 120 python3 tools/run_search.py >> "$OUT/ab2.log" 2>&1
  chk $? "z2 $v"
done
for v in ${ACC:-default nofract cos6}; do
  [ "$v" = default ] && v=""
  echo "== accuracy lib=${v:-default}" >> "$OUT/ab2.log"
  CRIMP_LIB_VARIANT=$v timeout -k 10 200 python3 tools/cmp_mfma2.py >> "$OUT/ab2.log" 2>&1
  chk $? "acc $v"
done
cat "$OUT/ab2.log"

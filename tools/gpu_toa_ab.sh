#!/bin/bash
# ToA-fit A/B timing: this library vs CRIMP_LIB_VARIANT builds, then the ToA GPU tests; each step time-limited.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
chk() { local rc=$1; echo "[$2] rc=$rc" | tee -a "$OUT/toa_steps.log"; if [ "$rc" -ne 0 ]; then exit "$rc"; fi; }
for v in default ${VARIANTS:-gp1} default ${VARIANTS:-gp1}; do
  [ "$v" = default ] && v=""
  CRIMP_LIB_VARIANT=$v timeout -k 10 120 python3 tools/run_toa.py >> "$OUT/toa_ab.log" 2>&1
  chk $? "toa $v"
done
cat "$OUT/toa_ab.log"

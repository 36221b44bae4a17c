#!/bin/bash
# Search-kernel A/B timing: this library vs variants (CRIMP_LIB_VARIANT), plus the fp64 path, each step time-limited.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
chk() { local rc=$1; echo "[$2] rc=$rc" | tee -a "$OUT/cmp_steps.log"; if [ "$rc" -ne 0 ]; then exit "$rc"; fi; }
for v in ${VARIANTS:-default dup default dup}; do
  [ "$v" = default ] && v=""
  REPS=3 CRIMP_LIB_VARIANT=$v timeout -k 10 120 python3 tools/run_search.py >> "$OUT/cmp.log" 2>&1
  chk $? "z2 $v"
done
NHARM=20 NPH=2000000 REPS=2 timeout -k 10 120 python3 tools/run_search.py >> "$OUT/cmp.log" 2>&1
chk $? h20
CRIMP_PRECISION=f64 NPH=1000000 NTR=100000 REPS=2 timeout -k 10 120 python3 tools/run_search.py >> "$OUT/cmp.log" 2>&1
chk $? f64z2
CRIMP_PRECISION=f64 NHARM=20 NPH=1000000 NTR=20000 REPS=2 timeout -k 10 120 python3 tools/run_search.py >> "$OUT/cmp.log" 2>&1
chk $? f64h20
cat "$OUT/cmp.log"

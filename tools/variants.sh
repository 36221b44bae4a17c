#!/bin/bash
# Time the factorised-search variants (f32-input MFMA, f16 split 1 or 2 tiles/wave) on config 3 and H_20.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in f32 t1 t2 t1 t2; do
  CRIMP_MFMA=$v timeout -k 10 120 python3 tools/run_search.py || exit $?
done
for v in t1 t2; do
  NHARM=20 NTR=100000 CRIMP_MFMA=$v timeout -k 10 120 python3 tools/run_search.py || exit $?
done

#!/bin/bash
# HBM traffic of the harmonic-sum kernel on the config-3 search: FETCH_SIZE and WRITE_SIZE in separate passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_${TAG:-traffic}
mkdir -p "$OUT"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace -d "$OUT/$c" -o pmc --output-format csv -- python3 tools/run_search.py > "$OUT/$c.log" 2>&1
  rc=$?; echo "[pmc $c] rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0

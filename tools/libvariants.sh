#!/bin/bash
# Time kernel experiments built by `make -C crimp_amd/csrc variants` against the default library,
# and check their accuracy (tools/cmp_mfma2.py vs the oracle).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in "" tab dglob "" tab dglob; do
  CRIMP_LIB_VARIANT=$v timeout -k 10 120 python3 tools/run_search.py || exit $?
done
for v in "" tab; do
  echo "== accuracy lib=${v:-default}"
  CRIMP_LIB_VARIANT=$v timeout -k 10 200 python3 tools/cmp_mfma2.py || exit $?
done

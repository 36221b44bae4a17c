# Round-4 session 17: the block H-test queued on a second stream beside the folding and fits (CRIMP_FLAG_ASYNC):
# the e2e tests, then the block-schedule sweep and the timeline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "measure_intervals or measuretoas or search_sets" > gpurun_out/e2e_tests.log 2>&1 || exit $?
BLOCKS=1,d,u6,u10,u12 TRACE_WEIGHTS=1,1,1,1,1,1,1,1 timeout -k 10 500 python -u tools/e2e_breakdown.py > gpurun_out/e2e_async.log 2>&1 || exit $?

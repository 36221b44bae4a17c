# Round-4 session 6: the pipelined measure_intervals (shrinking blocks, GIL switch interval) -- its tests and the
# e2e sweep over block counts --, then the GPU suite, smoke, the driver-style bench, a rocprofv3 kernel-trace profile
# of the bench, and the N=2 rehearsal.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "measure_intervals or fused" > gpurun_out/e2e_tests.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/e2e_breakdown.py > gpurun_out/e2e_breakdown.log 2>&1 || exit $?
STEPS=tests,smoke,bench,prof PYTEST_X= BENCH_ARGS="--steps 20 --warmup 5" bash tools/gpu_round.sh || exit $?
bash tools/rehearse_n2.sh

# Round-4 session 3: after the lazy-norm min fix (k_toa_grid_mf wrote the per-phShift min only for a0 == 0, so the
# lazy-norm launches left it unwritten and k_toa_grid_best's check read stale scratch): the two failing tests, the
# fast-vs-full ToA A/B (digests), the ToA leg breakdown, then the full GPU suite and the bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_certificate.py::test_fast_brute_grid_equals_full_kernel \
  tests/test_distributed_gpu.py::test_nccl_backend_single_rank_on_gpu > gpurun_out/fix_tests.log 2>&1 || exit $?
CRIMP_TOA_GRID_SLOW=1 timeout -k 10 300 python -u tools/ab_toa.py cur > gpurun_out/ab_toa_fast.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/ab_toa.py cur >> gpurun_out/ab_toa_fast.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/toa_leg_breakdown.py > gpurun_out/toa_breakdown.log 2>&1 || exit $?
CRIMP_TOA_NO_OVERLAP=1 timeout -k 10 300 python -u tools/toa_leg_breakdown.py >> gpurun_out/toa_breakdown.log 2>&1 || exit $?
STEPS=tests,bench PYTEST_X= BENCH_ARGS="--steps 20 --warmup 5" bash tools/gpu_round.sh || exit $?

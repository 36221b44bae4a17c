# Round-4 final evidence on the last tree: the ToA host trace, then the GPU suite, smoke, the driver-style bench, a
# rocprofv3 kernel-trace profile of the bench, and the N=2 rehearsal.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/toa_host_trace.py > gpurun_out/toa_host_trace3.log 2>&1 || exit $?
STEPS=tests,smoke,bench,prof PYTEST_X= BENCH_ARGS="--steps 20 --warmup 5" bash tools/gpu_round.sh || exit $?
bash tools/rehearse_n2.sh

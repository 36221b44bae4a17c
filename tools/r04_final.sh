# Round-4 final evidence: the GPU suite, smoke, the driver-style bench, a rocprofv3 kernel-trace profile of the bench,
# and the N=2 rehearsal of the bench's multi-GPU path.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STEPS=tests,smoke,bench,prof PYTEST_X= BENCH_ARGS="--steps 20 --warmup 5" bash tools/gpu_round.sh || exit $?
bash tools/rehearse_n2.sh

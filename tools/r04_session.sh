# Round-4 GPU session: ToA brute-grid A/B (full kernel vs fast form), parity tests, smoke, the driver-style bench,
# and the N=2 rehearsal of the bench's multi-GPU path. Each GPU step has its own time limit; stops on a fault.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
CRIMP_TOA_GRID_SLOW=1 timeout -k 10 300 python -u tools/ab_toa.py cur > gpurun_out/ab_toa_fast.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/ab_toa.py cur >> gpurun_out/ab_toa_fast.log 2>&1 || exit $?
CRIMP_TOA_GRID_SLOW=1 timeout -k 10 300 python -u tools/ab_toa.py cur >> gpurun_out/ab_toa_fast.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/ab_toa.py cur >> gpurun_out/ab_toa_fast.log 2>&1 || exit $?
STEPS=${STEPS:-tests,smoke,bench} PYTEST_X= BENCH_ARGS="--steps 20 --warmup 5" bash tools/gpu_round.sh || exit $?
bash tools/rehearse_n2.sh

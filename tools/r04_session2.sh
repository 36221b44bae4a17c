# Round-4 session 2: early-open A/B of the exact search kernel (config 3 and a 2-D grid, digests of every power);
# the config-5 ToA fit with the full brute-grid kernel vs the fast one and with / without the two-stream overlap;
# the parity tests, the driver-style bench and the N=2 rehearsal. Each GPU step has its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/ab_search.py ship early ship early > gpurun_out/ab_early.log 2>&1 || exit $?
NPH=2000000 NTR=131072 NFD=4 REPS=2 timeout -k 10 300 python -u tools/ab_search.py ship early early >> gpurun_out/ab_early.log 2>&1 || exit $?
CRIMP_TOA_GRID_SLOW=1 timeout -k 10 300 python -u tools/ab_toa.py cur > gpurun_out/ab_toa_fast.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/ab_toa.py cur >> gpurun_out/ab_toa_fast.log 2>&1 || exit $?
CRIMP_TOA_NO_OVERLAP=1 timeout -k 10 300 python -u tools/run_toa.py > gpurun_out/toa_overlap.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/run_toa.py >> gpurun_out/toa_overlap.log 2>&1 || exit $?
STEPS=tests,bench PYTEST_X= BENCH_ARGS="--steps 20 --warmup 5" bash tools/gpu_round.sh || exit $?
bash tools/rehearse_n2.sh

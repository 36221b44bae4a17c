# Fence / AGPR-clobber / contraction A/B of the exact search kernel. Part 3: the 2-D grid, every
# trial's power dumped per build (gpurun_out/ab2d/*.npy) and the run repeated for determinism; then the 1-D
# config-3 timing of the sched_barrier fences (CRIMP_EX_OPEN=2) against the shipped ones
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab2d
DUMP=gpurun_out/ab2d NPH=2000000 NTR=131072 NFD=4 REPS=2 timeout -k 10 300 python -u tools/ab_search.py ship2 noopen2 sb > gpurun_out/ab_fences3.log 2>&1 &&
NPH=2000000 NTR=131072 NFD=4 timeout -k 10 300 python -u tools/ab_search.py noopen2 >> gpurun_out/ab_fences3.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_search.py ship2 sb ship2 sb >> gpurun_out/ab_fences3.log 2>&1

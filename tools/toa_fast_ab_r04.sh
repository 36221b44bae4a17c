# Config-5 ToA fit: the full brute-grid kernel (CRIMP_TOA_GRID_SLOW) against the fast form, same build
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
CRIMP_TOA_GRID_SLOW=1 timeout -k 10 300 python -u tools/ab_toa.py cur > gpurun_out/ab_toa_fast.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_toa.py cur >> gpurun_out/ab_toa_fast.log 2>&1 &&
CRIMP_TOA_GRID_SLOW=1 timeout -k 10 300 python -u tools/ab_toa.py cur >> gpurun_out/ab_toa_fast.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_toa.py cur >> gpurun_out/ab_toa_fast.log 2>&1

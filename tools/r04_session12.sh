# Round-4 session 12: the fit kernel with 1024-thread workgroups (one per CU: 1250 intervals in 4.9 rounds of 256
# instead of 2.4 rounds of 512 two-per-CU slots) against the shipped 512, with digests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/ab_toa.py cur fb1024 cur fb1024 > gpurun_out/ab_toa_fb1024.log 2>&1 || exit $?

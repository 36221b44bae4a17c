# Round-4 session 7: the brute grid with norm-initialised MFMA accumulators (CRIMP_GM_CIN; cin0 = the previous kernel)
# A/B with digests, then the GPU suite (the brute-argmax tests hold the changed roundings) and the ToA leg breakdown.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ab_toa.py cin0 cur cin0 cur > gpurun_out/ab_toa_cin.log 2>&1 || exit $?
STEPS=tests PYTEST_X= bash tools/gpu_round.sh || exit $?
timeout -k 10 300 python -u tools/toa_leg_breakdown.py > gpurun_out/toa_breakdown.log 2>&1 || exit $?

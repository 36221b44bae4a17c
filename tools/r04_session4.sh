# Round-4 session 4: redChi2 as k_binphases (reciprocal estimate + np.histogram corrections, packed 8-bit counters)
# + k_toa_chi2, the two-stream overlap opt-in: the GPU suite, the ToA leg breakdown, the host->device upload A/B,
# the brute grid's MFMAs writing VGPRs (-mllvm -amdgpu-mfma-vgpr-form=1: no v_accvgpr_read per chunk) A/B,
# then the round's PMC passes (search traffic and SQ, ToA SQ / instruction classes / LDS / clock / traffic).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ab_toa.py cur vf cur vf > gpurun_out/ab_toa_vf.log 2>&1 || exit $?
STEPS=tests PYTEST_X= bash tools/gpu_round.sh || exit $?
grep -q " passed" gpurun_out/pytest_gpu.log && ! grep -q " failed" gpurun_out/pytest_gpu.log || exit 1
timeout -k 10 300 python -u tools/toa_leg_breakdown.py > gpurun_out/toa_breakdown.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/run_toa.py > gpurun_out/run_toa.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/upload_ab.py > gpurun_out/upload_ab.log 2>&1 || exit $?
bash tools/pmc_round.sh > gpurun_out/pmc_round.log 2>&1 || exit $?

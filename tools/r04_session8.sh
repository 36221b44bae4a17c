# Round-4 session 8: the brute grid's lazy-norm certificate (no per-phShift min h; CRIMP_TOA_NO_CERT = the min path)
# A/B with digests, the GPU suite, the ToA leg breakdown and the driver-style bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
CRIMP_TOA_NO_CERT=1 timeout -k 10 300 python -u tools/ab_toa.py cur > gpurun_out/ab_toa_cert.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/ab_toa.py cur >> gpurun_out/ab_toa_cert.log 2>&1 || exit $?
CRIMP_TOA_NO_CERT=1 timeout -k 10 300 python -u tools/ab_toa.py cur >> gpurun_out/ab_toa_cert.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/ab_toa.py cur >> gpurun_out/ab_toa_cert.log 2>&1 || exit $?
STEPS=tests PYTEST_X= bash tools/gpu_round.sh || exit $?
grep -q " passed" gpurun_out/pytest_gpu.log && ! grep -q " failed" gpurun_out/pytest_gpu.log || exit 1
timeout -k 10 300 python -u tools/toa_leg_breakdown.py > gpurun_out/toa_breakdown.log 2>&1 || exit $?
STEPS=smoke,bench BENCH_ARGS="--steps 20 --warmup 5" bash tools/gpu_round.sh || exit $?

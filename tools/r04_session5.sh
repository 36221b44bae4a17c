# Round-4 session 5: brute-grid A/B -- novf (MFMAs into AGPRs), t128np (round-3 tile: 128 photons, two threads per photon, no row pad; MFMAs into
# VGPRs), t128p (+ row pad), t256np (256-photon tile, one thread per photon, no pad), cur (256 + pad + v_perm
# packing) -- with digests; the ToA and binphases GPU tests; the e2e breakdown; the GPU suite and the bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/ab_toa.py novf t128np t128p t256np cur novf t128np t128p t256np cur > gpurun_out/ab_toa_tile.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_certificate.py \
  tests/test_gpu_parity.py -k "brute or binphases or measure_intervals or config5 or toa" > gpurun_out/grid_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/e2e_breakdown.py > gpurun_out/e2e_breakdown.log 2>&1 || exit $?
STEPS=tests,smoke,bench PYTEST_X= BENCH_ARGS="--steps 20 --warmup 5" bash tools/gpu_round.sh || exit $?

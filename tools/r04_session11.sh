# Round-4 session 11: brute-grid latency hiding A/B -- base (the certified grid as measured), nopipe (next tile's photons
# prefetched), cur (prefetch + next chunk's MFMAs issued before the current chunk's VALU work) -- with digests, then
# the ToA GPU tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/ab_toa.py base nopipe cur base nopipe cur > gpurun_out/ab_toa_pipe.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_certificate.py \
  tests/test_gpu_parity.py -k "brute or toa or config5 or certificate" > gpurun_out/grid_tests.log 2>&1 || exit $?

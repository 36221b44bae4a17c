# Round-4 session 18: the lazy-norm certificate with an amplitude-scaled margin -- its tests (bright and faint
# shapes) and the ToA GPU tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 180 --timeout-method thread -m gpu tests/test_gpu_certificate.py \
  tests/test_gpu_parity.py tests/test_gpu_scan_edges.py -k "certificate or brute or toa or scan" > gpurun_out/cert_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/ab_toa.py cur > gpurun_out/ab_toa_margin.log 2>&1 || exit $?

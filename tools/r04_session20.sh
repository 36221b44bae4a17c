# Round-4 session 20: the ToA call's uploads through page-locked staging (one drain for the host's copies): its
# host-phase trace, the ToA GPU tests, and the ToA A/B digest.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/toa_host_trace.py > gpurun_out/toa_host_trace2.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest -x -v --timeout 180 --timeout-method thread -m gpu tests/test_gpu_certificate.py \
  tests/test_gpu_parity.py tests/test_gpu_scan_edges.py -k "certificate or brute or toa or scan or measure" > gpurun_out/toa_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/ab_toa.py cur > gpurun_out/ab_toa_pin.log 2>&1 || exit $?

# Round-4 session 14 (+ the e2e timeline of session 13): the exact search kernel folding every 15 carry periods instead of 8 (f15 = the default now;
# f8 = the previous build): config-3 time and digests of every power, a 2-D digest check, the search GPU tests (the
# fold path included), and the rocprofv3 FETCH_SIZE / WRITE_SIZE passes of one config-3 search.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/ab_search.py f8 f15 f8 f15 > gpurun_out/ab_fold.log 2>&1 || exit $?
NPH=2000000 NTR=131072 NFD=4 REPS=2 timeout -k 10 300 python -u tools/ab_search.py f8 f15 >> gpurun_out/ab_fold.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -x -v --timeout 180 --timeout-method thread -m gpu tests/test_gpu_fullsize.py \
  tests/test_gpu_certificate.py tests/test_gpu_parity.py -k "search or fold or trial or config4 or exact" > gpurun_out/search_tests.log 2>&1 || exit $?
bash tools/pmc_traffic_quick.sh > gpurun_out/pmc_traffic.log 2>&1 || exit $?
python3 tools/pmc_traffic_json.py gpurun_out > gpurun_out/pmc_traffic.json || exit $?
cat gpurun_out/pmc_traffic.json
BLOCKS=1,4,d timeout -k 10 400 python -u tools/e2e_breakdown.py > gpurun_out/e2e_trace.log 2>&1 || exit $?

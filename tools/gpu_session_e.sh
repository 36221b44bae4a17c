mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u tools/diag_nufft_harm.py 7429 20 duplicated > gpurun_out/diag_harm.log 2>&1; rc=$?
cat gpurun_out/diag_harm.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -q -k "config5" -s --timeout 900 --timeout-method thread > gpurun_out/pytest_c5.log 2>&1; rc=$?
tail -8 gpurun_out/pytest_c5.log; exit $rc

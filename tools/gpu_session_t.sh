mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_nufft.py tests/test_gpu_best.py tests/test_gpu_certificate.py tests/test_gpu_parity.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_t.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_t.log; [ $rc -ne 0 ] && exit $rc
VARIANTS=";CRIMP_NUFFT_AP_SERIAL=1" REPS=10 timeout -k 10 300 python -u tools/ab_nufft.py > gpurun_out/ab_t.log 2>&1 || exit $?
cat gpurun_out/ab_t.log

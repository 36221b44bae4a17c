mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_best.py tests/test_gpu_dropin.py tests/test_gpu_nufft.py tests/test_distributed_gpu.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/pytest_c.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_c.log; echo "pytest rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
VARIANTS="CRIMP_NUFFT_PCHUNK=0;CRIMP_NUFFT_PCHUNK=2;CRIMP_NUFFT_PCHUNK=4;CRIMP_NUFFT_PCHUNK=8" REPS=8 timeout -k 10 200 python -u tools/ab_nufft.py > gpurun_out/ab_pchunk.log 2>&1 || exit $?
cat gpurun_out/ab_pchunk.log
timeout -k 10 200 python -u tools/step_probe.py > gpurun_out/step_probe.log 2>&1 || exit $?
cat gpurun_out/step_probe.log
timeout -k 10 300 python -u tools/diag_cert.py 20 1 default duplicated > gpurun_out/diag_nufft.log 2>&1 || exit $?
cat gpurun_out/diag_nufft.log

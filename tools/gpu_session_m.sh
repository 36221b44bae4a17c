mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_nufft.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_m.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_m.log; [ $rc -ne 0 ] && exit $rc
REPS=2 timeout -k 10 400 python -u tools/run_config4_nufft.py > gpurun_out/c4_m.log 2>&1 || exit $?
cat gpurun_out/c4_m.log

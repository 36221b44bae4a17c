mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_nufft.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_p.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_p.log; [ $rc -ne 0 ] && exit $rc
VARIANTS=";CRIMP_NUFFT_CS_MODE=2" REPS=10 timeout -k 10 200 python -u tools/ab_nufft.py > gpurun_out/ab_p.log 2>&1 || exit $?
cat gpurun_out/ab_p.log
timeout -k 10 300 python -u tools/shard_proxy.py > gpurun_out/shard_proxy.log 2>&1 || exit $?
cat gpurun_out/shard_proxy.log

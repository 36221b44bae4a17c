mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_nufft.py tests/test_gpu_best.py tests/test_distributed_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_u.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_u.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for v in 0 1; do
    if [ $v = 1 ]; then export CRIMP_NUFFT_AP_SERIAL=1; else unset CRIMP_NUFFT_AP_SERIAL; fi
    timeout -k 10 200 python -u bench.py --steps 50 --warmup 5 --no-cpu --no-toa --no-config2 --no-calcphase --no-config4 --no-exact > gpurun_out/bench_u_${v}_${i}.log 2>&1 || exit $?
    python -c "import json,sys; d=[json.loads(l) for l in open('gpurun_out/bench_u_${v}_${i}.log') if l.startswith('{')][-1]; print('serial=$v run $i', d['ms_per_step'], d['nufft']['fp64_fixup_trials'])"
  done
done

mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_nufft.py tests/test_gpu_best.py tests/test_distributed_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_i.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_i.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/step_probe.py > gpurun_out/step_probe_i.log 2>&1 || exit $?
cat gpurun_out/step_probe_i.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu --no-toa --no-config2 --no-calcphase --no-config4 --no-exact > gpurun_out/bench_i.log 2>&1 || exit $?
python -c "import json; d=json.loads(open('gpurun_out/bench_i.log').read().splitlines()[-1]); print(d['value'], d['ms_per_step'])"

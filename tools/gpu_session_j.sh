mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_nufft.py tests/test_gpu_best.py tests/test_gpu_parity.py tests/test_distributed_gpu.py tests/test_gpu_dropin.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_j.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_j.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/step_probe.py > gpurun_out/step_probe_j.log 2>&1 || exit $?
cat gpurun_out/step_probe_j.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu --no-toa --no-config2 --no-calcphase --no-config4 --no-exact > gpurun_out/bench_j.log 2>&1 || exit $?
python -c "import json; d=json.loads(open('gpurun_out/bench_j.log').read().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['step_ms'])"

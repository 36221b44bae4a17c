mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_certificate.py -m gpu -q -k correlated --timeout 300 --timeout-method thread > gpurun_out/pytest_cert.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_cert.log; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu --no-toa --no-config2 --no-calcphase --no-config4 --exact-steps 1 > gpurun_out/bench_f.log 2>&1 || exit $?
tail -c 1500 gpurun_out/bench_f.log; echo
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_f -o run --output-format csv -- python -u bench.py --steps 20 --warmup 3 --no-cpu --no-toa --no-config2 --no-calcphase --no-config4 --no-exact > gpurun_out/prof_f.log 2>&1 || exit $?
find gpurun_out/prof_f -name "*kernel_stats.csv" | head -1 | xargs head -20

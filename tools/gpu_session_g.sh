mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_nufft.py tests/test_gpu_best.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_g.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_g.log; [ $rc -ne 0 ] && exit $rc
VARIANTS=";CRIMP_NUFFT_LANES=1;CRIMP_NUFFT_LANES=4" REPS=8 timeout -k 10 200 python -u tools/ab_nufft.py > gpurun_out/ab_g.log 2>&1 || exit $?
cat gpurun_out/ab_g.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_g -o run --output-format csv -- python -u bench.py --steps 20 --warmup 3 --no-cpu --no-toa --no-config2 --no-calcphase --no-config4 --no-exact > gpurun_out/prof_g.log 2>&1 || exit $?
tail -c 400 gpurun_out/prof_g.log
find gpurun_out/prof_g -name "*kernel_stats.csv" | head -1 | xargs head -14 | cut -c1-60,200-

mkdir -p gpurun_out && export TMPDIR=/tmp
VARIANTS=";CRIMP_NUFFT_FINAL=separate" REPS=10 timeout -k 10 200 python -u tools/ab_nufft.py > gpurun_out/ab_l.log 2>&1 || exit $?
cat gpurun_out/ab_l.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu --no-toa --no-config2 --no-calcphase --no-config4 --no-exact > gpurun_out/bench_l.log 2>&1 || exit $?
python -c "import json; d=json.loads(open('gpurun_out/bench_l.log').read().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['ms_per_launch'], d['roofline']['frac'])"

mkdir -p gpurun_out && export TMPDIR=/tmp
for st in 0 0.3 1.0; do
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --settle $st --no-cpu --no-toa --no-config2 --no-calcphase --no-config4 --no-exact > gpurun_out/bench_k_$st.log 2>&1 || exit $?
python -c "import json; d=json.loads(open('gpurun_out/bench_k_$st.log').read().splitlines()[-1]); print('settle $st', d['value'], d['ms_per_step'], d['roofline']['step_ms'])" | tee -a gpurun_out/clock_settle.log
done
timeout -k 10 300 python -u bench.py --steps 200 --warmup 3 --settle 0 --no-cpu --no-toa --no-config2 --no-calcphase --no-config4 --no-exact > gpurun_out/bench_k_200.log 2>&1 || exit $?
python -c "import json; d=json.loads(open('gpurun_out/bench_k_200.log').read().splitlines()[-1]); print('settle 0, 200 steps', d['value'], d['ms_per_step'])" | tee -a gpurun_out/clock_settle.log

# Round-6 final evidence, part B: the default bench, rocprofv3 kernel stats of the bench's search, the NUFFT PMC
# traffic passes, the cell-start probe
mkdir -p gpurun_out && export TMPDIR=/tmp
OUT=gpurun_out/full_v4
mkdir -p $OUT
timeout -k 10 400 python -u bench.py > $OUT/bench.log 2>&1 || exit $?
tail -c 300 $OUT/bench.log; echo
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python -u bench.py --steps 20 --warmup 3 --no-cpu --no-toa --no-config2 --no-calcphase --no-config4 --no-exact > $OUT/prof.log 2>&1 || exit $?
TAG=nufft_r06d bash tools/pmc_nufft.sh > gpurun_out/pmc_nufft_r06d.log 2>&1 || exit $?
python tools/pmc_nufft_json.py gpurun_out/pmc_nufft_r06d > gpurun_out/pmc_nufft_traffic_r06d.json && cat gpurun_out/pmc_nufft_traffic_r06d.json
true


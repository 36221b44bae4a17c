# Round-6 evidence: the whole -m gpu suite, smoke, the default bench, rocprofv3 kernel stats of the bench's search.
mkdir -p gpurun_out && export TMPDIR=/tmp
OUT=gpurun_out/full
mkdir -p $OUT
timeout -k 10 1100 python -u -m pytest tests -m gpu -v -rs --durations=25 --timeout 900 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -5 $OUT/pytest_gpu.log; echo "pytest rc=$rc"; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log
timeout -k 10 600 python -u bench.py > $OUT/bench.log 2>&1 || exit $?
tail -c 300 $OUT/bench.log; echo
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python -u bench.py --steps 20 --warmup 3 --no-cpu --no-toa --no-config2 --no-calcphase --no-config4 --no-exact > $OUT/prof.log 2>&1 || exit $?
echo done

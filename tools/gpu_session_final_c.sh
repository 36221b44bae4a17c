# Round-6 closing evidence on the final tree: the whole -m gpu suite, smoke, the default bench, and the per-layer host
# cost of a search step (after the stream / device-guard trims in _native.Buffers)
mkdir -p gpurun_out && export TMPDIR=/tmp
OUT=gpurun_out/full_v5
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -rs --durations=25 --timeout 900 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -3 $OUT/pytest_gpu.log; echo "pytest rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log
timeout -k 10 400 python -u bench.py > $OUT/bench.log 2>&1 || exit $?
tail -c 300 $OUT/bench.log; echo
timeout -k 10 120 python -u tools/py_overhead.py 20000 > $OUT/py_overhead.log 2>&1 || exit $?
timeout -k 10 240 python -u tools/step_overhead.py 300 > $OUT/step_overhead.log 2>&1 || exit $?
cat $OUT/py_overhead.log $OUT/step_overhead.log | grep -v amdgpu.ids
true

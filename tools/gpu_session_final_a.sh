# Round-6 final evidence, part A: the whole -m gpu suite and smoke
mkdir -p gpurun_out && export TMPDIR=/tmp
OUT=gpurun_out/full_v4
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -rs --durations=25 --timeout 900 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -3 $OUT/pytest_gpu.log; echo "pytest rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log

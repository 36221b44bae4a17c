#!/bin/bash
# One GPU session: parity tests, smoke, a short bench, and a rocprofv3 kernel-trace profile.
# Every GPU step has its own time limit; a fault/abort/timeout ends the script (no retries).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
stop_on_fault() {  # rc 0 ok, 1 = test failures (not a fault); anything else: stop here
    local rc=$1 name=$2
    echo "[$name] rc=$rc" | tee -a "$OUT/steps.log"
    if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit "$rc"; fi
}
STEPS=${STEPS:-tests,smoke,bench,prof}
if [[ $STEPS == *c4w* ]]; then  # config-4 parity windows against the committed oracle values
  timeout -k 10 300 python -u tools/config4_windows.py > "$OUT/c4w.json" 2> "$OUT/c4w.err"
  stop_on_fault $? c4w
  head -c 600 "$OUT/c4w.json"; echo
fi
if [[ $STEPS == *tests* ]]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu ${PYTEST_X--x} -v -rs --durations=15 --timeout 180 --timeout-method thread ${PYTEST_ARGS:-} ${PYTEST_K:+-k "$PYTEST_K"} > "$OUT/pytest_gpu.log" 2>&1
  stop_on_fault $? pytest
  tail -5 "$OUT/pytest_gpu.log"
fi
if [[ $STEPS == *smoke* ]]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
  stop_on_fault $? smoke
  tail -2 "$OUT/smoke.log"
fi
if [[ $STEPS == *bench* ]]; then
  timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > "$OUT/bench.log" 2>&1
  stop_on_fault $? bench
  tail -1 "$OUT/bench.log"
fi
if [[ $STEPS == *prof* ]]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
      python bench.py ${PROF_ARGS:---steps 20 --warmup 3 --no-cpu --no-toa --no-config2 --no-calcphase --no-config4 --exact-steps 1} > "$OUT/prof.log" 2>&1
  stop_on_fault $? rocprof
  find "$OUT/prof" -name "*stats*" | head
fi
if [[ $STEPS == *nufft* ]]; then  # config-3 NUFFT search: timing, then a rocprofv3 kernel-trace profile
  CRIMP_PRECISION=nufft REPS=${NUFFT_REPS:-5} timeout -k 10 300 python -u tools/run_search.py > "$OUT/nufft_run.log" 2>&1
  stop_on_fault $? nufft_run
  cat "$OUT/nufft_run.log"
  CRIMP_PRECISION=nufft REPS=${NUFFT_REPS:-5} timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_nufft" \
      -o run --output-format csv -- python -u tools/run_search.py > "$OUT/prof_nufft.log" 2>&1
  stop_on_fault $? prof_nufft
  find "$OUT/prof_nufft" -name "*stats*" | head
fi
if [[ $STEPS == *h20* ]]; then  # H-test (m = 20) timing
  NHARM=20 NPH=2000000 NTR=1000000 timeout -k 10 200 python3 tools/run_search.py >> "$OUT/h20.log" 2>&1
  stop_on_fault $? h20
  cat "$OUT/h20.log"
fi

cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c --kernel-trace -d gpurun_out/tr_$c -o pmc --output-format csv -- python3 tools/run_search.py > gpurun_out/tr_$c.log 2>&1 || exit 1
  python3 tools/pmc_summary.py gpurun_out/tr_$c k_search_exact | head -2
done

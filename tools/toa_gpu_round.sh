cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 rocprofv3 -L > gpurun_out/rocprof_list.txt 2>&1; echo "[list] rc=$?"
timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu --no-config4 --no-config2 --no-calcphase --trials 100000 > gpurun_out/bench_toa.log 2>&1 || exit $?
tail -c 2500 gpurun_out/bench_toa.log
RUN=tools/run_toa.py TAG=toa PAT="k_toa_fit k_toa_grid" PMC_SETS="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY
GRBM_GUI_ACTIVE GRBM_COUNT" bash tools/pmc_exact.sh

# Round-4 session 10: SQ counters of the final brute grid and fit (config 5 over tools/run_toa.py): instruction mix,
# waits, matrix-pipe busy, LDS, clock -- each pass its own rocprofv3 run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
RUN=tools/run_toa.py TAG=toa_final PAT="k_toa_grid_mf k_toa_fit k_toa_grid_best" PMC_SETS="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY
SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE
GRBM_GUI_ACTIVE GRBM_COUNT" bash tools/pmc_exact.sh > gpurun_out/pmc_toa_final.log 2>&1 || exit $?
echo done

#!/bin/bash
# Round-end PMC evidence (each pass its own rocprofv3 run under its own time limit; stops at the first failure):
# search traffic (FETCH_SIZE / WRITE_SIZE over tools/run_search.py -> pmc_traffic.json), search SQ counters
# (clock, matrix-pipe busy, waits), ToA kernels' SQ mix (VALU, MFMA, busy, waits), fp64 / fp32 instruction classes,
# clock and HBM traffic (config 5 over tools/run_toa.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
set -o pipefail
bash tools/pmc_traffic_quick.sh > gpurun_out/pmc_traffic.log 2>&1 || exit $?
python3 tools/pmc_traffic_json.py gpurun_out > gpurun_out/pmc_traffic.json || exit $?
TAG=search PAT=k_search_exact bash tools/pmc_exact.sh > gpurun_out/pmc_search.log 2>&1 || exit $?
RUN=tools/run_toa.py TAG=toa PAT="k_toa_fit k_toa_grid_mf k_toa_grid_best k_binphases k_toa_chi2" PMC_SETS="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY
SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE
SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32
GRBM_GUI_ACTIVE GRBM_COUNT
FETCH_SIZE
WRITE_SIZE" bash tools/pmc_exact.sh > gpurun_out/pmc_toa.log 2>&1 || exit $?
echo done

#!/bin/bash
# PMC evidence for the NUFFT search (config 3 over tools/run_search.py with CRIMP_PRECISION=nufft): kernel-trace stats,
# SQ issue/wait/LDS counters, fp64 instruction classes, clock, HBM traffic -- one rocprofv3 pass per set.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export CRIMP_PRECISION=nufft REPS=${REPS:-3}
RUN=tools/run_search.py TAG=${TAG:-nufft} PAT="k_nu_cols256 k_nu_rows_iw k_nu_gather k_nu_cellstart" PMC_SETS="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU
SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR
SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 GRBM_GUI_ACTIVE GRBM_COUNT
FETCH_SIZE
WRITE_SIZE" bash tools/pmc_exact.sh

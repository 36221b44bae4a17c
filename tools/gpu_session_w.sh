mkdir -p gpurun_out && export TMPDIR=/tmp
export ROWS=8 REPS=0 TIMED=0
TAG=c4spread_v2 RUN=tools/run_config4_nufft.py PAT="k_nu_spread k_nu_merge" PMC_SETS="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES
SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD
GRBM_GUI_ACTIVE GRBM_COUNT" bash tools/pmc_exact.sh > gpurun_out/pmc_c4spread_v2.log 2>&1; rc=$?
tail -60 gpurun_out/pmc_c4spread_v2.log; exit $rc

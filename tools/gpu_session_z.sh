# ToA kernels' PMC mix on the round's final code (config 5 over tools/run_toa.py)
mkdir -p gpurun_out && export TMPDIR=/tmp
RUN=tools/run_toa.py TAG=toa_r06 PAT="k_toa_fit k_toa_grid_mf k_toa_grid_best" PMC_SETS="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY
SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE
SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 GRBM_GUI_ACTIVE GRBM_COUNT" bash tools/pmc_exact.sh > gpurun_out/pmc_toa_r06.log 2>&1; rc=$?
grep -E "^\[|^==" gpurun_out/pmc_toa_r06.log; exit $rc

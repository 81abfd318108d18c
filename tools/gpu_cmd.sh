R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
run() { timeout -s KILL 90 rocprofv3 --pmc $2 -d $R/gpurun_out/$1 -o s --output-format csv -- python3 $R/tools/pmc_run.py > $R/gpurun_out/$1.log 2>&1; }
run sqa "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES" &&
run sqb "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_ACTIVE_INST_MISC" &&
run sqc "SQ_INSTS_VMEM SQ_ACTIVE_INST_VMEM SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT"
rc=$?
cd $R
for p in sqa sqb sqc; do python tools/pmc_summary.py gpurun_out/$p/s_counter_collection.csv solve16 ts_fused universe_kernel; done > gpurun_out/sq_summary.txt 2>&1
exit $rc

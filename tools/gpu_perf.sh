# Kernel timings (tools/kbench.py, unfused and fused month pass) + SQ counters of the panel
# kernels; each step under its own limit, chained so that a crash ends the call.
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/kb.log
timeout -k 10 240 python tools/kbench.py >> gpurun_out/kb.log 2>&1 &&
KB_FUSED=1 timeout -k 10 240 python tools/kbench.py >> gpurun_out/kb.log 2>&1 || { cat gpurun_out/kb.log; exit 1; }
cat gpurun_out/kb.log
[ "$1" = "sq" ] || exit 0
cd /tmp && export TMPDIR=/tmp
run() { timeout -s KILL 90 rocprofv3 --pmc $2 -d $R/gpurun_out/$1 -o s --output-format csv -- python3 $R/tools/pmc_run.py > $R/gpurun_out/$1.log 2>&1; }
run sqa "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES" &&
run sqb "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_ACTIVE_INST_MISC" &&
run sqc "SQ_INSTS_VMEM SQ_ACTIVE_INST_VMEM SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT"
rc=$?
cd $R
for p in sqa sqb sqc; do python tools/pmc_summary.py gpurun_out/$p/s_counter_collection.csv gram_kernel select_pair_kernel month_kernel; done > gpurun_out/sq_summary.txt 2>&1
cat gpurun_out/sq_summary.txt
exit $rc

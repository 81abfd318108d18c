# SQ counters of the bench panel's universe, Gram and select kernels (tools/pmc_run.py); 2 passes
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
run() { timeout -s KILL 90 rocprofv3 --pmc $2 -d $R/gpurun_out/$1 -o s --output-format csv -- python3 $R/tools/pmc_run.py > $R/gpurun_out/$1.log 2>&1; }
run bsqa "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" &&
run bsqb "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES"
rc=$?
cd $R
for p in bsqa bsqb; do python tools/pmc_summary.py gpurun_out/$p/s_counter_collection.csv universe_kernel gram_kernel select_pair solve16 ts_fused; done
exit $rc

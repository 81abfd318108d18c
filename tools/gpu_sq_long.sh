# SQ counters of the long-month select (tools/selbench.py's 1,000 x 20,000 panel); 2 passes
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && export SB_CHILD=1 SB_T=300
run() { timeout -s KILL 90 rocprofv3 --pmc $2 -d $R/gpurun_out/$1 -o s --output-format csv -- python3 $R/tools/selbench.py > $R/gpurun_out/$1.log 2>&1; }
run lsqa "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" &&
run lsqb "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM"
rc=$?
cd $R
for p in lsqa lsqb; do python tools/pmc_summary.py gpurun_out/$p/s_counter_collection.csv select_long; done
exit $rc

# SQ counter passes over tools/selbench.py (one child, the library named by each argument):
#   bash tools/sq_select.sh <tag>=<lib.so> ...   (through gpurun; summaries in gpurun_out/sq_<tag>_{a,b}.summary)
R=${GRAFT_REPO_ROOT:-$(pwd)}
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU"
B="SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_INSTS_BRANCH"
for spec in "$@"; do
  tag=${spec%%=*}; lib=${spec#*=}
  for p in a b; do
    [ $p = a ] && C=$A || C=$B
    (cd /tmp && export TMPDIR=/tmp && SB_CHILD=1 FM_HIP_LIB=$R/$lib timeout -s KILL 90 rocprofv3 --pmc $C -d $R/gpurun_out/sq_${tag}_$p -o s --output-format csv -- python3 $R/tools/selbench.py > $R/gpurun_out/sq_${tag}_$p.log 2>&1) || exit 1
    python $R/tools/pmc_summary.py $R/gpurun_out/sq_${tag}_$p/s_counter_collection.csv select_long_hk > $R/gpurun_out/sq_${tag}_$p.summary 2>&1
  done
done

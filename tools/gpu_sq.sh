R=$GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "sq1:::300:::cd /tmp && export TMPDIR=/tmp && rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -d $R/gpurun_out/sq1 -o s --output-format csv -- python3 $R/tools/pmc_run.py" \
 "sq2:::300:::cd /tmp && export TMPDIR=/tmp && rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SALU -d $R/gpurun_out/sq2 -o s --output-format csv -- python3 $R/tools/pmc_run.py"

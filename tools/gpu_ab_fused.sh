# A/B: fm_select + fm_gram vs the fused fm_month_pass on the bench panel (kbench medians).
mkdir -p gpurun_out
timeout -k 10 300 python tools/kbench.py > gpurun_out/kb_split.log 2>&1 && \
KB_FUSED=1 timeout -k 10 300 python tools/kbench.py > gpurun_out/kb_fused.log 2>&1
rc=$?; cat gpurun_out/kb_split.log gpurun_out/kb_fused.log; exit $rc

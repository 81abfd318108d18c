mkdir -p gpurun_out
timeout -k 10 120 tools/probes/mfma_f64_rate > gpurun_out/mfma_rate.log 2>&1; cat gpurun_out/mfma_rate.log
timeout -k 10 300 python tools/overlap_probe.py > gpurun_out/overlap.log 2>&1; rc=$?; cat gpurun_out/overlap.log; exit $rc

set -e
mkdir -p gpurun_out
timeout -k 10 60 tools/probes/mfma_f64_rate > gpurun_out/mfma.log 2>&1
for d in 0 1 2; do FM_GRAM_DEBUG=$d timeout -k 10 120 python tools/gram_sweep.py 1280 5120 640 > gpurun_out/sweep_dbg$d.log 2>&1; done
cat gpurun_out/mfma.log gpurun_out/sweep_dbg*.log

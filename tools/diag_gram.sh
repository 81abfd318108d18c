# gram diagnostics: parity first, then timing of the debug variants
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/parity.log 2>&1 || { tail -30 gpurun_out/parity.log; exit 1; }
tail -2 gpurun_out/parity.log
for d in 0 1 2; do FM_GRAM_DEBUG=$d timeout -k 10 120 python tools/gram_sweep.py ${SWEEP:-1280 2560 640} > gpurun_out/sweep_dbg$d.log 2>&1 || exit 1; done
cat gpurun_out/sweep_dbg*.log | grep -v amdgpu.ids

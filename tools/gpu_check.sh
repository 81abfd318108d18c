# GPU check: parity tests, Gram chunk sweep, bench (no CPU leg).  Each step under its own limit.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/parity.log 2>&1 || { tail -40 gpurun_out/parity.log; exit 1; }
tail -2 gpurun_out/parity.log
if [ -n "$SWEEP" ]; then
  timeout -k 10 120 python tools/gram_sweep.py $SWEEP > gpurun_out/sweep.log 2>&1 || { cat gpurun_out/sweep.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/sweep.log
fi
timeout -k 10 180 python bench.py --no-cpu --steps 20 > gpurun_out/bench.log 2>&1 || { cat gpurun_out/bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/bench.log

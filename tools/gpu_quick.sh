# Quick GPU iteration: parity tests (or a -k subset via $K) then the bench (no CPU leg).
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread ${K:+-k "$K"} > gpurun_out/parity.log 2>&1
rc=$?; tail -3 gpurun_out/parity.log; grep -E "^FAILED|^E  " gpurun_out/parity.log | head -20
[ $rc -eq 0 ] || [ -n "$BENCH_ANYWAY" ] || exit $rc
timeout -k 10 180 python bench.py --no-cpu --no-chars --steps 20 > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/bench.log

# One GPU iteration: the full -m gpu suite (or a -k subset via $K), then kbench of the
# in-tree library against the given variant libraries.
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread \
  ${K:+-k "$K"} > gpurun_out/parity.log 2>&1
rc=$?; tail -3 gpurun_out/parity.log; grep -E "^FAILED|^E  " gpurun_out/parity.log | head -20
case $rc in 124|134|137|139|143) exit $rc;; esac
[ $rc -eq 0 ] || [ -n "$BENCH_ANYWAY" ] || exit $rc
timeout -k 10 300 python tools/kbench.py fm-returnprediction_amd/lib/libfm_hip.so "$@" > gpurun_out/kb.log 2>&1
rc=$?; cat gpurun_out/kb.log; exit $rc

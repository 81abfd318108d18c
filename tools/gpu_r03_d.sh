# Round-3 iteration d: long select v2 (high-word thresholds, histogram select of candidates)
T="python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread"
tools/gpu_steps.sh \
 "longsel:::300:::$T tests/test_gpu_parity.py -k 'long_month or long_segment or c5 or percentile or masked or universe'" \
 "selbench:::300:::python tools/selbench.py fm-returnprediction_amd/lib/libfm_hip.so build_variants/LA1/libfm_hip.so build_variants/LA2/libfm_hip.so" \
 "gputests:::600:::$T tests -m gpu" \
 "bench:::400:::python bench.py --steps 20"

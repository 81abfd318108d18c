# Round-3 iteration h: ballot compaction in the long-month select (variant LB): parity, timing,
# and SQ counters of the in-tree long select
V=build_variants
T="python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread"
tools/gpu_steps.sh \
 "LBtests:::300:::FM_HIP_LIB=$V/LB/libfm_hip.so $T tests/test_gpu_parity.py -k 'long_month or long_segment or c5 or percentile or masked or universe or level'" \
 "selbench:::300:::python tools/selbench.py fm-returnprediction_amd/lib/libfm_hip.so $V/LB/libfm_hip.so" \
 "sqlong:::300:::bash tools/gpu_sq_long.sh"

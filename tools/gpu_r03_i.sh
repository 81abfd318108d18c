# Round-3 (i): parity suite, long select A/B (sort skip, scalar-branch masking), solve
# moments-store A/B
tools/gpu_steps.sh \
 "gputests:::600:::python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread" \
 "selbench:::300:::python tools/selbench.py fm-returnprediction_amd/lib/libfm_hip.so build_variants/H/libfm_hip.so build_variants/MA/libfm_hip.so" \
 "kbsolve:::300:::python tools/kbench.py fm-returnprediction_amd/lib/libfm_hip.so build_variants/R/libfm_hip.so build_variants/N/libfm_hip.so"

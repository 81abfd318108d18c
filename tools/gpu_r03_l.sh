# Round-3 (l): DPP moves without zero-initialised destinations (Gram rotations, solve row
# broadcasts, xor_lanes), select_pair masking only past the full 128-row groups: parity + A/B
L=fm-returnprediction_amd/lib/libfm_hip.so
tools/gpu_steps.sh \
 "gputests:::600:::python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread" \
 "kbench:::400:::python tools/kbench.py $L build_variants/HEAD/libfm_hip.so build_variants/PM/libfm_hip.so $L build_variants/HEAD/libfm_hip.so" \
 "selbench:::300:::python tools/selbench.py $L build_variants/HEAD/libfm_hip.so $L build_variants/HEAD/libfm_hip.so"

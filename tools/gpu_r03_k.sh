# Round-3 (k): rolling std with shuffled previous ids and coalesced stores; Gram operand
# rotations without zero-initialised DPP moves: parity + A/B
L=fm-returnprediction_amd/lib/libfm_hip.so
tools/gpu_steps.sh \
 "gputests:::600:::python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread" \
 "stdbench:::300:::python tools/stdbench.py $L build_variants/IDL/libfm_hip.so build_variants/DIR/libfm_hip.so build_variants/OLD/libfm_hip.so $L build_variants/OLD/libfm_hip.so" \
 "kbgram:::300:::python tools/kbench.py $L build_variants/GOLD/libfm_hip.so build_variants/G1B/libfm_hip.so $L build_variants/GOLD/libfm_hip.so"

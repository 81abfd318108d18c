# Round-3 (m): Gram row mask only on a bucket's partial last group: parity + A/B
L=fm-returnprediction_amd/lib/libfm_hip.so
tools/gpu_steps.sh \
 "gputests:::600:::python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread" \
 "kbench:::400:::python tools/kbench.py $L build_variants/GMA/libfm_hip.so $L build_variants/GMA/libfm_hip.so"

# Round-3 (n): Gram MFMA operands two groups ahead inside a bucket: A/B
L=fm-returnprediction_amd/lib/libfm_hip.so
tools/gpu_steps.sh \
 "kbench:::400:::python tools/kbench.py $L build_variants/P2G/libfm_hip.so $L build_variants/P2G/libfm_hip.so"

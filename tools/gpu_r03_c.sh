# Round-3 iteration c: variant correctness + long-select / Gram / solve / rolling-std A/B timings
V=build_variants
T="python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread"
tools/gpu_steps.sh \
 "GO5tests:::300:::FM_HIP_LIB=$V/GO5/libfm_hip.so $T tests/test_gpu_parity.py -k 'pipeline or golden or edge or collinear or conditioning or inf_in_y or sharded or headline'" \
 "L1tests:::300:::FM_HIP_LIB=$V/L1/libfm_hip.so $T tests/test_gpu_parity.py -k 'long_month or long_segment or c5'" \
 "gs1tests:::400:::FM_HIP_LIB=$V/gs1/libfm_hip.so $T tests -m gpu" \
 "kbench:::400:::python tools/kbench.py fm-returnprediction_amd/lib/libfm_hip.so $V/gs1/libfm_hip.so $V/GO4/libfm_hip.so $V/GO5/libfm_hip.so" \
 "kbench2560:::400:::KB_CHUNK=2560 python tools/kbench.py fm-returnprediction_amd/lib/libfm_hip.so $V/gs1/libfm_hip.so $V/GO4/libfm_hip.so $V/GO5/libfm_hip.so" \
 "kbench1280:::300:::KB_CHUNK=1280 python tools/kbench.py $V/GO5/libfm_hip.so" \
 "selbench:::400:::python tools/selbench.py fm-returnprediction_amd/lib/libfm_hip.so $V/L1/libfm_hip.so $V/LA1/libfm_hip.so $V/LA1p/libfm_hip.so $V/LA2/libfm_hip.so" \
 "RS1tests:::200:::FM_HIP_LIB=$V/RS1/libfm_hip.so $T tests/test_gpu_parity.py -k 'std or chars'" \
 "RS1bench:::300:::FM_HIP_LIB=$V/RS1/libfm_hip.so python bench.py --no-cpu --no-c5 --steps 5"

# Round-3 (j): rolling-std ablations; Gram chunk sizes that fill 3 workgroups per CU evenly
L=fm-returnprediction_amd/lib/libfm_hip.so
tools/gpu_steps.sh \
 "stdbench:::300:::python tools/stdbench.py $L build_variants/STD1/libfm_hip.so build_variants/STD2/libfm_hip.so build_variants/STD3/libfm_hip.so build_variants/STD4/libfm_hip.so" \
 "kbchunk3907:::300:::KB_CHUNK=3907 python tools/kbench.py $L" \
 "kbchunk1954:::300:::KB_CHUNK=1954 python tools/kbench.py $L" \
 "kbchunk0:::300:::python tools/kbench.py $L"

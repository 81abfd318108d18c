# Round-3 iteration e: long select v3 (run merge) + MID variant for masked middle quantiles
T="python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread"
tools/gpu_steps.sh \
 "longsel:::300:::$T tests/test_gpu_parity.py -k 'long_month or long_segment or c5 or percentile or masked or universe'" \
 "selbench:::300:::python tools/selbench.py fm-returnprediction_amd/lib/libfm_hip.so build_variants/LA2/libfm_hip.so" \
 "gputests:::600:::$T tests -m gpu" \
 "bench:::400:::python bench.py --steps 20" \
 "kstats:::400:::cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/kt -o kt --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --no-chars --steps 10"

# Round-3 iteration b: long-month select test, new full-size tests, full suite, shard fixture,
# bench, rocprof kernel stats
R=$GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "longsel:::300:::python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k 'long_month or headline or gathered_c5'" \
 "gputests:::700:::python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread" \
 "fixture:::200:::python tools/dump_shard_pred.py gpurun_out/shard_pred.npz" \
 "bench:::400:::python bench.py --steps 20" \
 "kstats:::400:::cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats -d $R/gpurun_out/kt -o kt --output-format csv -- python3 $R/bench.py --no-cpu --no-chars --steps 10"

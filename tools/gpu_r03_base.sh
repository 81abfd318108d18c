# Round-3 baseline: parity suite, bench, rocprof kernel stats of the bench (no cpu / c5 legs)
R=$GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "gputests:::600:::python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread" \
 "bench:::400:::python bench.py --steps 20" \
 "kstats:::400:::cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats -d $R/gpurun_out/kt -o kt --output-format csv -- python3 $R/bench.py --no-cpu --no-chars --steps 10"

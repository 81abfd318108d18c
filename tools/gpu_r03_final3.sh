# Round-3 final (3): parity suite, smoke, bench, rocprof kernel stats, PMC traffic passes
R=$GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "gputests:::600:::python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread" \
 "smoke:::200:::python -c 'import __graft_entry__ as g; g.smoke()'" \
 "bench:::400:::python bench.py --steps 20" \
 "kstats:::400:::cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats -d $R/gpurun_out/kt -o kt --output-format csv -- python3 $R/bench.py --no-cpu --steps 10" \
 "pmcf:::300:::cd /tmp && export TMPDIR=/tmp && rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmcf -o f --output-format csv -- python3 $R/tools/pmc_run.py" \
 "pmcw:::300:::cd /tmp && export TMPDIR=/tmp && rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmcw -o w --output-format csv -- python3 $R/tools/pmc_run.py"

R=$GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "parity:::600:::python -m pytest tests/test_gpu_parity.py -q -m gpu -p no:cacheprovider --timeout 240" \
 "bench:::400:::python bench.py --no-cpu --steps 20" \
 "kstats:::400:::cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats -d $R/gpurun_out/kt -o kt --output-format csv -- python3 $R/bench.py --no-cpu --steps 10" \
 "pmcf:::400:::cd /tmp && export TMPDIR=/tmp && rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmcf -o f --output-format csv -- python3 $R/tools/pmc_run.py" \
 "pmcw:::400:::cd /tmp && export TMPDIR=/tmp && rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmcw -o w --output-format csv -- python3 $R/tools/pmc_run.py"

# Round-3 iteration f: long-series time-series kernels (chunked NW summary, sliding rolling,
# thread-per-row predictive, chunked compaction)
T="python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread"
tools/gpu_steps.sh \
 "tstests:::400:::$T tests/test_gpu_parity.py -k 'long_series or per_stage or unfitted or gathered or c5 or headline or newey'" \
 "gputests:::600:::$T tests -m gpu" \
 "bench:::400:::python bench.py --steps 20" \
 "kstats:::400:::cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/kt -o kt --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --no-chars --steps 10" \
 "mfma:::60:::tools/probes/mfma_f64_chains"

# End-of-round GPU evidence in one call (through gpurun): the GPU test suite, the PMC
# traffic passes (their summary copied over profiles/pmc_traffic.json on the box so the
# bench line carries `traffic`), the headline-only kernel statistics, then the full bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
bash tools/gpu.sh tests pmc || exit 1
[ -f gpurun_out/pmc_traffic.json ] && cp gpurun_out/pmc_traffic.json profiles/pmc_traffic.json
BENCH_ARGS="--no-c5 --no-standardize" bash tools/gpu.sh kstats || exit 1
bash tools/gpu.sh bench

# Round-3 final: A/B of the Gram at 4 waves/SIMD and the fused universe reductions, then the parity suite, smoke, bench,
# rocprof kernel stats, the two PMC passes (HBM traffic) and the FP64 MFMA probe
R=$GRAFT_REPO_ROOT
V=build_variants
tools/gpu_steps.sh \
 "kbGM4:::300:::python tools/kbench.py fm-returnprediction_amd/lib/libfm_hip.so $V/GM4/libfm_hip.so $V/UF/libfm_hip.so" \
 "kbGM4c2560:::300:::KB_CHUNK=2560 python tools/kbench.py fm-returnprediction_amd/lib/libfm_hip.so $V/GM4/libfm_hip.so" \
 "kbGM4c1664:::300:::KB_CHUNK=1664 python tools/kbench.py $V/GM4/libfm_hip.so" \
 "gputests:::600:::python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread" \
 "smoke:::200:::python -c 'import __graft_entry__ as g; g.smoke()'" \
 "bench:::400:::python bench.py --steps 20" \
 "kstats:::400:::cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats -d $R/gpurun_out/kt -o kt --output-format csv -- python3 $R/bench.py --no-cpu --no-c5 --steps 10" \
 "pmcf:::300:::cd /tmp && export TMPDIR=/tmp && rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmcf -o f --output-format csv -- python3 $R/tools/pmc_run.py" \
 "pmcw:::300:::cd /tmp && export TMPDIR=/tmp && rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmcw -o w --output-format csv -- python3 $R/tools/pmc_run.py" \
 "mfma:::60:::tools/probes/mfma_f64_chains"

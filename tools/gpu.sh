#!/bin/bash
# The one GPU launch script: tools/gpu.sh STEP [STEP ...], run through gpurun, e.g.
#   gpurun --timeout 1200 -- 'bash tools/gpu.sh tests smoke bench kstats'
# Each STEP is a preset below, run by tools/gpu_steps.sh under its own timeout (a crash or a
# timeout ends the sequence).  Environment knobs: K (pytest -k filter for `tests`/`parity`),
# BENCH_ARGS (extra bench.py flags), SQ_KERNELS (kernels summarised by `sq`).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
PT="python -u -m pytest -x -v -p no:cacheprovider --timeout 240 --timeout-method thread ${K:+-k \"$K\"}"
PROF="cd /tmp && export TMPDIR=/tmp && rocprofv3"
specs=()
for s in "$@"; do
  case $s in
    tests)   specs+=("tests:::900:::$PT -m gpu tests");;
    parity)  specs+=("parity:::600:::$PT -m gpu tests/test_gpu_parity.py");;
    dist)    specs+=("dist:::400:::$PT -m gpu tests/test_gpu_dist.py tests/test_gpu_rccl.py");;
    smoke)   specs+=("smoke:::200:::python -c 'import __graft_entry__ as g; g.smoke()'");;
    bench)   specs+=("bench:::500:::python bench.py $BENCH_ARGS");;
    quick)   specs+=("quick:::300:::python bench.py --no-cpu --no-chars --no-c5 --steps 20 $BENCH_ARGS");;
    scan)    specs+=("scan:::300:::python tools/size_scan.py");;
    split)   specs+=("split:::300:::python tools/split_scan.py");;
    rehearse) specs+=("rehearse:::400:::python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --dist-backend gloo --one-device --c5-months 400 --months 300");;
    spawn)   specs+=("spawn:::400:::python bench.py --gpus 2 --steps 5 --warmup 2 --dist-backend gloo --one-device --c5-months 400 --months 300 --no-headline");;
    tprobe)  specs+=("tprobe:::200:::FM_HIP_LIB=$R/build_variants/probe/libfm_hip.so python tools/tail_probe.py");;
    wgtime)  specs+=("wgtime:::200:::FM_HIP_LIB=$R/build_variants/wgtime/libfm_hip.so python tools/gram_wgtime.py");;
    kbench)  specs+=("kbench:::300:::python tools/kbench.py $KB_LIBS");;
    slab)    specs+=("slab:::300:::python tools/slab_probe.py");;
    cacheab) specs+=("cacheab:::300:::python tools/cache_ab.py");;
    selbench) specs+=("selbench:::300:::python tools/selbench.py $KB_LIBS");;
    stdbench) specs+=("stdbench:::300:::python tools/stdbench.py $KB_LIBS");;
    kstats)  specs+=("kstats:::500:::$PROF --kernel-trace --stats -d $R/gpurun_out/kt -o kt --output-format csv -- python3 $R/bench.py --no-cpu --no-chars --steps 10 $BENCH_ARGS");;
    pmc)     specs+=("pmcf:::300:::$PROF --pmc FETCH_SIZE -d $R/gpurun_out/pmcf -o f --output-format csv -- python3 $R/tools/pmc_run.py"
                     "pmcw:::300:::$PROF --pmc WRITE_SIZE -d $R/gpurun_out/pmcw -o w --output-format csv -- python3 $R/tools/pmc_run.py");;
    sq)      specs+=("sqa$SQ_TAG:::120:::$PROF --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU -d $R/gpurun_out/sqa$SQ_TAG -o s --output-format csv -- python3 $R/tools/pmc_run.py"
                     "sqb$SQ_TAG:::120:::$PROF --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES -d $R/gpurun_out/sqb$SQ_TAG -o s --output-format csv -- python3 $R/tools/pmc_run.py");;
    icache)  specs+=("icache$SQ_TAG:::120:::$PROF --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU -d $R/gpurun_out/icache$SQ_TAG -o s --output-format csv -- python3 $R/tools/pmc_run.py");;
    *) echo "unknown step $s"; exit 2;;
  esac
done
bash tools/gpu_steps.sh "${specs[@]}"
rc=$?
if [ -f gpurun_out/sqa$SQ_TAG/s_counter_collection.csv ]; then
  for p in sqa$SQ_TAG sqb$SQ_TAG; do
    python tools/pmc_summary.py gpurun_out/$p/s_counter_collection.csv ${SQ_KERNELS:-universe_kernel gram_kernel select_pair select_fixup solve16 ts_fused} > gpurun_out/$p.summary 2>&1
  done
fi
if [ -f gpurun_out/icache$SQ_TAG/s_counter_collection.csv ]; then
  python tools/pmc_summary.py gpurun_out/icache$SQ_TAG/s_counter_collection.csv ${SQ_KERNELS:-universe_kernel gram_kernel select_pair select_fixup solve16 ts_fused} > gpurun_out/icache$SQ_TAG.summary 2>&1
fi
if [ -f gpurun_out/pmcf/f_counter_collection.csv ] && [ -f gpurun_out/pmcw/w_counter_collection.csv ]; then
  sha=$(python -c "import hashlib;print(hashlib.sha256(open('fm-returnprediction_amd/lib/libfm_hip.so','rb').read()).hexdigest()[:16])")
  python tools/pmc_traffic.py gpurun_out/pmcf/f_counter_collection.csv gpurun_out/pmcw/w_counter_collection.csv gpurun_out/pmc_traffic.json "$sha" > gpurun_out/pmc_traffic.log 2>&1
fi
exit $rc

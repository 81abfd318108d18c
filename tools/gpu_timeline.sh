# rocprofv3 kernel trace of the bench (graph replay) -> one step's kernel timeline + stats
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/kt -o kt --output-format csv -- python3 $R/bench.py --no-cpu --no-chars --steps 20 > $R/gpurun_out/kt.log 2>&1
rc=$?
cd $R
f=$(ls gpurun_out/kt/*/kt_kernel_trace.csv gpurun_out/kt/kt_kernel_trace.csv 2>/dev/null | head -1)
python3 tools/step_timeline.py $f ${ANCHOR:-select_wave_kernel} 12 > gpurun_out/timeline.txt 2>&1
cat gpurun_out/timeline.txt
s=$(ls gpurun_out/kt/*/kt_kernel_stats.csv gpurun_out/kt/kt_kernel_stats.csv 2>/dev/null | head -1)
python3 - "$s" <<'PY' > gpurun_out/kernel_stats.txt
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:25]:
    print(f'{r["Name"][:70]:70s} calls={r["Calls"]:>5s} avg_us={float(r["AverageNs"])/1e3:9.2f} tot_ms={float(r["TotalDurationNs"])/1e6:8.3f}')
PY
cat gpurun_out/kernel_stats.txt | head -12
exit $rc

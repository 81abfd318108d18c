# rocprofv3 kernel-trace stats of the bench (true per-kernel device durations)
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/kt -o kt --output-format csv -- python3 $R/bench.py --no-cpu --steps 10 > $R/gpurun_out/kstats.log 2>&1
rc=$?
cd $R
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/kt/**/kt_kernel_stats.csv", recursive=True) + glob.glob("gpurun_out/kt/kt_kernel_stats.csv")
rows = list(csv.DictReader(open(f[0])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:25]:
    print(f'{r["Name"][:70]:70s} calls={r["Calls"]:>5s} avg_us={float(r["AverageNs"])/1e3:9.2f} tot_ms={float(r["TotalDurationNs"])/1e6:8.3f}')
PY
exit $rc

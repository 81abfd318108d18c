"""Print one pass of the bench's kernel sequence from a rocprofv3 kernel trace: start offset,
duration and the idle gap before each kernel.  usage: step_timeline.py TRACE_CSV [ANCHOR] [NTH]
A pass runs from the NTH launch of the anchor kernel (default: the first kernel of a step,
the winsorize select) to the next one."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
anchor = sys.argv[2] if len(sys.argv) > 2 else "select_wave_kernel"
nth = int(sys.argv[3]) if len(sys.argv) > 3 else 8
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]]
a = idx[min(nth, len(idx) - 2)]
b = idx[min(nth, len(idx) - 2) + 1]
# include kernels of the step that start before the anchor (side stream, same step)
t0 = int(rows[a]["Start_Timestamp"])
last_end = t0
for r in rows[a:b]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].split("(")[0][:70]
    print(f"{(s - t0) / 1e3:8.1f} us  dur {(e - s) / 1e3:7.1f}  gap {(s - last_end) / 1e3:6.1f}  "
          f"q{r.get('Stream_Id', r.get('Queue_Id', '?'))}  {name}")
    last_end = max(last_end, e)
print(f"span {(last_end - t0) / 1e3:.1f} us; next step starts at {(int(rows[b]['Start_Timestamp']) - t0) / 1e3:.1f} us")

"""Print one pass of the bench's kernel sequence from a rocprofv3 kernel trace: start offset,
duration and the idle gap before each kernel (usage: step_timeline.py TRACE_CSV [NTH_GRAM])."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
nth = int(sys.argv[2]) if len(sys.argv) > 2 else 8
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
grams = [i for i, r in enumerate(rows) if "gram_kernel" in r["Kernel_Name"]]
i0 = grams[min(nth, len(grams) - 1)]
# back up to the step's first kernel: the previous gram's successor chain
prev = grams[min(nth, len(grams) - 1) - 1]
j = prev + 1
while j < i0 and "ts_fused" not in rows[j]["Kernel_Name"]:
    j += 1
j += 1
while j < i0 and "ts_fused" in rows[j]["Kernel_Name"]:
    j += 1
start = j
end = grams[min(nth + 1, len(grams) - 1)]
t0 = int(rows[start]["Start_Timestamp"])
last_end = t0
for r in rows[start:end]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].split("(")[0][:60]
    print(f"{(s - t0) / 1e3:8.1f} us  dur {(e - s) / 1e3:7.1f}  gap {(s - last_end) / 1e3:6.1f}  "
          f"q{r.get('Stream_Id', r.get('Queue_Id', '?'))}  {name}")
    last_end = max(last_end, e)
print(f"span {(last_end - t0) / 1e3:.1f} us")

"""Average each PMC counter per kernel (largest-grid dispatches) from a rocprofv3
counter_collection.csv: python tools/pmc_summary.py <csv> [kernel-substring ...]"""
import csv
import sys
from collections import defaultdict


def main():
    path, pats = sys.argv[1], sys.argv[2:]
    vals = defaultdict(lambda: defaultdict(float))
    meta = {}
    for r in csv.DictReader(open(path)):
        d = r["Dispatch_Id"]
        vals[d][r["Counter_Name"]] += float(r["Counter_Value"])
        meta[d] = (r["Kernel_Name"], int(float(r.get("Grid_Size", 0) or 0)))
    groups = defaultdict(list)
    for d, (name, g) in meta.items():
        short = name.split("(")[0].split("<")[0][-40:] + ("<" + name.split("<")[1].split(">")[0] + ">" if "<" in name else "")
        if pats and not any(p in name for p in pats):
            continue
        groups[(short, g)].append(d)
    for (short, g), ds in sorted(groups.items()):
        print(f"{short}  grid={g}  dispatches={len(ds)}")
        names = sorted({c for d in ds for c in vals[d]})
        for c in names:
            print(f"    {c:28s} {sum(vals[d][c] for d in ds) / len(ds):16.1f}")


if __name__ == "__main__":
    main()

"""Per-launch HBM traffic from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; KiB).

Usage: python tools/pmc_traffic.py <fetch_counter_collection.csv> <write_counter_collection.csv> [out.json [lib_sha16]]

FETCH_SIZE is calibrated on the fm_stream_probe dispatches of tools/pmc_run.py (1 GiB read
with the panel kernels' 8-B-per-lane coalesced access): factor = true bytes / reported
bytes (MI355X_MICROARCH.md §HBM: gfx950 reports half of a 16-B/lane stream; other widths
must be calibrated).  WRITE_SIZE is taken as reported.  Output: {kernel: bytes per launch}
for the panel kernels, plus the calibration factor.
"""
import csv
import json
import sys
from collections import defaultdict

KERNELS = {"select_pair_kernel": "fm_select_cuts", "select_pair_hk_kernel": "fm_select_cuts",
           "select_fixup_universe_kernel": "fm_select_fixup_universe", "gram_kernel": "fm_gram",
           "solve16_kernel": "fm_solve", "probe_kernel": "fm_stream_probe",
           "universe_kernel": "fm_universe", "ts_fused_kernel": "fm_ts_fused"}


def per_dispatch(path, counter):
    """{dispatch: value}, {dispatch: (kernel name, grid size)}; the panel kernels are
    reported for their largest grid (fm_select_cuts also runs on the 1-column NYSE panel)."""
    vals = defaultdict(float)
    names = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            if r.get("Counter_Name") != counter:
                continue
            d = r["Dispatch_Id"]
            vals[d] += float(r["Counter_Value"])
            names[d] = (r["Kernel_Name"], int(float(r.get("Grid_Size", 0) or 0)))
    return vals, names


def main():
    fetch_csv, write_csv = sys.argv[1], sys.argv[2]
    out = sys.argv[3] if len(sys.argv) > 3 else None
    fv, fn = per_dispatch(fetch_csv, "FETCH_SIZE")
    wv, wn = per_dispatch(write_csv, "WRITE_SIZE")
    probe = [fv[d] * 1024 for d in fv if "probe_kernel" in fn[d][0]]
    true_probe = float(1 << 30)
    factor = true_probe / (sum(probe) / len(probe)) if probe else 2.0
    agg = defaultdict(lambda: {"fetch": [], "write": []})
    big = defaultdict(int)
    for names in (fn, wn):
        for d, (nm, g) in names.items():
            for k, tag in KERNELS.items():
                if k in nm:
                    big[tag] = max(big[tag], g)
    for d, v in fv.items():
        for k, tag in KERNELS.items():
            if k in fn[d][0] and fn[d][1] == big[tag]:
                agg[tag]["fetch"].append(v * 1024 * factor)
    for d, v in wv.items():
        for k, tag in KERNELS.items():
            if k in wn[d][0] and wn[d][1] == big[tag]:
                agg[tag]["write"].append(v * 1024)
    res = {"fetch_calibration_factor": factor}
    if len(sys.argv) > 4:
        res["lib_sha16"] = sys.argv[4]
    for tag, a in agg.items():
        f = sum(a["fetch"]) / len(a["fetch"]) if a["fetch"] else 0.0
        w = sum(a["write"]) / len(a["write"]) if a["write"] else 0.0
        res[tag] = f + w
        res[tag + ":fetch"] = f
        res[tag + ":write"] = w
        res[tag + ":dispatches"] = len(a["fetch"])
    print(json.dumps(res, indent=1))
    if out:
        json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()

"""Phase timeline of the latency-tail kernels on the bench panel (probe build only):
    tools/build_variant.sh probe "-DFM_PROBE=1" fm_ts.hip fm_solve.hip fm_select.hip
    FM_HIP_LIB=build_variants/probe/libfm_hip.so python tools/tail_probe.py
Each kernel's workgroups write s_memrealtime (100 MHz) at numbered points (FM_PROBE_AT in
the sources); for one re-issued launch per tag this prints, per probe point, the quantiles of
the time since the launch's first workgroup started, and per phase the workgroup-duration
quantiles -- where the launch's critical path goes."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "fm-returnprediction_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from fmcore import engine as E  # noqa: E402
from fmcore import lewellen as LW  # noqa: E402

SLOTS = 8
# tag -> (probe buffer, slot names)
TAGS = {
    "fm_universe": ("sel", {0: "start", 1: "loaded+reduced", 4: "hs: histogram", 5: "hs: scan+locate",
                            6: "hs: lists", 7: "hs: sorted", 2: "hist_select", 3: "levels"}),
    "fm_select_cuts": ("sel", {4: "fixup start", 5: "fixup read nwork"}),
    "fm_solve": ("solve", {0: "start", 1: "partials", 2: "cumulative", 4: "w0 gram rows", 5: "w0 centered",
                           6: "w0 cholesky", 7: "w0 back-subst", 3: "problems"}),
    "fm_solve_fixup": ("solve", {4: "start", 5: "end"}),
    "fm_ts_fused": ("ts", {0: "start", 1: "compact", 2: "gather", 3: "dropna|prefix", 4: "nw|rolled",
                           5: "pred preload", 6: "rolling done", 7: "end (+pred summary)"}),
    "fm_ts_fused[pred]": ("ts", {0: "start", 1: "compact", 2: "gather", 3: "dropna", 4: "nw", 7: "end"}),
}


def q(v):
    v = np.asarray(v, dtype=np.float64) / 100.0   # us
    if v.size == 0:
        return "-"
    return "/".join(f"{np.percentile(v, p):.2f}" for p in (0, 50, 90, 100))


def probe(tag, buf, names):
    lib = E.L.load()
    name, struct, keep = E.LAST_LAUNCH[tag]
    args = (E.L.C.byref(struct),) if struct is not None else keep[1]
    st = E._stream()
    for _ in range(3):
        E.L.call(name, *args, st)
    torch.cuda.synchronize()
    assert getattr(lib, f"fm_probe_clear_{buf}")() == 0
    torch.cuda.synchronize()
    E.L.call(name, *args, st)
    torch.cuda.synchronize()
    n = 8192
    host = (ctypes.c_uint32 * (SLOTS * n))()
    assert getattr(lib, f"fm_probe_copy_{buf}")(host, n) == 0
    f = np.frombuffer(host, dtype=np.uint32).reshape(n, SLOTS).astype(np.int64)
    slots = list(names)   # in the listed (execution) order
    live = (f[:, slots[0]] != 0)
    f = f[live]
    if f.shape[0] == 0:
        print(f"{tag}: no workgroup wrote slot {slots[0]}")
        return
    base = f[:, slots[0]].min()
    print(f"{tag}: {f.shape[0]} workgroups (time since first start, us: p0/p50/p90/p100)", flush=True)
    prev = None
    for sl in slots:
        col = f[:, sl]
        ok = col != 0
        line = f"  [{sl}] {names[sl]:>16}: at {q(col[ok] - base)}"
        if prev is not None:
            both = ok & (f[:, prev] != 0)
            line += f"   phase {q(col[both] - f[both, prev])}"
        print(line, flush=True)
        prev = sl


def main():
    dev = E.require_device()
    panel = E.panel_synthetic(600, 5000, 1, device=dev)
    if os.environ.get("KB_PLANES", "1") == "1":
        E.split_planes(panel)
    cfg = LW.PipelineConfig()
    for _ in range(3):
        LW.run_pipeline(panel, cfg)
    torch.cuda.synchronize()
    for tag, (buf, names) in TAGS.items():
        if tag in E.LAST_LAUNCH:
            probe(tag, buf, names)
    for tag in sorted(E.LAST_LAUNCH):
        print(f"time_launch {tag}: {E.time_launch(tag, 20) * 1e3:.1f} us", flush=True)


if __name__ == "__main__":
    main()

"""Per-workgroup timeline of fm_gram on the bench panel (probe build only):
    tools/build_variant.sh wgtime "-DFM_GRAM_WGTIME=1" fm_gram.hip
    FM_HIP_LIB=build_variants/wgtime/libfm_hip.so python tools/gram_wgtime.py
Each workgroup writes its start / end (s_memrealtime, 100 MHz) and HW_ID into the reserved
flags buffer; printed: the launch span, workgroup duration quantiles, start skew, and the
busiest CUs' serial time, for the whole-month plan and the balanced plan."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "fm-returnprediction_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from fmcore import engine as E  # noqa: E402
from fmcore import lewellen as LW  # noqa: E402


def run(panel, pol):
    panel.chunk_policy = pol
    panel.__dict__.pop("_chunk_cache", None)
    cfg = LW.PipelineConfig()
    for _ in range(3):
        LW.run_pipeline(panel, cfg)
    torch.cuda.synchronize()
    ga = E.LAST_LAUNCH["fm_gram"][1]   # the captured GramArgs (the last model group's launch)
    nwg = ga.nwg if ga.wg_chunk_off else ga.nchunks
    for _ in range(3):
        E.L.call("fm_gram", E.L.C.byref(ga), E._stream())
    torch.cuda.synchronize()
    import ctypes
    host = (ctypes.c_uint32 * (4 * nwg))()
    assert E.L.load().fm_gram_wgtime_copy(host, nwg) == 0
    f = np.frombuffer(host, dtype=np.uint32).reshape(nwg, 4).astype(np.int64)
    t0, t1, hw, nch = f[:, 0], f[:, 1], f[:, 2], f[:, 3]
    base = t0.min()
    s, e = (t0 - base) * 10, (t1 - base) * 10   # ns
    d = e - s
    cu = (hw >> 8) & 0xF | ((hw >> 13) & 0x3) << 4 | ((hw >> 12) & 1) << 6   # cu, se, sh bits (per XCC)
    print(f"{pol}: {nwg} workgroups, span {e.max() / 1e3:.1f} us, wg duration p0/p50/p90/p100 "
          f"{np.percentile(d, 0) / 1e3:.1f}/{np.percentile(d, 50) / 1e3:.1f}/{np.percentile(d, 90) / 1e3:.1f}/"
          f"{d.max() / 1e3:.1f} us, start p50/p90/max {np.percentile(s, 50) / 1e3:.1f}/{np.percentile(s, 90) / 1e3:.1f}/"
          f"{s.max() / 1e3:.1f} us, end p10/p50 {np.percentile(e, 10) / 1e3:.1f}/{np.percentile(e, 50) / 1e3:.1f} us, "
          f"chunks/wg max {nch.max()}", flush=True)
    hist = np.histogram(e / 1e3, bins=10)
    print("  end-time histogram (us):", " ".join(f"{b:.0f}:{c}" for b, c in zip(hist[1], hist[0])))


def main():
    dev = E.require_device()
    panel = E.panel_synthetic(600, 5000, 1, device=dev)
    if os.environ.get("KB_PLANES") == "1":
        E.split_planes(panel)
    run(panel, ("months", 5000))
    run(panel, E.chunk_policy(panel.nrows, panel.nseg, panel.max_seg_len))


if __name__ == "__main__":
    main()

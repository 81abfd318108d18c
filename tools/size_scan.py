"""Per-kernel device time vs the number of months (the grid size) at 5,000 firms, and the
Gram / select re-read from the Infinity Cache: python tools/size_scan.py

1. months in (256, 384, 512, 600, 640, 768, 1024): one whole month per Gram workgroup, so
   the workgroups per CU go 1, 1.5, 2, 2.34, 2.5, 3, 4 -- whether the headline's 600-month
   grid (2 or 3 months per CU) pays a per-CU imbalance shows as a higher us / month at 600.
2. a 150-month panel (90 MB: fits the 256 MiB Infinity Cache) with 4 Gram chunks per month
   (600 workgroups, the headline's grid): back-to-back launches re-read it on-die, against
   the same launch after a 1 GiB copy has flushed the cache."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "fm-returnprediction_amd"), ROOT]

import torch  # noqa: E402

from fmcore import engine as E  # noqa: E402
from fmcore import lewellen as LW  # noqa: E402

TAGS = ("fm_select_cuts", "fm_universe", "fm_gram", "fm_solve", "fm_ts_fused", "fm_ts_fused[pred]")


def flushed(tag, flush_a, flush_b, reps=10):
    """Average device ms of `tag`'s latest launch, each launch after a 1 GiB copy."""
    name, struct, keep = E.LAST_LAUNCH[tag]
    from fmcore import _lib as L
    st = torch.cuda.current_stream().cuda_stream
    args = (L.C.byref(struct),) if struct is not None else keep[1]
    tot = 0.0
    for _ in range(reps):
        flush_b.copy_(flush_a)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        L.call(name, *args, st)
        e1.record()
        e1.synchronize()
        tot += e0.elapsed_time(e1)
    return tot / reps


def main():
    dev = E.require_device()
    cfg = LW.PipelineConfig()
    for T in (256, 384, 512, 600, 640, 768, 1024):
        panel = E.panel_synthetic(T, 5000, 1, device=dev)
        E.LAST_LAUNCH.clear()
        for _ in range(2):
            LW.run_pipeline(panel, cfg)
        torch.cuda.synchronize()
        ms = {t: E.time_launch(t, 20) for t in TAGS if t in E.LAST_LAUNCH}
        print(f"T={T:5d} " + " ".join(f"{t}={v * 1e3:7.1f}us({v * 1e6 / T:6.1f}ns/mo)" for t, v in ms.items()),
              flush=True)
        del panel
        torch.cuda.empty_cache()
    fa = torch.empty(1 << 27, dtype=torch.float64, device=dev)
    fb = torch.empty_like(fa)
    for T, ch in ((150, 1250), (600, 5000), (600, 1250)):
        panel = E.panel_synthetic(T, 5000, 1, device=dev)
        panel.chunk_rows = ch
        E.LAST_LAUNCH.clear()
        for _ in range(2):
            LW.local_stage(panel, cfg, LW.table2_models())
        torch.cuda.synchronize()
        warm = {t: E.time_launch(t, 20) for t in ("fm_gram", "fm_select_cuts")}
        cold = {t: flushed(t, fa, fb) for t in ("fm_gram", "fm_select_cuts")}
        print(f"T={T} chunk={ch} nchunks={E._chunk_plan(panel).nchunks} " +
              " ".join(f"{t}: back-to-back {warm[t] * 1e3:.1f}us, after flush {cold[t] * 1e3:.1f}us" for t in warm),
              flush=True)
        del panel
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

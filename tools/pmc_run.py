"""Workload for the rocprofv3 PMC passes (run under `rocprofv3 --pmc FETCH_SIZE` and,
separately, `--pmc WRITE_SIZE`; see tools/pmc_traffic.py).

1. Calibration: fm_stream_probe reads a 1 GiB FP64 buffer as a coalesced 16-byte-per-lane
   stream; its true byte count calibrates FETCH_SIZE (gfx950 reports half of a wide
   streaming read, MI355X_MICROARCH.md §HBM).
2. The bench workload (C3+C4 panel, full pipeline) for a few steps.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "fm-returnprediction_amd"), ROOT]

import torch  # noqa: E402

from fmcore import engine as E  # noqa: E402
from fmcore import lewellen as LW  # noqa: E402


def main(steps=3):
    dev = E.require_device()
    buf = torch.ones(1 << 27, dtype=torch.float64, device=dev)   # 1 GiB
    for _ in range(3):
        E.stream_probe(buf)
    del buf
    T, N = (1000, 20000) if os.environ.get("FM_PMC_LONG") == "1" else (600, 5000)   # C5-shaped months
    # the bench's planes-only panel (fm_gen_panel_planes); FM_PLANES=0: FP64 columns
    panel = E.panel_synthetic(T, N, 1, device=dev, layout="planes" if os.environ.get("FM_PLANES", "1") == "1" else "f64")
    panel.chunk_policy = E.chunk_policy(panel.nrows, panel.nseg, panel.max_seg_len)   # as bench.make_step
    cfg = LW.PipelineConfig()
    for _ in range(steps):
        LW.run_pipeline(panel, cfg)
    torch.cuda.synchronize()
    print("pmc workload done")


if __name__ == "__main__":
    main()

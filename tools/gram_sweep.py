"""Time fm_gram alone on the bench panel for several chunk sizes (HIP events on the launch
stream, engine.time_launch).  python tools/gram_sweep.py [chunk_rows ...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "fm-returnprediction_amd"), ROOT]

import torch  # noqa: E402

from fmcore import engine as E  # noqa: E402
from fmcore import lewellen as LW  # noqa: E402


def main():
    dev = E.require_device()
    panel = E.panel_synthetic(600, 5000, 1, device=dev)
    cfg = LW.PipelineConfig()
    sizes = [int(x) for x in sys.argv[1:]] or [1280, 2560, 5120, 768, 512]
    for ch in sizes:
        panel.chunk_rows = ch
        panel.__dict__.pop("_chunk_cache", None)
        for _ in range(3):
            LW.local_stage(panel, cfg, LW.table2_models())
        torch.cuda.synchronize()
        # device time of the latest launch re-issued back to back (no host gaps)
        print(f"chunk_rows={ch} nchunks={E._chunk_plan(panel).nchunks} "
              f"gram_ms={E.time_launch('fm_gram', 50):.4f} solve_ms={E.time_launch('fm_solve', 50):.4f}",
              flush=True)


if __name__ == "__main__":
    main()

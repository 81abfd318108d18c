"""fm_gram / fm_solve device time, whole-month vs split-month (engine.make_chunks_split) Gram
plans, at 5,000 firms: python tools/split_scan.py [months ...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "fm-returnprediction_amd"), ROOT]

import torch  # noqa: E402

from fmcore import engine as E  # noqa: E402
from fmcore import lewellen as LW  # noqa: E402


def main():
    dev = E.require_device()
    cfg = LW.PipelineConfig()
    months = [int(x) for x in sys.argv[1:]] or [512, 600, 700, 768, 1024]
    for T in months:
        panel = E.panel_synthetic(T, 5000, 1, device=dev)
        out = []
        for split in (False, True):
            panel.chunk_split = split
            panel.__dict__.pop("_chunk_cache", None)
            E.LAST_LAUNCH.clear()
            for _ in range(3):
                LW.run_pipeline(panel, cfg)   # the select runs before the Gram, as in a step
            torch.cuda.synchronize()
            g = sorted(E.time_launch("fm_gram", 20) for _ in range(5))[2]
            sv = sorted(E.time_launch("fm_solve", 20) for _ in range(5))[2]
            out.append(f"{'split' if split else 'whole'}: nchunks={E._chunk_plan(panel).nchunks} "
                       f"gram={g * 1e3:6.1f}us solve={sv * 1e3:5.1f}us")
        print(f"T={T:5d} " + " | ".join(out), flush=True)
        del panel
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

"""Cold-vs-warm A/B of the Gram's panel read (is the second read of the
panel served by the 256 MiB Infinity Cache?).  On the bench's planes-only 600 x 5,000 x 15
panel, after one pipeline pass has filled engine.LAST_LAUNCH, the captured Gram launch is
timed (HIP events on the launch stream, median of 15) right after:

  warm_select   the two-wave select + fix-up/universe launch (the order inside a step: the
                select has just streamed the 180 MB high plane, last months last);
  warm_gram     another Gram launch (363 MB: more than the cache, so LRU leaves its tail);
  cold_write    a 1 GiB write to another buffer (evicts the caches, but leaves up to 256 MiB
                of dirty lines whose write-back then competes with the Gram's reads);
  cold          a 1 GiB READ of another buffer (evicts the Infinity Cache and the L2s clean);
  warm_half     a read of the high plane's last 300 months only (90 MB, the part of the
                select's stream most likely still resident).

python tools/cache_ab.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "fm-returnprediction_amd"), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from fmcore import _lib as L, engine as E, lewellen as LW  # noqa: E402


def reissue(tag):
    name, struct, keep = E.LAST_LAUNCH[tag]
    args = (L.C.byref(struct),) if struct is not None else keep[1]
    L.call(name, *args, E._stream())


def main():
    E.require_device()
    panel = E.panel_synthetic(600, 5000, 1, layout="planes")
    cfg = LW.PipelineConfig()
    for _ in range(2):
        LW.run_pipeline(panel, cfg)
    torch.cuda.synchronize()
    junk = torch.empty(1 << 27, dtype=torch.float64, device=panel.device)   # 1 GiB
    hi_tail = panel.planes[0][:, 300 * 5000:]
    sink = torch.zeros(1, dtype=torch.float64, device=panel.device)

    def before(kind):
        if kind == "warm_select":
            reissue("fm_select_cuts")
        elif kind == "warm_gram":
            reissue("fm_gram")
        elif kind == "cold_write":
            junk.fill_(1.0)
        elif kind == "cold":
            E.stream_probe(junk)
        elif kind == "warm_half":
            sink.add_(hi_tail.sum(dtype=torch.int64).to(torch.float64))

    out = {}
    junk.fill_(1.0)
    torch.cuda.synchronize()
    for kind in ("warm_select", "warm_gram", "cold", "cold_write", "warm_half", "warm_select", "cold"):
        ts = []
        for _ in range(15):
            before(kind)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            reissue("fm_gram")
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        out.setdefault(kind, []).append(float(np.median(ts)))
    print("CACHE_AB " + json.dumps({k: [round(x, 1) for x in v] for k, v in out.items()}), flush=True)


if __name__ == "__main__":
    main()

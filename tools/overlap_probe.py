"""Does fm_select overlap fm_gram when both are in flight on two streams?  (A/B probe for the
fused-pass design; no dependency between the two launches here: the Gram re-uses the cuts
of the previous pass.)  Prints device ms of select alone, gram alone, both sequential on one
stream, and both on two streams."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "fm-returnprediction_amd"), ROOT]
import torch  # noqa: E402
from fmcore import _lib as L  # noqa: E402
from fmcore import engine as E  # noqa: E402
from fmcore import lewellen as LW  # noqa: E402


def main():
    dev = E.require_device()
    panel = E.panel_synthetic(600, 5000, 1, device=dev)
    cfg = LW.PipelineConfig()
    for _ in range(3):
        LW.run_pipeline(panel, cfg)
    torch.cuda.synchronize()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def issue(tag, stream):
        name, struct, keep = E.LAST_LAUNCH[tag]
        L.call(name, L.C.byref(struct), stream.cuda_stream)

    def timed(fn, reps=20):
        torch.cuda.synchronize()
        t0 = torch.cuda.Event(enable_timing=True)
        t1 = torch.cuda.Event(enable_timing=True)
        t0.record(s1)
        s2.wait_event(t0)
        for _ in range(reps):
            fn()
        e2 = torch.cuda.Event()
        e2.record(s2)
        s1.wait_event(e2)
        t1.record(s1)
        t1.synchronize()
        return t0.elapsed_time(t1) / reps

    r = {}
    r["select"] = timed(lambda: issue("fm_select_cuts", s1))
    r["gram"] = timed(lambda: issue("fm_gram", s1))
    r["universe"] = timed(lambda: L.call("fm_universe", *E.LAST_LAUNCH["fm_universe"][2][1], s1.cuda_stream))
    r["seq_select_gram"] = timed(lambda: (issue("fm_select_cuts", s1), issue("fm_gram", s1)))
    r["par_select_gram"] = timed(lambda: (issue("fm_select_cuts", s1), issue("fm_gram", s2)))
    r["par_gram_select"] = timed(lambda: (issue("fm_gram", s2), issue("fm_select_cuts", s1)))
    for k, v in r.items():
        print(f"{k:18s} {v * 1e3:8.1f} us", flush=True)


if __name__ == "__main__":
    main()

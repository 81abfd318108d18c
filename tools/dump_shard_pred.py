"""Fixture for tests/test_dist_gloo.py: the per-shard predictive records of the real device
pipeline (GPU run).  A ragged 96-month panel is split into 3 month ranges with
dist.shard_bounds; each range runs local_stage with the global chunk policy, the records are
concatenated (what the all-gather assembles) and every shard runs time_series_stage on the
full series with its own moments and month range.  Saved: each shard's (pred, pst) -- rows
of other shards' months as the kernels left them -- and the unsharded run's (pred, pst).
Usage (GPU box): python tools/dump_shard_pred.py tests/golden/shard_pred.npz"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "fm-returnprediction_amd"), ROOT, os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main(path):
    from fmcore import dist as D, engine as E, lewellen as LW, synth
    E.require_device()
    a = synth.synth_arrays(96, 400, 13, nan_rate=0.03, present_rate=0.6)
    early = a["month"] < a["month"].min() + 17          # Model-3-only column missing early
    a["log_return_13_36"][early] = np.nan
    cols = list(dict.fromkeys(["retx"] + [c for xs in LW.table2_models().values() for c in xs] + LW.FIG1_VARS))
    panel = E.panel_from_arrays([a[c] for c in cols], cols, a["month"], me=a["me"], nyse=a["nyse"])
    cfg = LW.PipelineConfig()
    mc = LW.table2_models()
    full = LW.run_pipeline(panel, cfg, model_cols=mc)
    off = panel.seg_off_h
    ch = E.default_chunk_rows(panel.nrows, panel.nseg, panel.max_seg_len)
    bounds = D.shard_bounds(np.diff(off), 3)
    locs = []
    for s0, s1 in bounds:
        r0, r1 = int(off[s0]), int(off[s1])
        so = off[s0:s1 + 1] - off[s0]
        sub = E.DevicePanel(cols=panel.cols[:, r0:r1].contiguous(), names=panel.names,
                            seg_off=torch.from_numpy(so).to(panel.cols.device), seg_off_h=so,
                            me=panel.me[r0:r1].contiguous(), nyse=panel.nyse[r0:r1].contiguous(), chunk_rows=ch)
        locs.append(LW.local_stage(sub, cfg, mc)[0])
    rec = torch.cat([r.rec for r in locs])
    st = torch.cat([r.status for r in locs])
    out = {"bounds": np.array(bounds, dtype=np.int64), "full_pred": full.pred.cpu().numpy(),
           "full_pst": full.pred_status.cpu().numpy()}
    for i, ((s0, s1), loc) in enumerate(zip(bounds, locs)):
        g = E.FMResult(problems=loc.problems, rec=rec, status=st, pmax=loc.pmax, moments=loc.moments,
                       mom_stride=loc.mom_stride)
        _, _, _, p, ps = LW.time_series_stage(g, cfg, moments=loc.moments, seg_lo=s0, seg_hi=s1)
        out[f"pred{i}"] = p.cpu().numpy()
        out[f"pst{i}"] = ps.cpu().numpy()
    np.savez_compressed(path, **out)
    print("wrote", path, {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main(sys.argv[1])

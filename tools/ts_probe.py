"""Time the fused time-series kernel phase by phase at the bench panel size (GPU)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "fm-returnprediction_amd"))
import torch  # noqa: E402
from fmcore import engine as E  # noqa: E402
from fmcore import lewellen as LW  # noqa: E402

dev = torch.device("cuda", 0)
panel = E.panel_synthetic(600, 5000, 0, device=dev)
cfg = LW.PipelineConfig()
res, names, cuts, level, bp = LW.local_stage(panel, cfg, LW.table2_models())
torch.cuda.synchronize()
for roll, pred in ((False, False), (True, False), (True, True)):
    out = E.time_series_result(res, rolling=roll, predictive=pred)
    torch.cuda.synchronize()
    print(f"ts_fused rolling={roll} predictive={pred}: {E.time_launch('fm_ts_fused', 50) * 1e3:.1f} us")
pred, pst = out[3], out[4]
E.summarize_predictive(pred, pst, 4)
torch.cuda.synchronize()
print(f"summarize_predictive: {E.time_launch('fm_ts_fused', 50) * 1e3:.1f} us")

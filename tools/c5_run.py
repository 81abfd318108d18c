"""One rank's C5 shard (12,500 months x 20,000 firms) through run_pipeline, for rocprofv3."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "fm-returnprediction_amd"), ROOT]

import torch  # noqa: E402

from fmcore import engine as E  # noqa: E402
from fmcore import lewellen as LW  # noqa: E402

p = E.panel_synthetic(12500, 20000, 20150101, month0=50000)
cfg = LW.PipelineConfig()
for _ in range(3):
    LW.run_pipeline(p, cfg)
torch.cuda.synchronize()
print("c5 done")

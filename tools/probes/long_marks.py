"""Probe: how many (month, column) units the long-month select leaves marked for the
streaming fallback (nvalid == -1), on the selbench panel.  Needs a library built with
-DFM_AB_NOFB=1 (no fallback launch): FM_HIP_LIB=<that .so> python tools/probes/long_marks.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "fm-returnprediction_amd"), ROOT]
import torch  # noqa: E402
from fmcore import engine as E  # noqa: E402

E.require_device()
T, N = int(os.environ.get("SB_T", "200")), int(os.environ.get("SB_N", "20000"))
p = E.panel_synthetic(T, N, 20150101, month0=50000)
cuts = E.select_cuts(p, 0.01, 0.99, 5, center=True)
torch.cuda.synchronize()
nv = cuts.nvalid
print("units", nv.numel(), "marked", int((nv == -1).sum()))

"""Diagnostic: which (month, column) units does the wave select kernel hand to the fallback
pass on the bench panel?  Needs a diagnostic library built with
-DFM_SELECT_DIAG_NO_FALLBACK (marks stay as nvalid == -1); the shipped library never is."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "fm-returnprediction_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from fmcore import engine as E  # noqa: E402


def main():
    dev = E.require_device()
    panel = E.panel_synthetic(600, 5000, 1, device=dev)
    cuts = E.select_cuts(panel, 0.01, 0.99, 5, E.LERP_NUMPY, center=True)
    nv = cuts.nvalid.cpu().numpy()
    marks = nv == -1
    print("marked units:", int(marks.sum()), "of", nv.size)
    print("per column:", marks.sum(axis=1).tolist())
    cols = panel.cols.cpu().numpy()
    for c, s in list(zip(*np.nonzero(marks)))[:6]:
        x = cols[c, s * 5000:(s + 1) * 5000]
        v = x[~np.isnan(x)]
        n = len(v)
        lanes = [x[l::64] for l in range(64)]
        mins = np.array([np.nanmin(t) if np.any(~np.isnan(t)) else np.nan for t in lanes])
        j0 = int(np.floor((n - 1) * 0.01)) + 1
        tau = np.sort(mins)[j0]
        print(f"col {c} ({panel.names[c]}) month {s}: n={n} j0={j0} tau={tau!r} "
              f"cand_lo={int((v < tau).sum())} ninf={int(np.isinf(v).sum())} nuniq={len(np.unique(v))}")


if __name__ == "__main__":
    main()

"""Drop-in for the reference's src/transform_compustat.py annual -> monthly expansion.

expand_compustat_annual_to_monthly keeps the reference's name, signature and output
(reference src/transform_compustat.py:101-172): per `id_col` group, one row for every
month-end from its first `report_date` to min(the table's latest report date, its own last
report date + 12 months), each carrying the group's latest record at or before that month
(pandas reindex(method="ffill")), columns [id_col, "fund_date", <the input columns except
fyear>], sorted by (id_col, fund_date).  The forward-fill gather runs on the device
(fmcore.etl.expand_monthly -> fm_ffill_expand); float64 columns are gathered there, columns
of other dtypes by the same source indices on the host.  Like the reference (whose
reindex raises on duplicate labels), a repeated (id, report_date) raises ValueError.
The CCM link merge (merge_CRSP_and_Compustat) is a string/date-keyed pandas join upstream of
the panel and stays with the reference module.
"""
from __future__ import annotations

import os
import sys

import numpy as np
import pandas as pd

_HERE = os.path.dirname(os.path.abspath(__file__))
_PKG = os.path.dirname(_HERE)
if _PKG not in sys.path:
    sys.path.insert(0, _PKG)

from fmcore import etl as _X  # noqa: E402


def expand_compustat_annual_to_monthly(comp_annual: pd.DataFrame, id_col: str = "gvkey",
                                       report_date_col: str = "report_date") -> pd.DataFrame:
    df = comp_annual.drop(columns=["fyear"], errors="ignore")
    dates = pd.to_datetime(df[report_date_col])
    if df.duplicated(subset=[id_col, report_date_col]).any():
        raise ValueError("cannot reindex on an axis with duplicate labels")
    codes, uniq = pd.factorize(df[id_col], sort=True)
    fcols = [c for c in df.columns if df[c].dtype == np.float64]
    gcode, fund_date, outs, src = _X.expand_monthly(codes.astype(np.int64), dates.to_numpy(),
                                                    [df[c].to_numpy() for c in fcols])
    out = {id_col: uniq.take(gcode).to_numpy() if hasattr(uniq, "take") else np.asarray(uniq)[gcode],
           "fund_date": fund_date}
    fi = dict(zip(fcols, outs))
    for c in df.columns:
        if c == id_col:
            continue
        out[c] = fi[c] if c in fi else df[c].to_numpy().take(src)
    res = pd.DataFrame(out)
    res[id_col] = res[id_col].astype(df[id_col].dtype)
    return res

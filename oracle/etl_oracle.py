"""CPU restatement of the reference's annual -> monthly Compustat expansion -- TEST
INFRASTRUCTURE ONLY (tests/ import it as the checker; the product path,
fm-returnprediction_amd/, never does).

expand_compustat_annual_to_monthly follows reference src/transform_compustat.py:101-172:
drop fyear (:139), fund_date = report_date (:142), sort by (id, fund_date) (:145-146), per
group a month-end range from its first fund_date to min(the table's latest fund_date, its
last + 12 months) (:149-157), each month taking the group's last record at or before it
(reindex(method="ffill"), :166), concatenated in id order and reset to columns
[id, fund_date, ...] (:169-176).  Pinned by tests/golden/etl.npz (the reference's own
output, tests/golden/gen_etl_goldens.py).
"""
from __future__ import annotations

import numpy as np
import pandas as pd


def expand_compustat_annual_to_monthly(comp_annual, id_col="gvkey", report_date_col="report_date"):
    df = comp_annual.drop(columns=["fyear"], errors="ignore").copy()
    df["fund_date"] = pd.to_datetime(df[report_date_col])
    df = df.sort_values([id_col, "fund_date"], kind="mergesort").reset_index(drop=True)
    max_all = df["fund_date"].max()
    parts = []
    for key, grp in df.groupby(id_col, sort=True):
        d = grp["fund_date"].to_numpy()
        end = min(max_all, grp["fund_date"].max() + pd.DateOffset(months=12))
        months = pd.date_range(grp["fund_date"].min(), end, freq="ME")
        src = np.searchsorted(d, months.to_numpy(), side="right") - 1
        part = grp.iloc[src].drop(columns=["fund_date"]).reset_index(drop=True)
        part["fund_date"] = months.to_numpy()
        parts.append(part)
    out = pd.concat(parts, ignore_index=True)
    cols = [id_col, "fund_date"] + [c for c in df.columns if c not in (id_col, "fund_date")]
    return out[cols]


def merge_CRSP_and_Compustat(crsp, comp, ccm):
    """Restatement of reference src/transform_compustat.py:175-226 with pandas' own merges:
    open-ended links (NaT linkenddt) end today (:218), the gvkey left merge (:220), the link
    window jdate in [linkdt, linkenddt] (:222), columns permno + comp's (:224-225), the inner
    (permno, jdate) merge with CRSP (:228)."""
    ccm = ccm.copy()
    ccm["linkenddt"] = ccm["linkenddt"].fillna(pd.to_datetime("today"))
    comp = comp.rename(columns={"fund_date": "jdate"})
    m = pd.merge(comp, ccm, how="left", on=["gvkey"])
    m = m[(m["jdate"] >= m["linkdt"]) & (m["jdate"] <= m["linkenddt"])]
    m = m[["permno"] + list(comp.columns)]
    return pd.merge(crsp, m, how="inner", on=["permno", "jdate"])

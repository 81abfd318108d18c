"""Drop-in for the reference's src/transform_compustat.py annual -> monthly expansion.

expand_compustat_annual_to_monthly keeps the reference's name, signature and output
(reference src/transform_compustat.py:101-172): per `id_col` group, one row for every
month-end from its first `report_date` to min(the table's latest report date, its own last
report date + 12 months), each carrying the group's latest record at or before that month
(pandas reindex(method="ffill")), columns [id_col, "fund_date", <the input columns except
fyear>], sorted by (id_col, fund_date); fund_date is datetime64[ns] whatever the input unit
(pd.date_range's default), rows with a missing id are dropped (groupby), a NaT report date
raises ValueError (as the reference's date_range / reindex do).  The forward-fill gather runs on the device
(fmcore.etl.expand_monthly -> fm_ffill_expand); float64 columns are gathered there, columns
of other dtypes by the same source indices on the host.  Like the reference (whose
reindex raises on duplicate labels), a repeated (id, report_date) raises ValueError.

merge_CRSP_and_Compustat keeps the reference's name, signature and output (reference
src/transform_compustat.py:175-226): the gvkey link merge, the link-date window and the
(permno, jdate) inner merge with CRSP, with pandas' row order (left rows in order, each with
its matches in the right frame's order), column order and _x / _y suffixes.  The two
equality joins run on the device (fmcore.etl.join_pairs -> fm_sorted_join) on integer
codes of the keys; the frames are assembled from the matched row indices.
"""
from __future__ import annotations


import numpy as np
import pandas as pd

from fmcore import etl as _X


def expand_compustat_annual_to_monthly(comp_annual: pd.DataFrame, id_col: str = "gvkey",
                                       report_date_col: str = "report_date") -> pd.DataFrame:
    df = comp_annual.drop(columns=["fyear"], errors="ignore")
    # groupby(level=id_col) drops rows whose id is missing (reference :165-168)
    df = df.loc[df[id_col].notna().to_numpy()]
    dates = pd.to_datetime(df[report_date_col])
    if dates.isna().any():
        # the reference's per-group date_range / reindex raise ValueError on a NaT date
        raise ValueError("report_date contains NaT")
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


def _codes(*cols):
    """Joint integer codes of equal values across the given Series (NaN -> its own code,
    since pandas merge matches NaN keys with NaN keys)."""
    allv = pd.concat([pd.Series(c).reset_index(drop=True) for c in cols], ignore_index=True)
    codes, _ = pd.factorize(allv, use_na_sentinel=False)
    out, o = [], 0
    for c in cols:
        out.append(codes[o:o + len(c)].astype(np.int64))
        o += len(c)
    return out


def _assemble(left, right, li, rj, keys):
    """pandas merge(left, right, on=keys) output from matched row indices: the key columns
    come from the left frame, overlapping non-key columns get _x / _y."""
    lf = left.iloc[li].reset_index(drop=True)
    rf = right.drop(columns=keys).iloc[rj].reset_index(drop=True)
    dup = [c for c in rf.columns if c in lf.columns]
    lf = lf.rename(columns={c: f"{c}_x" for c in dup})
    rf = rf.rename(columns={c: f"{c}_y" for c in dup})
    return pd.concat([lf, rf], axis=1)


def merge_CRSP_and_Compustat(crsp, comp, ccm):
    # if linkenddt is missing then set to today (the reference mutates the caller's ccm)
    ccm["linkenddt"] = ccm["linkenddt"].fillna(pd.to_datetime("today"))
    comp = comp.rename(columns={"fund_date": "jdate"})
    # ccm1 = merge(comp, ccm, how="left", on="gvkey"), restricted to the link window: an
    # unmatched comp row (NaN link dates) never passes the window, so the inner pairs suffice
    gl, gr = _codes(comp["gvkey"], ccm["gvkey"])
    li, rj = _X.join_pairs([gl], [gr])
    jd = comp["jdate"].to_numpy()[li]
    ok = (jd >= ccm["linkdt"].to_numpy()[rj]) & (jd <= ccm["linkenddt"].to_numpy()[rj])
    li, rj = li[ok], rj[ok]
    comp_col = ["permno"] + list(comp.columns)
    ccm2 = _assemble(comp, ccm, li, rj, ["gvkey"])
    ccm2["gvkey"] = comp["gvkey"].to_numpy()[li]
    ccm2 = ccm2[comp_col]
    # crsp_comp_merged = merge(crsp, ccm2, how="inner", on=["permno", "jdate"])
    pl, pr = _codes(crsp["permno"], ccm2["permno"])
    dl, dr = _codes(crsp["jdate"], ccm2["jdate"])
    li2, rj2 = _X.join_pairs([pl, dl], [pr, dr])
    return _assemble(crsp, ccm2, li2, rj2, ["permno", "jdate"])

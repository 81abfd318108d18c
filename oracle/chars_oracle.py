"""CPU ORACLE — test infrastructure only, never the product path.

numpy restatement of the firm-axis characteristic construction that feeds winsorize in the
reference's get_factors (BaileyMeche/FM-ReturnPrediction, src/calc_Lewellen_2014.py:531-575):
the twelve monthly calc_* functions (:137-341) and the daily calc_std_12 (:438-466).  Only
``tests/`` and ``bench.py``'s ``cpu_baseline`` leg may import it.

Pinning: ``tests/test_oracle_golden.py`` checks every function here against
``tests/golden/chars.npz``, produced by running the reference's own calc_* functions
(AST-extracted, numpy 1.26.4 / pandas 2.3.3) in ``tests/golden/gen_goldens.py:gen_chars``.

Semantics restated (pandas 2.x):
* ``groupby("permno").shift(k)`` is positional within the group, in frame order; with the
  rows stably grouped by permno, row i's lag-k value exists iff ids[i-k] == ids[i].
* ``groupby(..).rolling(w, min_periods=m)`` windows are the last w rows of the group;
  ``_prep_values`` turns +-inf into NaN; an observation is a non-NaN value; the result is NaN
  when fewer than m observations are in the window.  ``.sum()`` adds the observations
  (pandas: Kahan add/remove; the difference is rounding only).  ``.apply(np.prod, raw=True)``
  multiplies the raw window (NaN in it -> NaN).  ``.std()`` is ddof=1 and exactly 0 when every
  observation in the window is equal (pandas' consecutive-same-value rule).
"""
from __future__ import annotations

import numpy as np
import pandas as pd

FIELDS = ["me", "be", "retx", "accruals", "depreciation", "earnings", "assets", "dvc", "prc",
          "shrout", "total_debt", "sales"]
CHARS = ["log_size", "log_bm", "return_12_2", "accruals_final", "roa", "log_assets_growth",
         "dy", "log_return_13_36", "log_issues_12", "log_issues_36", "debt_price", "sales_price"]


def group_order(ids):
    """Stable grouping permutation (groupby keeps each group's rows in frame order)."""
    return np.argsort(np.asarray(ids), kind="stable")


def _lag(ids, x, k):
    """groupby(ids).shift(k) for rows already grouped (contiguous, in group order)."""
    n = len(x)
    out = np.full(n, np.nan)
    if k < n:
        same = ids[k:] == ids[:-k] if k > 0 else np.ones(n, bool)
        out[k:][same] = x[:-k][same]
    return out


def _windows(ids, x, w):
    """[n, w] matrix of the last w rows of each row's group (oldest first), NaN outside."""
    n = len(x)
    m = np.full((n, w), np.nan)
    for j in range(w):
        m[:, w - 1 - j] = _lag(ids, x, j) if j else x
    return m


def rolling_sum(ids, x, w, minp):
    """groupby(..).rolling(w, min_periods=minp).sum(), src/calc_Lewellen_2014.py:273-278, 302-306."""
    m = _windows(ids, np.where(np.isinf(x), np.nan, x), w)
    obs = ~np.isnan(m)
    s = np.where(obs, m, 0.0).sum(axis=1)
    return np.where(obs.sum(axis=1) >= minp, s, np.nan)


def rolling_prod(ids, x, w):
    """groupby(..).rolling(w, min_periods=w).apply(np.prod, raw=True), :180-186."""
    m = _windows(ids, np.where(np.isinf(x), np.nan, x), w)
    out = np.full(len(x), np.nan)
    ok = ~np.isnan(m).any(axis=1)
    if ok.any():
        acc = m[ok, 0].copy()
        for j in range(1, w):
            acc = acc * m[ok, j]
        out[ok] = acc
    return out


def firm_chars(ids, f):
    """All twelve monthly characteristics for rows grouped by firm (contiguous groups, frame
    order inside a group).  ``f`` maps FIELDS -> float64 arrays in that order."""
    with np.errstate(all="ignore"):
        me1 = _lag(ids, f["me"], 1)
        out = {}
        out["log_size"] = np.log(me1)                                          # :144-146
        out["log_bm"] = np.log(_lag(ids, f["be"], 1)) - np.log(me1)            # :156-159
        out["return_12_2"] = rolling_prod(ids, 1 + _lag(ids, f["retx"], 2), 11) - 1   # :173-190
        out["accruals_final"] = f["accruals"] - f["depreciation"]              # :203
        out["roa"] = f["earnings"] / f["assets"]                               # :248
        out["log_assets_growth"] = np.log(f["assets"] / _lag(ids, f["assets"], 12))   # :258-260
        out["dy"] = rolling_sum(ids, f["dvc"], 12, 1) / _lag(ids, f["prc"], 1)  # :273-284
        lr = np.log(1 + f["retx"])                                             # :298
        out["log_return_13_36"] = rolling_sum(ids, _lag(ids, lr, 13), 24, 24)  # :301-308
        sh1 = np.log(_lag(ids, f["shrout"], 1))
        out["log_issues_12"] = sh1 - np.log(_lag(ids, f["shrout"], 12))        # :230-235
        out["log_issues_36"] = sh1 - np.log(_lag(ids, f["shrout"], 36))        # :213-218
        out["debt_price"] = f["total_debt"] / me1                              # :321-323
        out["sales_price"] = f["sales"] / me1                                  # :335-337
    return out


def rolling_std(ids, x, w=252, minp=100, scale=np.sqrt(252)):
    """groupby(permno)["retx"].rolling(252, min_periods=100).std() * sqrt(252), :448-456,
    for rows grouped by firm.  Direct two-pass per window (pandas slides Welford/Kahan)."""
    n = len(x)
    v = np.where(np.isinf(x), np.nan, x)
    out = np.full(n, np.nan)
    start = 0
    for i in range(n):
        if i > 0 and ids[i] != ids[i - 1]:
            start = i
        a = v[max(start, i - w + 1):i + 1]
        a = a[~np.isnan(a)]
        if len(a) < max(minp, 2):
            continue
        if np.all(a == a[-1]):
            out[i] = 0.0
            continue
        mu = a.sum() / len(a)
        out[i] = np.sqrt(((a - mu) ** 2).sum() / (len(a) - 1)) * scale
    return out


def month_end(dates):
    """dt.to_period("M").dt.to_timestamp("M") as datetime64[ns] (:460)."""
    return pd.to_datetime(dates).to_period("M").to_timestamp("M").values.astype("datetime64[ns]")


def std_12_merge(d_permno, d_dates, d_std, m_permno, m_jdate):
    """drop_duplicates(["permno","jdate"], keep="last") over the daily frame in its order,
    then the left merge onto the monthly rows (:460-463): one value per monthly row."""
    jd = month_end(d_dates).astype(np.int64)
    last = {}
    for p, j, s in zip(np.asarray(d_permno), jd, np.asarray(d_std)):
        last[(int(p), int(j))] = s
    mj = np.asarray(m_jdate).astype("datetime64[ns]").astype(np.int64)
    return np.array([last.get((int(p), int(j)), np.nan) for p, j in zip(np.asarray(m_permno), mj)])


# ----------------------------------------------------------------------------------------
# calculate_rolling_beta (src/calc_Lewellen_2014.py:344-434) -- PARITY UNPINNED: the
# reference computes it with polars (pinned polars==1.22.0, requirements.txt:36), which is
# not installed here, so no golden from the reference exists.  Restated from the polars
# semantics the reference code relies on:
#   * inner join of the daily stock rows with the daily market index on the date (:375);
#     log_Ri = log(1 + Ri), log_Rm = log(1 + Rm) (:379-382); sorted by (permno, date);
#   * group_by_dynamic(index_column="date", every="1w", period="156w", by="permno") with
#     polars 1.x defaults: offset 0, closed="left", label="left", start_by="window": per
#     permno, windows [S, S + 156 weeks) for the Mondays S from the week of the first date
#     (dt.truncate("1w") = Monday) while S <= the last date; a window with no rows is not
#     emitted; the row's `date` is S (:393-401);
#   * sums of log_Ri, log_Rm, log_Ri * log_Rm, log_Rm ** 2 and the row count; polars float
#     sums propagate NaN (the pandas -> polars constructor keeps NaN as NaN, not null);
#     beta = (sum_RiRm - sum_Ri * sum_Rm / N) / (sum_Rm2 - sum_Rm ** 2 / N) (:402-416);
#   * jdate = month end of S; drop_duplicates(["permno", "jdate"], keep="last") -- the LAST
#     window starting in that month -- then a left merge onto crsp_comp (:426-431).
# ----------------------------------------------------------------------------------------
WEEK = 7


def week_start(days):
    """polars dt.truncate('1w') on day numbers since 1970-01-01 (a Thursday): Monday."""
    days = np.asarray(days, dtype=np.int64)
    return days - np.mod(days + 3, WEEK)


def rolling_beta_windows(permno, days, lri, lrm, period_weeks=156):
    """All emitted windows: (permno, window start day, beta).  Rows sorted by (permno, day)."""
    permno = np.asarray(permno)
    days = np.asarray(days, dtype=np.int64)
    out_p, out_s, out_b = [], [], []
    bounds = np.flatnonzero(np.r_[True, permno[1:] != permno[:-1], True])
    span = period_weeks * WEEK
    for a, b in zip(bounds[:-1], bounds[1:]):
        d = days[a:b]
        x, y = lri[a:b], lrm[a:b]
        S = int(week_start(d[:1])[0])
        while S <= d[-1]:
            i0 = np.searchsorted(d, S, side="left")
            i1 = np.searchsorted(d, S + span, side="left")
            if i1 > i0:
                xs, ys = x[i0:i1], y[i0:i1]
                n = float(i1 - i0)
                with np.errstate(invalid="ignore", divide="ignore", over="ignore"):
                    s_ri, s_rm = xs.sum(), ys.sum()
                    num = (xs * ys).sum() - s_ri * s_rm / n
                    den = (ys ** 2).sum() - s_rm ** 2 / n
                    out_b.append(num / den)
                out_p.append(permno[a])
                out_s.append(S)
            S += WEEK
    return np.array(out_p), np.array(out_s, dtype=np.int64), np.array(out_b, dtype=np.float64)


def calculate_rolling_beta(crsp_d, crsp_index_d, crsp_comp, period_weeks=156):
    """The reference's calculate_rolling_beta restated (see the block comment above)."""
    df = crsp_d[["permno", "dlycaldt", "retx"]].rename(columns={"retx": "Ri", "dlycaldt": "date"})
    mkt = crsp_index_d[["caldt", "vwretx"]].rename(columns={"vwretx": "Rm", "caldt": "date"})
    j = df.merge(mkt, on="date", how="inner")
    with np.errstate(invalid="ignore", divide="ignore"):
        j["lri"] = np.log(j["Ri"].to_numpy(dtype=np.float64) + 1.0)
        j["lrm"] = np.log(j["Rm"].to_numpy(dtype=np.float64) + 1.0)
    j = j.sort_values(["permno", "date"], kind="stable")
    days = j["date"].values.astype("datetime64[D]").astype(np.int64)
    p, s, b = rolling_beta_windows(j["permno"].to_numpy(), days, j["lri"].to_numpy(),
                                   j["lrm"].to_numpy(), period_weeks)
    beta = pd.DataFrame({"permno": p, "date": s.astype("datetime64[D]").astype("datetime64[ns]"), "beta": b})
    beta["jdate"] = beta["date"].dt.to_period("M").dt.to_timestamp("M")
    beta = beta.drop_duplicates(subset=["permno", "jdate"], keep="last")
    return pd.merge(left=crsp_comp, right=beta[["permno", "jdate", "beta"]], on=["permno", "jdate"], how="left")

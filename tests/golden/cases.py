"""Golden-case panel definitions shared by the generator and the tests.

This file defines *inputs* only (seeded synthetic panels plus deterministic edge-case
edits).  It must stay importable by the oracle interpreter used for golden generation
(/opt/conda/bin/python3.9, numpy 1.26.4, pandas 2.3.3) and by the product interpreter.
"""
from __future__ import annotations

import os
import sys

import numpy as np
import pandas as pd

_PKG = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "fm-returnprediction_amd")
if _PKG not in sys.path:
    sys.path.insert(0, _PKG)

from fmcore import synth  # noqa: E402

WINSOR_VARS = list(synth.WINSOR_VARS)

# Lewellen model definitions: src/calc_Lewellen_2014.py:714-745 (labels) mapped through the
# notebook's variables_dict (src/get_data.ipynb cell 24).
VARIABLES_DICT = {
    "Return (%)": "retx",
    "Log Size (-1)": "log_size",
    "Log B/M (-1)": "log_bm",
    "Return (-2, -12)": "return_12_2",
    "Log Issues (-1,-12)": "log_issues_12",
    "Accruals (-1)": "accruals_final",
    "ROA (-1)": "roa",
    "Log Assets Growth (-1)": "log_assets_growth",
    "Dividend Yield (-1,-12)": "dy",
    "Log Return (-13,-36)": "log_return_13_36",
    "Log Issues (-1,-36)": "log_issues_36",
    "Beta (-1,-36)": "beta",
    "Std Dev (-1,-12)": "rolling_std_252",
    "Debt/Price (-1)": "debt_price",
    "Sales/Price (-1)": "sales_price",
}
MODEL1 = ["log_size", "log_bm", "return_12_2"]
MODEL2 = MODEL1 + ["log_issues_36", "accruals_final", "roa", "log_assets_growth"]
MODEL3 = ["log_size", "log_bm", "return_12_2", "log_issues_12", "accruals_final", "roa",
          "log_assets_growth", "dy", "log_return_13_36", "log_issues_36", "beta",
          "rolling_std_252", "debt_price", "sales_price"]
FIG1_VARS = ["log_bm", "return_12_2", "log_issues_36", "accruals_final", "log_assets_growth"]
MODELS = {"M1": MODEL1, "M2": MODEL2, "M3": MODEL3}
SUBSETS = ["All stocks", "All-but-tiny stocks", "Large stocks"]


def _month_rows(df, k):
    months = np.sort(df["mthcaldt"].unique())
    return df.index[df["mthcaldt"] == months[k]]


def wins_panel():
    """Winsorize golden input: ragged months, ties, ±inf, ±0, <5 and ==5 valid values."""
    df = synth.synth_frame(20, 100, 101, nan_rate=0.05, present_rate=0.92)
    r = _month_rows(df, 2)
    df.loc[r[4:], "roa"] = np.nan                       # only 4 valid -> unchanged
    r = _month_rows(df, 4)
    df.loc[r[: int(0.6 * len(r))], "beta"] = 1.0          # heavy ties
    r = _month_rows(df, 6)
    df.loc[r[[0, 5]], "debt_price"] = np.inf
    df.loc[r[[1, 9]], "debt_price"] = -np.inf
    r = _month_rows(df, 7)
    df.loc[r[:3], "sales_price"] = np.inf                # 3 inf at top -> hi cut from inf
    r = _month_rows(df, 8)
    df.loc[r[::3], "log_bm"] = 0.0
    df.loc[r[1::3], "log_bm"] = -0.0
    r = _month_rows(df, 10)
    df.loc[r[5:], "accruals_final"] = np.nan             # exactly 5 valid
    r = _month_rows(df, 12)
    df.loc[r, "dy"] = np.nan                             # all NaN
    # scramble row order and give a non-default index: winsorize must sort and keep labels
    rng = np.random.default_rng(7)
    df = df.iloc[rng.permutation(len(df))]
    df.index = pd.Index(rng.permutation(len(df)) * 3 + 1000)
    return df


def fm_panel():
    """FM golden input (clean of inf): 30 months, NYSE edge months, small Large subsets."""
    df = synth.synth_frame(30, 150, 202, nan_rate=0.03, present_rate=0.95)
    r = _month_rows(df, 3)
    df.loc[r, "primaryexch"] = "Q"                       # no NYSE -> ABT/Large empty
    r = _month_rows(df, 5)
    df.loc[r, "primaryexch"] = "Q"
    df.loc[r[10], "primaryexch"] = "N"                   # exactly one NYSE firm
    r = _month_rows(df, 9)
    nyse = df.loc[r, "primaryexch"] == "N"
    # make month 9 NYSE me huge so Large has few firms (< K+1 for Model 3)
    big = r[nyse.values]
    df.loc[big, "me"] = df.loc[big, "me"] * 0.0 + 1e9
    df.loc[big[:10], "me"] = 1.0
    rng = np.random.default_rng(11)
    df = df.iloc[rng.permutation(len(df))].reset_index(drop=True)
    return df


def fig1_panel():
    return synth.synth_frame(150, 60, 303, nan_rate=0.02, present_rate=0.97)


def fig1_const_panel():
    """fig1_panel with Figure-1 regressors constant within a month (has_constant='add': the
    pinv splits the intercept over [1, c1, c2], reference src/calc_Lewellen_2014.py:913-921)
    -- one month with one nonzero constant, one with two."""
    df = fig1_panel()
    m = np.sort(df.mthcaldt.unique())
    df.loc[df.mthcaldt == m[40], FIG1_VARS[1]] = 0.8
    df.loc[df.mthcaldt == m[100], FIG1_VARS[0]] = -0.3
    df.loc[df.mthcaldt == m[100], FIG1_VARS[2]] = 1.7
    return df


def mid_panel():
    return synth.synth_frame(600, 500, 404, nan_rate=0.02, present_rate=0.97)


def _edge_base(T, n, K, seed):
    rng = np.random.default_rng(seed)
    months = pd.date_range("2000-01-31", periods=T, freq=pd.offsets.MonthEnd())
    rows = []
    for t, m in enumerate(months):
        x = rng.standard_normal((n, K))
        y = 0.01 + x @ np.linspace(0.1, -0.1, K) + rng.standard_normal(n)
        d = {"mthcaldt": [m] * n, "retx": y}
        for k in range(K):
            d[f"x{k}"] = x[:, k]
        rows.append(pd.DataFrame(d))
    return pd.concat(rows, ignore_index=True)


def edge_cases():
    """(name, df, predictor_cols) regression edge cases; see SURVEY.md §8 quirks table."""
    out = []
    K = 3
    xs = [f"x{k}" for k in range(K)]
    df = _edge_base(14, 12, K, 1)
    m = np.sort(df.mthcaldt.unique())
    df = df[~((df.mthcaldt == m[2]) & (df.index % 12 >= K + 1))]   # N == K+1
    df = df[~((df.mthcaldt == m[4]) & (df.index % 12 >= K))]       # N == K  -> skipped
    df.loc[(df.mthcaldt == m[6]) & (df.index % 12 < 5), "retx"] = np.nan  # dropna on y
    df.loc[(df.mthcaldt == m[7]), "x1"] = np.nan                   # whole month dropped
    out.append(("n_edges", df.reset_index(drop=True), xs))
    df = _edge_base(12, 15, K, 2)
    df["x1"] = 0.0
    out.append(("zero_col", df, xs))
    df = _edge_base(12, 15, K, 3)
    df["x2"] = 2.0 * df["x1"]
    out.append(("collinear", df, xs))
    df = _edge_base(8, 15, K, 4)
    out.append(("few_months", df, xs))
    df = _edge_base(12, 15, K, 5)
    df.loc[20, "retx"] = np.inf
    out.append(("inf_y", df, xs))
    df = _edge_base(12, 15, K, 6)
    df.loc[33, "x0"] = np.inf
    out.append(("inf_x", df, xs))
    df = _edge_base(12, 15, K, 7)
    m = np.sort(df.mthcaldt.unique())
    df.loc[df.mthcaldt == m[3], "x2"] = 1.5
    out.append(("const_col", df, xs))
    df = _edge_base(12, 15, K, 8)
    m = np.sort(df.mthcaldt.unique())
    df.loc[df.mthcaldt == m[3], "x2"] = 0.0                          # zero (not nonzero const)
    out.append(("zero_in_month", df, xs))
    df = _edge_base(15, 40, 1, 9)
    out.append(("k1", df, ["x0"]))
    df = _edge_base(12, 60, 15, 10)
    out.append(("k15", df, [f"x{k}" for k in range(15)]))
    return out


def divergence_cases():
    """Rank-deficiency cases beyond edge_cases (DESIGN.md §2 'Known divergences'): an affine
    dependence x2 = 2 x1 + 0.5 (the pinv null space involves the intercept) in every month,
    and a near-collinear pair x2 = x1 + 1e-7 noise (sigma_min / sigma_max ~ 1e-7)."""
    out = []
    K = 3
    xs = [f"x{k}" for k in range(K)]
    df = _edge_base(12, 15, K, 21)
    df["x2"] = 2.0 * df["x1"] + 0.5
    out.append(("affine_collinear", df, xs))
    df = _edge_base(12, 40, K, 22)
    rng = np.random.default_rng(23)
    df["x2"] = df["x1"] + 1e-7 * rng.standard_normal(len(df))
    out.append(("near_collinear", df, xs))
    return out


def nw_series():
    rng = np.random.default_rng(12)
    out = []
    for T in (0, 1, 2, 3, 4, 5, 6, 11, 50, 600):
        out.append(rng.standard_normal(T) * 0.3 + 0.05)
    out.append(np.full(20, 0.25))
    return out


def percentile_arrays():
    rng = np.random.default_rng(13)
    arrs = []
    for i in range(600):
        n = int(rng.integers(1, 250))
        kind = i % 6
        if kind == 0:
            v = rng.standard_normal(n)
        elif kind == 1:
            v = rng.standard_t(2, n) * 100
        elif kind == 2:
            v = rng.integers(-3, 4, n).astype(float)            # heavy ties
        elif kind == 3:
            v = rng.standard_normal(n)
            v[rng.random(n) < 0.3] = 0.0
            v[rng.random(n) < 0.2] = -0.0
        elif kind == 4:
            v = rng.standard_normal(n) * 1e-300                  # subnormal-ish range
        else:
            v = rng.standard_normal(n)
            v[rng.random(n) < 0.03] = np.inf
            v[rng.random(n) < 0.03] = -np.inf
        arrs.append(v)
    return arrs


# ------------------------------------------------------------------------------------------
# Firm-axis characteristic construction: raw monthly CRSP/Compustat
# fields and daily returns, before get_factors (src/calc_Lewellen_2014.py:531-575).
# ------------------------------------------------------------------------------------------
RAW_FIELDS = ["me", "be", "retx", "accruals", "depreciation", "earnings", "assets", "dvc", "prc",
              "shrout", "total_debt", "sales"]
CHAR_NAMES = ["log_size", "log_bm", "return_12_2", "accruals_final", "roa", "log_assets_growth",
              "dy", "log_return_13_36", "log_issues_12", "log_issues_36", "debt_price", "sales_price"]


def raw_monthly_panel(nfirms=70, nmonths=60, seed=21, shuffle=True):
    """Ragged firm histories (1..60 rows, random starts, 5% dropped months), NaNs, zeros,
    negatives and infinities in the fields the characteristics take logs / ratios of."""
    rng = np.random.default_rng(seed)
    months = pd.date_range("2001-01-31", periods=nmonths, freq=pd.offsets.MonthEnd())
    parts = []
    for f in range(nfirms):
        start = int(rng.integers(0, nmonths))
        length = int(rng.integers(1, nmonths - start + 1))
        if f % 7 == 0:
            start, length = 0, nmonths                      # long histories (all windows fill)
        idx = np.arange(start, start + length)
        idx = idx[rng.random(len(idx)) > 0.05] if len(idx) > 3 else idx
        n = len(idx)
        if n == 0:
            continue
        d = {"permno": np.full(n, 10000 + 7 * f, dtype=np.int64), "mthcaldt": months[idx]}
        d["me"] = np.exp(rng.normal(5, 2, n))
        d["be"] = d["me"] * np.exp(rng.normal(-0.5, 0.8, n))
        d["retx"] = rng.standard_t(4, n) * 0.08
        d["accruals"] = rng.normal(0.0, 0.05, n)
        d["depreciation"] = np.abs(rng.normal(0.03, 0.01, n))
        d["earnings"] = rng.normal(0.02, 0.1, n) * 100
        d["assets"] = np.exp(rng.normal(6, 1.5, n))
        d["dvc"] = np.where(rng.random(n) < 0.7, 0.0, np.abs(rng.normal(0.5, 0.3, n)))
        d["prc"] = np.exp(rng.normal(3, 1, n)) * np.where(rng.random(n) < 0.05, -1.0, 1.0)
        d["shrout"] = np.exp(rng.normal(9, 1, n)) * np.exp(np.cumsum(rng.normal(0, 0.01, n)))
        d["total_debt"] = np.abs(rng.normal(100, 60, n))
        d["sales"] = np.abs(rng.normal(300, 200, n))
        for k in RAW_FIELDS:
            d[k][rng.random(n) < 0.03] = np.nan
        parts.append(pd.DataFrame(d))
    df = pd.concat(parts, ignore_index=True)
    # edge values: log(0) = -inf, log(<0) = NaN, 1 + retx = 0, +-inf returns and fields
    df.loc[df.index[5], "me"] = 0.0
    df.loc[df.index[40], "be"] = -3.0
    long_rows = df.index[df["permno"] == 10000]
    df.loc[long_rows[20], "retx"] = -1.0
    df.loc[long_rows[45], "retx"] = np.inf
    long2 = df.index[df["permno"] == 10000 + 7 * 7]
    df.loc[long2[30], "dvc"] = np.inf
    df.loc[long2[10:14], "dvc"] = np.nan                   # dy over an all-NaN stretch
    df.loc[long2[33], "shrout"] = -np.inf
    df.loc[long2[50], "assets"] = 0.0
    df["jdate"] = df["mthcaldt"]
    if shuffle:
        df = df.iloc[rng.permutation(len(df))]
        df.index = pd.Index(rng.permutation(len(df)) * 2 + 500)
    return df


def raw_daily_panel(nfirms=14, ndays=700, seed=22, shuffle=True):
    """Daily returns for calc_std_12 (src/calc_Lewellen_2014.py:438-466): ragged histories
    (some shorter than the 100-day minimum), NaN stretches, infinities and a long run of one
    repeated value (pandas reports an exact 0 std there)."""
    rng = np.random.default_rng(seed)
    days = pd.bdate_range("2001-01-02", periods=ndays)
    parts = []
    for f in range(nfirms):
        start = 0 if f % 3 == 0 else int(rng.integers(0, ndays - 50))
        length = ndays - start if f % 3 == 0 else int(rng.integers(50, ndays - start + 1))
        idx = np.arange(start, start + length)
        n = len(idx)
        r = rng.normal(0.0005, 0.02, n)
        r[rng.random(n) < 0.02] = np.nan
        if f == 0:
            r[300:420] = 0.0                               # 120 equal values
            r[100:130] = np.nan
        if f == 3:
            r[200] = np.inf
            r[450] = -np.inf
        parts.append(pd.DataFrame({"permno": np.full(n, 10000 + 7 * f, dtype=np.int64),
                                   "dlycaldt": days[idx], "retx": r}))
    df = pd.concat(parts, ignore_index=True)
    if shuffle:
        df = df.iloc[rng.permutation(len(df))]
        df.index = pd.Index(rng.permutation(len(df)) + 10)
    return df

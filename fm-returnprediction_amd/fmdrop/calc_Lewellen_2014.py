"""Drop-in replacement for the hot-path functions of the reference's
src/calc_Lewellen_2014.py, on MI355X.

Mirrored (same names, signatures, return types and row/column/index order):
  winsorize        reference :505-529   per-month 1/99 cuts (fm_select_cuts) + clip (fm_clip)
  get_subsets      reference :44-112    NYSE me breakpoints (fm_select_cuts, pandas lerp)
  build_table_1    reference :577-670   monthly moments + distinct permnos on device (§8(f) row 1)
  build_table_2    reference :674-868   9 FM passes batched into one Gram pass on device
  create_figure_1  reference :871-957   F1 OLS + 120-month rolling means on device
Extensions the north star names (not in the reference; parity unpinned):
  standardize, monthly_coefficients, rolling_coefficients, expected_return_forecasts,
  predictive_slope_regressions, lewellen_pipeline.
Firm-axis characteristic builders (§8(f) row 2; one fused device pass, fm_firm_chars):
  calc_log_size, calc_log_bm, calc_return_12_2, calc_accruals, calc_roa,
  calc_log_assets_growth, calc_dy, calc_log_return_13_36, calc_log_issues_12,
  calc_log_issues_36, calc_debt_price, calc_sales_price   reference :137-341
  calc_std_12      reference :438-466   252-day rolling std on device (fm_rolling_std)
  calc_characteristics (extension): all twelve monthly characteristics in one launch.
  calculate_rolling_beta reference :344-434  polars 156-week weekly-window beta on device
                   (fm_rolling_beta; parity unpinned: no polars here)
Data pulls and LaTeX output of the reference are outside this drop-in (scope).
"""
import os
from pathlib import Path
from typing import Union

import numpy as np
import pandas as pd

from fmcore import _lib as _L
from fmcore import api as _api
from fmcore import engine as _E
from fmcore import lewellen as _LW

from .regressions import fama_macbeth_summary, run_monthly_cs_regressions  # noqa: F401

OUTPUT_DIR = Path(os.environ.get("OUTPUT_DIR", "_output"))


# ------------------------------------------------------------------------------------------
# Universes
# ------------------------------------------------------------------------------------------
def _nyse_cuts(df):
    """me_20/me_50 per month (device) for a frame already sorted by [mthcaldt, permno]."""
    me = _api.as_f64(df["me"])
    nyse = (df["primaryexch"] == "N").to_numpy().astype(np.uint8)
    panel = _E.panel_from_arrays([me], ["me"], df["mthcaldt"].values, me=me, nyse=nyse)
    a, b, level = _E.universe(panel)
    return panel, a.cpu().numpy(), b.cpu().numpy(), level.cpu().numpy()


def get_subsets(crsp_comp: pd.DataFrame) -> dict:
    """All / All-but-tiny / Large universes from NYSE 20th and 50th `me` percentiles per
    month (reference src/calc_Lewellen_2014.py:44-112).  Returns the same 3-key dict; the
    frames carry me_20, me_50, is_all_but_tiny, is_large and a fresh RangeIndex."""
    df = crsp_comp.sort_values(["mthcaldt", "permno"]).copy()
    panel, me20, me50, level = _nyse_cuts(df)
    codes, _ = pd.factorize(df["mthcaldt"], sort=True)
    codes = np.asarray(codes)
    valid = codes >= 0
    # NYSE-less months (or all-NaN NYSE me) carry NaN breakpoints, as after the left merge
    row20 = np.full(len(df), np.nan)
    row50 = np.full(len(df), np.nan)
    row20[valid] = me20[codes[valid]]
    row50[valid] = me50[codes[valid]]
    out = df.reset_index(drop=True)
    out["me_20"] = row20
    out["me_50"] = row50
    lvl = np.zeros(len(df), dtype=np.uint8)
    lvl[panel.order] = level
    out["is_all_but_tiny"] = lvl >= 1
    out["is_large"] = lvl >= 2
    return {
        "All stocks": out.copy(),
        "All-but-tiny stocks": out.loc[out["is_all_but_tiny"]].copy(),
        "Large stocks": out.loc[out["is_large"]].copy(),
    }


# ------------------------------------------------------------------------------------------
# Winsorize / standardize
# ------------------------------------------------------------------------------------------
def _split_runs(varlist):
    runs, cur = [], []
    for v in varlist:
        if v in cur:
            runs.append(cur)
            cur = []
        cur.append(v)
    if cur:
        runs.append(cur)
    return runs


def winsorize(crsp_comp: pd.DataFrame, varlist: list, lower_percentile=1, upper_percentile=99) -> pd.DataFrame:
    """Clip each variable at its per-month [lower, upper] linear percentiles, months with
    fewer than 5 non-NaN values untouched (reference src/calc_Lewellen_2014.py:505-529).
    Returns the frame sorted by [mthcaldt, permno] with the original index labels."""
    df = crsp_comp.sort_values(["mthcaldt", "permno"]).copy()
    varlist = list(varlist)
    if not varlist:
        return df
    codes, _ = pd.factorize(df["mthcaldt"], sort=True)
    if (np.asarray(codes) < 0).any():
        df = df.loc[np.asarray(codes) >= 0]       # groupby(...).apply drops NaT months
    for run in _split_runs(varlist):
        arrays = [_api.as_f64(df[v]) for v in run]
        panel = _E.panel_from_arrays(arrays, run, df["mthcaldt"].values)
        cuts = _E.select_cuts(panel, lower_percentile / 100, upper_percentile / 100, 5, _E.LERP_NUMPY)
        out = _E.clip(panel, cuts).cpu().numpy()
        inv = np.empty_like(panel.order)
        inv[panel.order] = np.arange(len(panel.order))
        for i, v in enumerate(run):
            df[v] = out[i][inv]
    return df


def standardize(crsp_comp: pd.DataFrame, varlist: list, date_col: str = "mthcaldt") -> pd.DataFrame:
    """Per-month z-scores (x - mean_t) / std_t(ddof=1) over non-NaN values (north-star
    extension A9; the reference has no standardization, so this is OFF on parity paths)."""
    df = crsp_comp.copy()
    varlist = list(varlist)
    arrays = [_api.as_f64(df[v]) for v in varlist]
    panel = _E.panel_from_arrays(arrays, varlist, df[date_col].values)
    mom = _E.select_cuts(panel, 0.0, 1.0, 2 ** 31 - 1, _E.LERP_NUMPY, moments=True)
    z = _E.standardize(panel, mom.mean, mom.sd).cpu().numpy()
    for i, v in enumerate(varlist):
        col = np.full(len(df), np.nan)
        col[panel.order] = z[i]
        df[v] = col
    return df


# ------------------------------------------------------------------------------------------
# Firm-axis characteristics (reference :137-466)
# ------------------------------------------------------------------------------------------
def _firm_grouping(permno):
    """groupby("permno") row order: each firm's rows contiguous, frame order inside a firm
    (a stable sort by permno; None when the frame is already grouped that way).  pandas'
    groupby drops rows whose permno is missing; such rows are rejected here rather than
    read as a garbage id."""
    p = np.asarray(permno)
    if p.dtype.kind == "f":
        if np.isnan(p).any():
            raise ValueError("permno contains NaN: drop those rows first (groupby would drop them)")
    elif p.dtype.kind not in "iu":
        p = pd.to_numeric(pd.Series(p), errors="raise").to_numpy()
        if np.isnan(p.astype(np.float64)).any():
            raise ValueError("permno contains missing values")
    ids = p.astype(np.int64)
    if len(ids) < 2 or bool(np.all(ids[1:] >= ids[:-1])):
        return ids, None
    order = np.argsort(ids, kind="stable")
    return ids[order], order


def _device_chars(df, names):
    """{name: float64 ndarray in df's row order} for the requested characteristics."""
    import torch
    dev = _E.require_device()
    ids, order = _firm_grouping(df["permno"].to_numpy())
    reads = set()
    for nm in names:
        reads |= _CHAR_READS[nm]
    fields = {}
    for f in reads:
        v = _api.as_f64(df[f])
        fields[f] = torch.from_numpy(np.ascontiguousarray(v if order is None else v[order])).to(dev)
    out = _E.firm_chars(torch.from_numpy(ids).to(dev), fields, names)
    res = {}
    for nm in names:
        v = out[nm].cpu().numpy()
        if order is not None:
            u = np.empty_like(v)
            u[order] = v
            v = u
        res[nm] = v
    return res


_CHAR_READS = {
    "log_size": {"me"}, "log_bm": {"me", "be"}, "return_12_2": {"retx"},
    "accruals_final": {"accruals", "depreciation"}, "roa": {"earnings", "assets"},
    "log_assets_growth": {"assets"}, "dy": {"dvc", "prc"}, "log_return_13_36": {"retx"},
    "log_issues_12": {"shrout"}, "log_issues_36": {"shrout"}, "debt_price": {"me", "total_debt"},
    "sales_price": {"me", "sales"},
}


def _add_char(crsp_comp, name):
    crsp_comp[name] = _device_chars(crsp_comp, [name])[name]
    return crsp_comp


def calc_log_size(crsp_comp: pd.DataFrame) -> pd.DataFrame:
    """log(me) of the firm's previous row (reference :137-147)."""
    return _add_char(crsp_comp, "log_size")


def calc_log_bm(crsp_comp: pd.DataFrame) -> pd.DataFrame:
    """log(be[t-1]) - log(me[t-1]) (reference :150-163)."""
    return _add_char(crsp_comp, "log_bm")


def calc_return_12_2(crsp_comp: pd.DataFrame) -> pd.DataFrame:
    """prod(1 + retx) over the firm's rows t-12..t-2, all 11 present, minus 1 (:166-192)."""
    return _add_char(crsp_comp, "return_12_2")


def calc_accruals(crsp_comp: pd.DataFrame) -> pd.DataFrame:
    """accruals - depreciation (reference :195-204)."""
    return _add_char(crsp_comp, "accruals_final")


def calc_roa(crsp_comp: pd.DataFrame) -> pd.DataFrame:
    """earnings / assets (reference :241-249)."""
    return _add_char(crsp_comp, "roa")


def calc_log_assets_growth(crsp_comp: pd.DataFrame) -> pd.DataFrame:
    """log(assets / assets twelve firm rows back) (reference :252-262)."""
    return _add_char(crsp_comp, "log_assets_growth")


def calc_dy(crsp_comp: pd.DataFrame) -> pd.DataFrame:
    """Sum of dvc over the firm's last 12 rows (min_periods=1) / prc[t-1], on a copy sorted by
    [permno, mthcaldt], which is returned (reference :265-287)."""
    df = crsp_comp.sort_values(["permno", "mthcaldt"]).copy()
    return _add_char(df, "dy")


def calc_log_return_13_36(crsp_comp: pd.DataFrame) -> pd.DataFrame:
    """Sum of log(1 + retx) over the firm's rows t-36..t-13, all 24 present (:290-313)."""
    return _add_char(crsp_comp, "log_return_13_36")


def calc_log_issues_12(crsp_comp: pd.DataFrame) -> pd.DataFrame:
    """log(shrout[t-1]) - log(shrout[t-12]) (reference :224-238)."""
    return _add_char(crsp_comp, "log_issues_12")


def calc_log_issues_36(crsp_comp: pd.DataFrame) -> pd.DataFrame:
    """log(shrout[t-1]) - log(shrout[t-36]) (reference :207-221)."""
    return _add_char(crsp_comp, "log_issues_36")


def calc_debt_price(crsp_comp: pd.DataFrame) -> pd.DataFrame:
    """total_debt / me[t-1] (reference :316-327)."""
    return _add_char(crsp_comp, "debt_price")


def calc_sales_price(crsp_comp: pd.DataFrame) -> pd.DataFrame:
    """sales / me[t-1] (reference :330-341)."""
    return _add_char(crsp_comp, "sales_price")


def calc_characteristics(crsp_comp: pd.DataFrame, names=None) -> pd.DataFrame:
    """Extension: the twelve monthly characteristics in get_factors order (reference
    :537-547) from ONE device pass; same values as calling the calc_* one by one on a frame
    sorted by [permno, mthcaldt] (calc_dy's re-sort is then a no-op)."""
    names = list(_E.CHAR_NAMES if names is None else names)
    out = _device_chars(crsp_comp, names)
    for nm in names:
        crsp_comp[nm] = out[nm]
    return crsp_comp


def calculate_rolling_beta(crsp_d: pd.DataFrame, crsp_index_d: pd.DataFrame,
                           crsp_comp: pd.DataFrame) -> pd.DataFrame:
    """156-week rolling market beta from daily log returns, merged onto crsp_comp as `beta`
    (reference src/calc_Lewellen_2014.py:344-434).  The reference's polars
    group_by_dynamic(every="1w", period="156w", by="permno") windows, sums and beta formula
    run on device (fm_rolling_beta); the inner join on the date, the (permno, date) sort
    and the final left merge on (permno, jdate) are the reference's pandas steps.  Parity
    unpinned: polars is not installed here (oracle/chars_oracle.py restates its semantics)."""
    import torch
    dev = _E.require_device()
    df = crsp_d[["permno", "dlycaldt", "retx"]].rename(columns={"retx": "Ri", "dlycaldt": "date"})
    mkt = crsp_index_d[["caldt", "vwretx"]].rename(columns={"vwretx": "Rm", "caldt": "date"})
    j = df.merge(mkt, on="date", how="inner").sort_values(["permno", "date"], kind="stable")
    permno = j["permno"].to_numpy()
    days = j["date"].values.astype("datetime64[D]").astype(np.int64)
    if len(days) and (days.min() < -(2 ** 31) or days.max() >= 2 ** 31):
        raise ValueError("calculate_rolling_beta: dates out of range")
    starts = np.flatnonzero(np.r_[True, permno[1:] != permno[:-1]]) if len(permno) else np.zeros(0, np.int64)
    seg_off = np.r_[starts, len(permno)].astype(np.int64)
    uperm = permno[starts]
    keys = crsp_comp[["permno", "jdate"]].drop_duplicates()
    kp = keys["permno"].to_numpy()
    pos = np.searchsorted(uperm, kp) if len(uperm) else np.zeros(len(kp), dtype=np.int64)
    ok = pos < len(uperm)
    ok[ok] = uperm[pos[ok]] == kp[ok]
    kq = keys.loc[ok]
    per = pd.to_datetime(kq["jdate"]).dt.to_period("M")
    d0 = per.dt.start_time.values.astype("datetime64[D]").astype(np.int64)
    d1 = per.dt.end_time.values.astype("datetime64[D]").astype(np.int64)
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a, dtype=dt)).to(dev)  # noqa: E731
    beta = _E.rolling_beta(t(days, np.int32), t(j["Ri"].to_numpy(dtype=np.float64), np.float64),
                           t(j["Rm"].to_numpy(dtype=np.float64), np.float64), t(seg_off, np.int64),
                           t(pos[ok], np.int32), t(d0, np.int32), t(d1, np.int32)).cpu().numpy()
    # a (permno, month) without an emitted window is NaN after the merge either way
    right = kq.assign(beta=beta)
    return pd.merge(left=crsp_comp, right=right[["permno", "jdate", "beta"]], on=["permno", "jdate"], how="left")


def calc_std_12(crsp_d: pd.DataFrame, crsp_comp: pd.DataFrame) -> pd.DataFrame:
    """Annualized 252-day rolling std of daily retx per permno (min_periods=100), the last
    day of each (permno, month), left-merged onto crsp_comp on [permno, jdate]
    (reference :438-466).  The rolling std runs on device; the month-end pick and the merge
    are the reference's pandas steps."""
    import torch
    dev = _E.require_device()
    df_std_12 = crsp_d.copy()
    ids, order = _firm_grouping(df_std_12["permno"].to_numpy())
    x = _api.as_f64(df_std_12["retx"])
    xs = torch.from_numpy(np.ascontiguousarray(x if order is None else x[order])).to(dev)
    sd = _E.rolling_std(torch.from_numpy(ids).to(dev), xs, 252, 100, float(np.sqrt(252))).cpu().numpy()
    if order is not None:
        u = np.empty_like(sd)
        u[order] = sd
        sd = u
    df_std_12["rolling_std_252"] = sd
    df_std_12["jdate"] = df_std_12["dlycaldt"].dt.to_period("M").dt.to_timestamp("M")
    df_std_12.drop_duplicates(subset=["permno", "jdate"], keep="last", inplace=True)
    return pd.merge(left=crsp_comp, right=df_std_12[["permno", "jdate", "rolling_std_252"]],
                    on=["permno", "jdate"], how="left")


# ------------------------------------------------------------------------------------------
# Table 1
# ------------------------------------------------------------------------------------------
def build_table_1(subsets_crsp_comp: dict, variables_dict: dict) -> pd.DataFrame:
    """Lewellen Table 1: per universe and variable, the time-series averages of the monthly
    cross-sectional mean and std (ddof=1) after inf->NaN and dropna, and the number of
    distinct permnos (reference src/calc_Lewellen_2014.py:577-670)."""
    import torch
    partial = []
    for subset_name, df_subset in subsets_crsp_comp.items():
        present = list(dict.fromkeys(c for c in variables_dict.values() if c in df_subset.columns))
        stats = {}
        if present:
            arrays = [_api.as_f64(df_subset[c]) for c in present]
            panel = _E.panel_from_arrays(arrays, present, df_subset["mthcaldt"].values)
            cnt, mean, sd = _E.segment_moments(panel, finite_only=True)
            T = panel.nseg
            C = len(present)
            vals = torch.cat([mean, sd], dim=0).t().contiguous()           # [T, 2C]
            if T:
                am, _, _, an = _api.records_summary_device(vals, nw_lags=0)
            else:
                am, an = np.full(2 * C, np.nan), np.zeros(2 * C, dtype=np.int64)
            dev = panel.device
            allv = torch.from_numpy(np.stack(arrays)).to(dev)                # every row, NaT months too
            ids = torch.from_numpy(df_subset["permno"].to_numpy(dtype=np.int64)).to(dev)
            nuniq = _E.distinct_count(ids, allv, finite_only=True).cpu().numpy()
            tot = cnt.sum(dim=1).cpu().numpy()
            for i, c in enumerate(present):
                stats[c] = (tot[i], am[i] if an[i] else np.nan, am[C + i] if an[C + i] else np.nan,
                            int(nuniq[i]))
        rows = []
        for var_label, var_col in variables_dict.items():
            st = stats.get(var_col)
            if st is None or (st[0] == 0 and st[3] == 0):
                rows.append({"Column": var_label, "Avg": np.nan, "Std": np.nan, "N": np.nan})
            else:
                rows.append({"Column": var_label, "Avg": st[1], "Std": st[2], "N": st[3]})
        part = pd.DataFrame(rows).set_index("Column")
        part.columns = pd.MultiIndex.from_product([[subset_name], part.columns])
        partial.append(part)
    return pd.concat(partial, axis=1)


# ------------------------------------------------------------------------------------------
# Table 2
# ------------------------------------------------------------------------------------------
def _batched_subsets(subsets):
    """If the dict is get_subsets' output, all 9 passes run as one levelled pass on the
    All-stocks frame; returns (frame, level) or None."""
    if not all(k in subsets for k in _LW.SUBSET_NAMES):
        return None
    a = subsets["All stocks"]
    if not {"is_all_but_tiny", "is_large"} <= set(a.columns):
        return None
    abt = a["is_all_but_tiny"].to_numpy(dtype=bool)
    lg = a["is_large"].to_numpy(dtype=bool)
    if (lg & ~abt).any():
        return None
    if len(subsets["All-but-tiny stocks"]) != abt.sum() or len(subsets["Large stocks"]) != lg.sum():
        return None
    return a, abt.astype(np.uint8) + lg.astype(np.uint8)


def _fm_summaries(df, model_cols, level=None, nlevels=1, fig1=False, moments=False):
    """Device FM pass of several models over one frame (optionally levelled)."""
    cols = []
    for xs in model_cols.values():
        for c in ["retx"] + list(xs):
            if c not in cols:
                cols.append(c)
    if fig1:
        for c in _LW.FIG1_VARS:
            if c not in cols:
                cols.append(c)
    arrays = [_api.as_f64(df[c]) for c in cols]
    panel = _E.panel_from_arrays(arrays, cols, df["mthcaldt"].values)
    lvl_t = None
    if level is not None:
        import torch
        lvl_t = torch.from_numpy(np.ascontiguousarray(level[panel.order])).to(panel.device)
    levels = tuple(range(nlevels))
    models = [_E.Model(n, y=panel.col("retx"), xs=[panel.col(c) for c in xs], levels=levels)
              for n, xs in model_cols.items()]
    res = _E.fm_pass(panel, models, level=lvl_t, nlevels=nlevels, moments=moments)
    return panel, models, res


def _summary_series(res, k, xs, status_h, rec_h, summ_h):
    mean, se, t, nobs = summ_h
    return _api.summary_from_device(mean[k], se[k], t[k], nobs[k], xs, k_slope0=1, k_r2=res.pmax,
                                    k_n=res.pmax + 1)


def _check_errors(res, status_h, models):
    for k, p in enumerate(res.problems):
        _api.raise_like_reference(status_h[:, k], p.K)


def _format_table_2(stats, subset_names):
    """Table-2 layout of the reference (src/calc_Lewellen_2014.py:797-866): rows
    (Model, Predictor) with a trailing N row per model; columns (subset, Slope/t-stat/R^2);
    3-decimal strings, R^2 only on each model's first row, N with thousands separators."""
    subset_order = ["All stocks", "All-but-tiny stocks", "Large stocks"]
    metrics = ["Slope", "t-stat", "R^2"]
    present = [s for s in subset_order if s in subset_names]
    rows, index = [], []
    for model, labels in _LW.MODELS_PREDICTORS.items():
        for r, lbl in enumerate(labels + ["N"]):
            index.append((model, lbl))
            row = []
            for s in present:
                st = stats.get((model, s))
                for mtr in metrics:
                    v = np.nan
                    if st is not None:
                        if lbl == "N":
                            v = st["mean_N"] if mtr == "Slope" else np.nan
                        elif mtr == "Slope":
                            v = st["coef"][r]
                        elif mtr == "t-stat":
                            v = st["tstat"][r]
                        elif r == 0:
                            v = st["mean_R2"]
                    if v is None or (isinstance(v, float) and np.isnan(v)):
                        row.append("")
                    elif lbl == "N":
                        row.append(f"{int(round(float(v))):,.0f}")
                    else:
                        row.append(f"{float(v):.3f}")
            rows.append(row)
    cols = pd.MultiIndex.from_tuples([(s, m) for s in present for m in metrics], names=[None, None])
    idx = pd.MultiIndex.from_tuples(index, names=["Model", "Predictor"])
    return pd.DataFrame(rows, index=idx, columns=cols, dtype=object)


def build_table_2(subsets_comp_crsp: dict, variables_dict: dict) -> pd.DataFrame:
    """Lewellen Table 2: Fama-MacBeth slopes, NW(4) t-stats, mean R^2 and mean N for
    Models 1-3 on each universe (reference src/calc_Lewellen_2014.py:674-868)."""
    model_cols = _LW.table2_models(variables_dict)
    stats = {}
    batched = _batched_subsets(subsets_comp_crsp)
    jobs = []
    if batched is not None:
        frame, level = batched
        jobs.append((frame, level, 3, {i: s for i, s in enumerate(_LW.SUBSET_NAMES)}))
    else:
        for s, frame in subsets_comp_crsp.items():
            jobs.append((frame, None, 1, {0: s}))
    for frame, level, nlevels, level_names in jobs:
        panel, models, res = _fm_summaries(frame, model_cols, level, nlevels)
        status_h = res.status.cpu().numpy()
        # the reference loop order is model-major, subset-minor: raise on the first failure
        order = sorted(range(len(res.problems)), key=lambda k: (res.problems[k].model, res.problems[k].level))
        for k in order:
            _api.raise_like_reference(status_h[:, k], res.problems[k].K)
        summ, _ = _E.summarize_result(res)
        mean, se, t, nobs = (summ.mean.cpu().numpy(), summ.se.cpu().numpy(), summ.tstat.cpu().numpy(),
                             summ.nobs.cpu().numpy())
        for k, p in enumerate(res.problems):
            name = models[p.model].name
            xs = model_cols[name]
            ser = _api.summary_from_device(mean[k], se[k], t[k], nobs[k], xs, k_slope0=1,
                                           k_r2=res.pmax, k_n=res.pmax + 1)
            stats[(name, level_names[p.level])] = {
                "coef": [ser[f"{x}_coef"] for x in xs],
                "tstat": [ser[f"{x}_tstat"] for x in xs],
                "mean_R2": ser["mean_R2"], "mean_N": ser["mean_N"]}
    return _format_table_2(stats, list(subsets_comp_crsp.keys()))


# ------------------------------------------------------------------------------------------
# Figure 1
# ------------------------------------------------------------------------------------------
def figure_1_coefficients(subsets_comp_crsp: dict, model_vars=None, window=120, min_periods=60):
    """Numerical core of create_figure_1 (reference :882-926): per subset ('All stocks',
    'Large stocks') the monthly OLS params (const + slopes, has_constant='add', months with
    N < K+1 skipped) and their rolling(window, min_periods) means.  Returns
    {subset: (monthly_df, rolling_df)} indexed by mthcaldt."""
    model_vars = list(model_vars or _LW.FIG1_VARS)
    out = {}
    for name in ["All stocks", "Large stocks"]:
        if name not in subsets_comp_crsp:
            continue
        d = subsets_comp_crsp[name]
        cols = model_vars + ["retx"]
        arrays = [_api.as_f64(d[c]) for c in cols]
        panel = _E.panel_from_arrays(arrays, cols, d["mthcaldt"].values)
        if panel.nrows == 0:
            continue
        K = len(model_vars)
        res = _E.fm_pass(panel, [_E.Model("fig1", y=K, xs=list(range(K)), const_check=False)])
        status = res.status[:, 0].cpu().numpy()
        fitted = (status & _L.FM_ST_FITTED) != 0
        if not fitted.any():
            continue
        if (status[fitted] & _L.FM_ST_INF_IN_X).any():
            raise _api.MissingDataError("exog contains inf or nans")
        ix = _E.compact_result(res)
        roll = _E.rolling_result(res, ix, window, min_periods)[0].cpu().numpy()
        rec = res.rec[:, 0, :].cpu().numpy()
        months = pd.Index(np.asarray(panel.months)[fitted], name="mthcaldt")
        names = ["const"] + model_vars
        monthly = pd.DataFrame(rec[fitted][:, :K + 1], index=months, columns=names)
        rolling = pd.DataFrame(roll[:fitted.sum(), :K + 1], index=months, columns=names)
        out[name] = (monthly, rolling)
    return out


def create_figure_1(subsets_comp_crsp: dict, save_plot: bool = True,
                    output_dir: Union[None, Path] = OUTPUT_DIR) -> tuple:
    """Figure 1: ten-year rolling Fama-MacBeth slopes of the 5-variable model for All and
    Large stocks, two stacked panels (reference src/calc_Lewellen_2014.py:871-957)."""
    import matplotlib
    if os.environ.get("DISPLAY") is None:
        matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    labels = {"log_bm": "B/M", "return_12_2": "Ret12", "log_issues_36": "Issue36",
              "accruals_final": "Accruals", "log_assets_growth": "Log AG"}
    coefs = figure_1_coefficients(subsets_comp_crsp)
    fig, axes = plt.subplots(nrows=2, ncols=1, figsize=(14, 10), sharex=True)
    for ax, name, title in ((axes[0], "All stocks", "Panel A: All Stocks (10-Year Rolling Slopes)"),
                            (axes[1], "Large stocks", "Panel B: Large Stocks (10-Year Rolling Slopes)")):
        if name not in coefs:
            continue
        roll = coefs[name][1]
        for v in _LW.FIG1_VARS:
            ax.plot(roll.index, roll[v], label=labels[v])
        ax.set_title(title)
        ax.set_ylabel("Slope Coefficient")
        if name == "Large stocks":
            ax.set_xlabel("Month")
        ax.legend()
        ax.margins(x=0)
    plt.tight_layout()
    return fig, axes


# ------------------------------------------------------------------------------------------
# Forecast extensions (A7/A8; not in the reference — parity unpinned)
# ------------------------------------------------------------------------------------------
def monthly_coefficients(df: pd.DataFrame, return_col: str, predictor_cols: list,
                         date_col: str = "mthcaldt") -> pd.DataFrame:
    """Per-month intercept and slopes on the run_monthly_cs_regressions row set."""
    predictor_cols = list(predictor_cols)
    names = predictor_cols + [return_col]
    arrays = [_api.as_f64(df[c]) for c in names]
    panel = _E.panel_from_arrays(arrays, names, df[date_col].values)
    K = len(predictor_cols)
    res = _E.fm_pass(panel, [_E.Model("m", y=K, xs=list(range(K)))])
    status = res.status[:, 0].cpu().numpy()
    _api.raise_like_reference(status, K)
    fitted = (status & _L.FM_ST_FITTED) != 0
    rec = res.rec[:, 0, :].cpu().numpy()
    return pd.DataFrame(rec[fitted][:, :K + 1], index=pd.Index(np.asarray(panel.months)[fitted], name=date_col),
                        columns=["const"] + predictor_cols)


def rolling_coefficients(params_df: pd.DataFrame, window=120, min_periods=60, lag=1) -> pd.DataFrame:
    """rolling(window, min_periods) means of the coefficient table, shifted by ``lag`` rows
    (the forecast for month t uses coefficients through t-lag)."""
    import torch
    dev = _E.require_device()
    T, k = params_df.shape
    vals = np.ascontiguousarray(params_df.to_numpy(dtype=np.float64))
    rec = torch.from_numpy(vals).to(dev).view(T, 1, k)
    status = torch.full((T, 1), _L.FM_ST_FITTED, dtype=torch.int32, device=dev)
    ix = _E.ts_compact(status, 1, 1, T, 1)
    out = torch.empty((1, T, k), dtype=torch.float64, device=dev)
    _L.call("fm_rolling_mean", rec.data_ptr(), k, k, ix.idx.data_ptr(), ix.count.data_ptr(), T, 1, k,
            int(window), int(min_periods), out.data_ptr(), _E._stream())
    roll = pd.DataFrame(out[0].cpu().numpy(), index=params_df.index, columns=params_df.columns)
    return roll.shift(lag)


def expected_return_forecasts(df: pd.DataFrame, coef_rolling: pd.DataFrame, predictor_cols: list,
                              date_col: str = "mthcaldt") -> pd.Series:
    """Out-of-sample expected returns F_it = a_{t-1} + sum_k b_{k,t-1} x_ikt (A7); NaN for
    months without a lagged rolling coefficient row or rows with a NaN characteristic."""
    import torch
    predictor_cols = list(predictor_cols)
    arrays = [_api.as_f64(df[c]) for c in predictor_cols]
    panel = _E.panel_from_arrays(arrays, predictor_cols, df[date_col].values)
    c = coef_rolling[["const"] + predictor_cols].reindex(pd.Index(panel.months))
    coef = torch.from_numpy(np.ascontiguousarray(c.to_numpy(dtype=np.float64))).to(panel.device)
    f = _E.forecast(panel, coef).cpu().numpy()
    out = np.full(len(df), np.nan)
    out[panel.order] = f
    return pd.Series(out, index=df.index, name="forecast")


def predictive_slope_regressions(df: pd.DataFrame, forecast, return_col: str = "retx",
                                 date_col: str = "mthcaldt", nw_lags: int = 4):
    """A8: monthly OLS of returns on the forecast, then the FM summary with NW(nw_lags).
    Returns (monthly results frame, summary Series)."""
    d = pd.DataFrame({date_col: df[date_col].values, return_col: df[return_col].values,
                      "forecast": np.asarray(forecast, dtype=np.float64)})
    cs = run_monthly_cs_regressions(d, return_col, ["forecast"], date_col)
    return cs, fama_macbeth_summary(cs, ["forecast"], date_col, nw_lags)


def lewellen_pipeline(crsp_comp: pd.DataFrame, variables_dict: dict = None, **cfg):
    """The whole Table-2 / Figure-1 / forecast pass device-resident from one frame
    (winsorize -> universes -> 3 models x 3 universes + Figure 1 -> NW -> rolling ->
    predictive slopes).  Returns fmcore.lewellen.PipelineResult (device tensors)."""
    vd = variables_dict or _LW.VARIABLES_DICT
    model_cols = _LW.table2_models(vd)
    cols = list(dict.fromkeys(["retx"] + [c for xs in model_cols.values() for c in xs] + _LW.FIG1_VARS))
    df = crsp_comp.sort_values(["mthcaldt", "permno"])
    me = _api.as_f64(df["me"])
    nyse = (df["primaryexch"] == "N").to_numpy().astype(np.uint8)
    panel = _E.panel_from_arrays([_api.as_f64(df[c]) for c in cols], cols, df["mthcaldt"].values,
                                 me=me, nyse=nyse)
    return _LW.run_pipeline(panel, _LW.PipelineConfig(**cfg), model_cols=model_cols)

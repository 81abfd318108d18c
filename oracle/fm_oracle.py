"""CPU ORACLE — test infrastructure only, never the product path.

A plain numpy restatement of the reference's Fama-MacBeth hot path
(BaileyMeche/FM-ReturnPrediction @ /root/reference).  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this
module, and only as the checker / the timed CPU baseline.  The product
(``fm-returnprediction_amd``) never imports it and has no CPU fallback.

Pinning: every function here is checked against golden vectors produced by running the
reference itself (numpy 1.26.4 / pandas 2.3.3 / statsmodels 0.12.2, see
``tests/golden/gen_goldens.py``) in ``tests/test_oracle_golden.py``.  The three
extensions the north star names but the reference lacks (per-month standardization,
out-of-sample forecasts, predictive slopes) are restated from their build definition
 and are "parity unpinned" against the reference.

Citations are ``path:line`` into /root/reference.
"""
from __future__ import annotations

import math

import numpy as np
import pandas as pd


class MissingDataError(ValueError):
    """Mirrors statsmodels.tools.sm_exceptions.MissingDataError (raised by sm.OLS)."""


# ----------------------------------------------------------------------------------------
# Order statistics
# ----------------------------------------------------------------------------------------
def percentile_linear(vals, pct):
    """np.percentile(vals, pct), method 'linear', restated.

    Reference call site: src/calc_Lewellen_2014.py:522-523.  numpy's algorithm
    (function_base._quantile/_lerp, identical in 1.26.4 and 2.2): q = pct/100;
    vi = (n-1)*q; prev = floor(vi), next = prev+1 (both -> n-1 when vi >= n-1);
    g = vi - prev; lerp a+(b-a)*g for g < 0.5 else b-(b-a)*(1-g).  No FMA.
    """
    s = np.sort(np.asarray(vals, dtype=np.float64), kind="stable")
    n = s.size
    q = np.float64(pct) / np.float64(100)
    vi = np.float64(n - 1) * q
    if vi >= n - 1:
        # numpy sets both neighbours to index -1 and gamma = vi - (-1); the lerp still runs
        i = j = n - 1
        g = vi + np.float64(1)
    else:
        i = int(math.floor(vi))
        j = i + 1
        g = vi - np.float64(i)
    a, b = s[i], s[j]
    if (a == 0.0 or b == 0.0) and _both_zero_signs(s):
        # -0.0 == +0.0: which signed zero numpy leaves at i / i+1 is its partition's swap
        # order over the values in frame order (oracle/np_select.py), not the sorted order
        from oracle import np_select
        a, b = np_select.percentile_pair(vals, i if vi < n - 1 else -1)
    with np.errstate(invalid="ignore"):
        d = b - a
    with np.errstate(invalid="ignore"):
        if g >= 0.5:
            return float(b - d * (np.float64(1) - g))
        return float(a + d * g)


def _both_zero_signs(s):
    z = s[s == 0.0]
    return z.size > 1 and np.signbit(z).any() and not np.signbit(z).all()


def pandas_quantile(vals, q):
    """pandas groupby(...).quantile(q) per group, restated (Cython group_quantile).

    Reference call site: src/calc_Lewellen_2014.py:74-82.  idx = int(q*(n-1));
    frac = (q*(n-1)) % 1; frac == 0 -> v[idx] else v[idx] + (v[idx+1]-v[idx])*frac.
    NaN are skipped; empty -> NaN.
    """
    v = np.asarray(vals, dtype=np.float64)
    v = np.sort(v[~np.isnan(v)], kind="stable")
    n = v.size
    if n == 0:
        return float("nan")
    qi = np.float64(q) * np.float64(n - 1)
    i = int(qi)
    frac = qi - np.float64(math.floor(qi))
    if frac == 0.0:
        return float(v[i])
    with np.errstate(invalid="ignore"):
        return float(v[i] + (v[i + 1] - v[i]) * frac)


# ----------------------------------------------------------------------------------------
# Characteristic prep
# ----------------------------------------------------------------------------------------
def winsorize(crsp_comp, varlist, lower_percentile=1, upper_percentile=99):
    """src/calc_Lewellen_2014.py:505-529.  Sort by [mthcaldt, permno] (labels kept),
    then per var per month: non-NaN values; <5 -> unchanged; clip at the linear
    percentiles; NaN bounds are ignored by pandas clip (only arises from inf-inf)."""
    df = crsp_comp.sort_values(["mthcaldt", "permno"]).copy()
    codes, _ = pd.factorize(df["mthcaldt"], sort=True)
    order = np.argsort(codes, kind="stable")
    bounds = np.searchsorted(codes[order], np.arange(codes.max() + 2 if len(codes) else 1))
    for var in varlist:
        col = df[var].to_numpy(dtype=np.float64, copy=True)
        for t in range(len(bounds) - 1):
            idx = order[bounds[t]:bounds[t + 1]]
            v = col[idx]
            vals = v[~np.isnan(v)]
            if vals.size < 5:
                continue
            lo = percentile_linear(vals, lower_percentile)
            hi = percentile_linear(vals, upper_percentile)
            w = v.copy()
            if not np.isnan(lo):
                w = np.where(w < lo, lo, w)
            if not np.isnan(hi):
                w = np.where(w > hi, hi, w)
            col[idx] = w
        df[var] = col
    return df


def standardize(df, varlist, date_col="mthcaldt"):
    """Build-defined extension A9 (not in the reference; parity unpinned):
    z = (x - mean_t) / std_t(ddof=1) over the non-NaN values of each month."""
    out = df.copy()
    g = out.groupby(date_col)
    for var in varlist:
        m = g[var].transform("mean")
        s = g[var].transform("std")
        out[var] = (out[var] - m) / s
    return out


def get_subsets(crsp_comp):
    """src/calc_Lewellen_2014.py:44-112: NYSE me 20th/50th pandas quantiles per month,
    masks me>=me_20 / me>=me_50 (NaN -> False); returns the 3-key dict."""
    df = crsp_comp.sort_values(["mthcaldt", "permno"]).copy()
    nyse = df.loc[df["primaryexch"] == "N"]
    rows = []
    for m, grp in nyse.groupby("mthcaldt"):
        rows.append((m, pandas_quantile(grp["me"].values, 0.2), pandas_quantile(grp["me"].values, 0.5)))
    cuts = pd.DataFrame(rows, columns=["mthcaldt", "me_20", "me_50"])
    df = pd.merge(df, cuts, on="mthcaldt", how="left")
    df["is_all_but_tiny"] = df["me"] >= df["me_20"]
    df["is_large"] = df["me"] >= df["me_50"]
    return {
        "All stocks": df.copy(),
        "All-but-tiny stocks": df.loc[df["is_all_but_tiny"]].copy(),
        "Large stocks": df.loc[df["is_large"]].copy(),
    }


def build_table_1(subsets, variables_dict):
    """src/calc_Lewellen_2014.py:577-670: per subset and variable, inf->NaN, dropna, monthly
    mean/std(ddof=1), their time-series means, distinct permnos; MultiIndex columns."""
    parts = []
    for name, d in subsets.items():
        rows = []
        for label, col in variables_dict.items():
            if col not in d.columns:
                rows.append({"Column": label, "Avg": np.nan, "Std": np.nan, "N": np.nan})
                continue
            v = d[col].to_numpy(dtype=np.float64).copy()
            v[np.isinf(v)] = np.nan
            keep = ~np.isnan(v)
            if not keep.any():
                rows.append({"Column": label, "Avg": np.nan, "Std": np.nan, "N": np.nan})
                continue
            months = d["mthcaldt"].values[keep]
            vv = v[keep]
            uniq, order, bounds = month_groups(months)
            means, stds = [], []
            for t in range(len(uniq)):
                x = vv[order[bounds[t]:bounds[t + 1]]]
                means.append(x.mean())
                stds.append(x.std(ddof=1) if x.size > 1 else np.nan)
            means, stds = np.array(means), np.array(stds)
            rows.append({"Column": label, "Avg": np.nanmean(means) if means.size else np.nan,
                         "Std": np.nanmean(stds) if np.isfinite(stds).any() else np.nan,
                         "N": len(np.unique(d["permno"].values[keep]))})
        p = pd.DataFrame(rows).set_index("Column")
        p.columns = pd.MultiIndex.from_product([[name], p.columns])
        parts.append(p)
    return pd.concat(parts, axis=1)


# ----------------------------------------------------------------------------------------
# Cross-sectional OLS (statsmodels semantics restated)
# ----------------------------------------------------------------------------------------
def _has_nonzero_const(X):
    """statsmodels add_constant(has_constant='skip') detection: ptp==0 & all != 0."""
    if X.shape[0] == 0:
        return False
    with np.errstate(invalid="ignore"):
        ptp = np.max(X, axis=0) - np.min(X, axis=0)
    return bool(np.any((ptp == 0) & np.all(X != 0.0, axis=0)))


def ols_pinv(X, y):
    """statsmodels OLS.fit(method='pinv'): SVD pseudo-inverse, cutoff 1e-15*smax;
    returns (params, rsquared) with centered TSS (model has a constant)."""
    u, s, vt = np.linalg.svd(X, full_matrices=False)
    cutoff = 1e-15 * np.max(s) if s.size else 0.0
    sinv = np.where(s > cutoff, 1.0 / np.where(s > cutoff, s, 1.0), 0.0)
    pinv = (vt.T * sinv) @ u.T
    with np.errstate(invalid="ignore", over="ignore"):
        params = pinv @ y
        resid = y - X @ params
        ssr = float(resid @ resid)
        yc = y - y.mean()
        tss = float(yc @ yc)
        r2 = 1.0 - ssr / tss if tss != 0 else float("nan")
    return params, r2


def month_groups(dates):
    """Ascending unique months and row indices per month (pandas groupby order)."""
    codes, uniq = pd.factorize(pd.Series(dates), sort=True)
    order = np.argsort(codes, kind="stable")
    bounds = np.searchsorted(codes[order], np.arange(len(uniq) + 1))
    return uniq, order, bounds


def run_monthly_cs_regressions(df, return_col, predictor_cols, date_col="mthcaldt"):
    """src/regressions.py:9-76 restated (dropna on [ret, date]+X; per month in ascending
    order: skip N<K+1; intercept prepended unless a nonzero-constant column exists (then
    IndexError at :71); inf in X -> MissingDataError; pinv OLS; rsquared)."""
    sub = df[[return_col, date_col] + list(predictor_cols)].dropna()
    K = len(predictor_cols)
    y_all = sub[return_col].to_numpy(dtype=np.float64)
    X_all = sub[list(predictor_cols)].to_numpy(dtype=np.float64)
    uniq, order, bounds = month_groups(sub[date_col].values)
    rows = []
    for t, m in enumerate(uniq):
        idx = order[bounds[t]:bounds[t + 1]]
        X = X_all[idx]
        y = y_all[idx]
        if len(idx) < K + 1:
            continue
        if _has_nonzero_const(X):
            raise IndexError(f"index {K - 1} is out of bounds for axis 0 with size {K - 1}")
        if not np.all(np.isfinite(X)):
            raise MissingDataError("exog contains inf or nans")
        Xc = np.column_stack([np.ones(len(idx)), X])
        params, r2 = ols_pinv(Xc, y)
        row = {date_col: m, "N": len(idx), "R2": r2}
        for i, c in enumerate(predictor_cols):
            row[f"slope_{c}"] = params[1 + i]
        rows.append(row)
    return pd.DataFrame(rows)


def newey_west_mean_se(slopes, lags=4):
    """src/regressions.py:78-100: weights 1-k/T (break when negative), var/T^2, sqrt."""
    x = np.asarray(slopes, dtype=float)
    T = x.size
    if T < 2:
        return np.nan
    u = x - x.mean()
    gamma0 = np.sum(u * u)
    acc = 0.0
    for k in range(1, lags + 1):
        w = 1.0 - (k / T)
        if w < 0:
            break
        acc += w * np.sum(u[k:] * u[:-k])
    with np.errstate(invalid="ignore"):
        return np.sqrt((gamma0 + 2.0 * acc) / (T ** 2))


def fama_macbeth_summary(cs_results, predictor_cols, date_col="mthcaldt", nw_lags=4):
    """src/regressions.py:102-131."""
    out = {}
    for col in predictor_cols:
        s = cs_results[f"slope_{col}"].dropna()
        if len(s) < 10:
            out[f"{col}_coef"] = np.nan
            out[f"{col}_tstat"] = np.nan
            continue
        mean = s.mean()
        out[f"{col}_coef"] = mean
        with np.errstate(divide="ignore", invalid="ignore"):
            out[f"{col}_tstat"] = mean / newey_west_mean_se(s, lags=nw_lags)
    out["mean_R2"] = cs_results["R2"].mean()
    out["mean_N"] = cs_results["N"].mean()
    return pd.Series(out)


def rolling_mean(x, window=120, min_periods=60):
    """pandas rolling(window, min_periods).mean() on a row-ordered series (NaN skipped,
    min_periods counts non-NaN), src/calc_Lewellen_2014.py:926.  pandas converts +-inf to
    NaN before the window sums (Window._prep_values), so infinities are skipped too."""
    x = np.asarray(x, dtype=np.float64)
    out = np.full(x.size, np.nan)
    for i in range(x.size):
        w = x[max(0, i - window + 1):i + 1]
        w = w[np.isfinite(w)]
        if w.size >= min_periods:
            out[i] = w.sum() / w.size
    return out


def figure1_coefficients(subsets, model_vars=None, window=120, min_periods=60):
    """create_figure_1 numerical core (src/calc_Lewellen_2014.py:882-926): per subset
    ("All stocks", "Large stocks") monthly OLS with has_constant='add', skip N<6, then
    the rolling means of const and slopes.  Returns {subset: (monthly_df, rolling_df)}."""
    model_vars = model_vars or ["log_bm", "return_12_2", "log_issues_36",
                                "accruals_final", "log_assets_growth"]
    res = {}
    for name in ["All stocks", "Large stocks"]:
        if name not in subsets:
            continue
        d = subsets[name].sort_values(["mthcaldt", "permno"]).dropna(subset=["retx"] + model_vars)
        if d.empty:
            continue
        uniq, order, bounds = month_groups(d["mthcaldt"].values)
        y_all = d["retx"].to_numpy(dtype=np.float64)
        X_all = d[model_vars].to_numpy(dtype=np.float64)
        rows = []
        for t, m in enumerate(uniq):
            idx = order[bounds[t]:bounds[t + 1]]
            if len(idx) < len(model_vars) + 1:
                continue
            if not np.all(np.isfinite(X_all[idx])):
                raise MissingDataError("exog contains inf or nans")
            Xc = np.column_stack([np.ones(len(idx)), X_all[idx]])
            p, _ = ols_pinv(Xc, y_all[idx])
            rows.append([m] + list(p))
        monthly = pd.DataFrame(rows, columns=["mthcaldt", "const"] + model_vars).set_index("mthcaldt").sort_index()
        roll = monthly.apply(lambda c: pd.Series(rolling_mean(c.values, window, min_periods), index=c.index))
        res[name] = (monthly, roll)
    return res


# ----------------------------------------------------------------------------------------
# Build-defined extensions A7/A8 (parity unpinned vs the reference)
# ----------------------------------------------------------------------------------------
def monthly_params(df, return_col, predictor_cols, date_col="mthcaldt"):
    """Per-month full params (intercept + slopes) on the run_monthly_cs_regressions row
    set; used to build rolling coefficients for the forecasts."""
    sub = df[[return_col, date_col] + list(predictor_cols)].dropna()
    K = len(predictor_cols)
    uniq, order, bounds = month_groups(sub[date_col].values)
    y_all = sub[return_col].to_numpy(dtype=np.float64)
    X_all = sub[list(predictor_cols)].to_numpy(dtype=np.float64)
    months, params = [], []
    for t, m in enumerate(uniq):
        idx = order[bounds[t]:bounds[t + 1]]
        if len(idx) < K + 1:
            continue
        p, _ = ols_pinv(np.column_stack([np.ones(len(idx)), X_all[idx]]), y_all[idx])
        months.append(m)
        params.append(p)
    return pd.DataFrame(np.array(params).reshape(len(months), K + 1), index=pd.Index(months, name=date_col),
                        columns=["const"] + list(predictor_cols))


def rolling_coefficients(params_df, window=120, min_periods=60, lag=1):
    """A7: rolling(window,min_periods) means of intercept and slopes over fitted-month
    rows, shifted by ``lag`` rows so month t uses information through t-1."""
    roll = params_df.apply(lambda c: pd.Series(rolling_mean(c.values, window, min_periods), index=c.index))
    return roll.shift(lag)


def expected_return_forecasts(df, coef_rolling, predictor_cols, date_col="mthcaldt"):
    """A7: F_it = a_{t-1} + sum_k b_{k,t-1} x_{ikt} for rows whose month has a lagged
    rolling coefficient row (NaN otherwise, or if any x is NaN)."""
    c = coef_rolling.reindex(df[date_col].values)
    F = c["const"].to_numpy(dtype=np.float64).copy()
    for k in predictor_cols:
        F = F + c[k].to_numpy(dtype=np.float64) * df[k].to_numpy(dtype=np.float64)
    return pd.Series(F, index=df.index, name="forecast")


def predictive_slope_regressions(df, forecast, return_col="retx", date_col="mthcaldt", nw_lags=4):
    """A8: per-month OLS of returns on the forecast, then the FM summary with NW(4)."""
    d = pd.DataFrame({date_col: df[date_col].values, return_col: df[return_col].values,
                      "forecast": np.asarray(forecast, dtype=np.float64)})
    cs = run_monthly_cs_regressions(d, return_col, ["forecast"], date_col)
    return cs, fama_macbeth_summary(cs, ["forecast"], date_col, nw_lags)


# ----------------------------------------------------------------------------------------
# Array-level pipeline (bench cpu_baseline) — the same semantics over month-sorted arrays
# ----------------------------------------------------------------------------------------
def standardize_segments(v, seg_off):
    """A9 on one month-sorted column: per month z = (x - mean_t) / std_t(ddof=1) over the
    non-NaN values (pandas groupby transform('mean') / transform('std'), as ``standardize``);
    a month with < 2 values or zero dispersion gives NaN z."""
    out = np.full(v.size, np.nan)
    for t in range(len(seg_off) - 1):
        seg = v[seg_off[t]:seg_off[t + 1]]
        vals = seg[~np.isnan(seg)]
        if vals.size == 0:
            continue
        m = vals.mean()
        s = vals.std(ddof=1) if vals.size > 1 else np.nan
        with np.errstate(invalid="ignore", divide="ignore"):
            out[seg_off[t]:seg_off[t + 1]] = (seg - m) / s
    return out


def pipeline_arrays(cols, seg_off, me, nyse, models, fig1_model, nw_lags=4, window=120, min_periods=60,
                    winsor=True, standardize=False, y_name="retx"):
    """Full C3/C4 pass on month-sorted arrays: winsorize all columns (1/99), NYSE
    universes, per (model, universe) monthly pinv OLS, FM summaries with NW, Figure-1
    rolling coefficients, lagged-rolling forecasts and predictive-slope FM summaries.

    cols: dict name -> float64 array (month-sorted); seg_off: int64 [T+1].
    models: dict name -> (y name, [x names], [universe levels]).  Returns a dict of
    per-problem outputs keyed by (model, universe level).
    ``standardize`` (A9, build-defined): after winsorizing, every column except ``y_name`` is
    replaced by its per-month z-score (standardize_segments) before the regressions."""
    T = len(seg_off) - 1
    w = {}
    for name, v in cols.items():
        v = v.copy()
        if winsor:
            for t in range(T):
                seg = v[seg_off[t]:seg_off[t + 1]]
                vals = seg[~np.isnan(seg)]
                if vals.size < 5:
                    continue
                lo = percentile_linear(vals, 1)
                hi = percentile_linear(vals, 99)
                if not np.isnan(lo):
                    seg = np.where(seg < lo, lo, seg)
                if not np.isnan(hi):
                    seg = np.where(seg > hi, hi, seg)
                v[seg_off[t]:seg_off[t + 1]] = seg
        w[name] = v
    if standardize:
        for name in w:
            if name != y_name:
                w[name] = standardize_segments(w[name], seg_off)
    level = np.zeros(len(me), dtype=np.int8)
    for t in range(T):
        sl = slice(seg_off[t], seg_off[t + 1])
        mt = me[sl]
        ny = mt[nyse[sl]]
        q20 = pandas_quantile(ny, 0.2)
        q50 = pandas_quantile(ny, 0.5)
        with np.errstate(invalid="ignore"):
            level[sl] = (mt >= q20).astype(np.int8) + (mt >= q50).astype(np.int8)
    out = {}
    for mname, (yname, xs, univs) in models.items():
        X_all = np.column_stack([w[x] for x in xs])
        y_all = w[yname]
        ok = ~np.isnan(y_all) & ~np.isnan(X_all).any(axis=1)
        for u in univs:
            rows = []
            for t in range(T):
                sl = np.arange(seg_off[t], seg_off[t + 1])
                sel = sl[ok[sl] & (level[sl] >= u)]
                if sel.size < len(xs) + 1:
                    continue
                Xc = np.column_stack([np.ones(sel.size), X_all[sel]])
                p, r2 = ols_pinv(Xc, y_all[sel])
                rows.append((t, sel.size, r2, p))
            months = np.array([r[0] for r in rows], dtype=np.int64)
            P = np.array([r[3] for r in rows]).reshape(len(rows), len(xs) + 1)
            N = np.array([r[1] for r in rows], dtype=np.int64)
            R2 = np.array([r[2] for r in rows])
            summ = {}
            for k in range(len(xs)):
                s = P[:, 1 + k]
                s = s[~np.isnan(s)]
                if s.size < 10:
                    summ[xs[k]] = (np.nan, np.nan)
                else:
                    mu = s.mean()
                    summ[xs[k]] = (mu, mu / newey_west_mean_se(s, nw_lags))
            roll = np.column_stack([rolling_mean(P[:, k], window, min_periods) for k in range(P.shape[1])]) \
                if len(rows) else np.zeros((0, len(xs) + 1))
            # forecasts with the previous fitted row's rolling coefficients
            pred = []
            for i in range(1, len(rows)):
                c = roll[i - 1]
                if np.isnan(c).any():
                    continue
                t = rows[i][0]
                sl = np.arange(seg_off[t], seg_off[t + 1])
                sel = sl[ok[sl] & (level[sl] >= u)]
                F = c[0] + X_all[sel] @ c[1:]
                p, r2 = ols_pinv(np.column_stack([np.ones(sel.size), F]), y_all[sel])
                pred.append((t, sel.size, r2, p[1]))
            ps = np.array([r[3] for r in pred])
            ps_sum = (np.nan, np.nan) if ps.size < 10 else (ps.mean(), ps.mean() / newey_west_mean_se(ps, nw_lags))
            out[(mname, u)] = dict(month=months, N=N, R2=R2, params=P, summary=summ,
                                   mean_R2=R2.mean() if R2.size else np.nan,
                                   mean_N=N.mean() if N.size else np.nan, rolling=roll,
                                   pred_month=np.array([r[0] for r in pred], dtype=np.int64),
                                   pred_slope=ps, pred_R2=np.array([r[2] for r in pred]),
                                   pred_summary=ps_sum)
    return out

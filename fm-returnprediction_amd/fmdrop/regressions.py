"""Drop-in replacement for the reference's src/regressions.py, on MI355X.

Same names, signatures, return types, column/key order and error behaviour as
BaileyMeche/FM-ReturnPrediction src/regressions.py:9-131; the per-month OLS, the
Newey-West errors and the time-series means run in libfm_hip kernels (fm_gram, fm_solve,
fm_ts_summary) through ctypes.  statsmodels is not needed.
"""

import numpy as np
import pandas as pd

from fmcore import api as _api
from fmcore import engine as _E

MissingDataError = _api.MissingDataError


def run_monthly_cs_regressions(df: pd.DataFrame, return_col: str, predictor_cols: list,
                               date_col: str = "mthcaldt") -> pd.DataFrame:
    """Per-month cross-sectional OLS of ``return_col`` on an intercept and
    ``predictor_cols`` (reference src/regressions.py:9-76).

    Rows with NaN in any of [return_col, date_col] + predictor_cols are dropped; months
    with fewer than K+1 rows are skipped; returns one row per fitted month with columns
    [date_col, 'N', 'R2', 'slope_<col>'...] in ascending month order.
    """
    predictor_cols = list(predictor_cols)
    sub = df[[return_col, date_col] + predictor_cols]
    names = predictor_cols + [return_col]
    arrays = [_api.as_f64(sub[c]) for c in names]
    panel = _E.panel_from_arrays(arrays, names, sub[date_col].values)
    K = len(predictor_cols)
    res = _E.fm_pass(panel, [_E.Model("m", y=K, xs=list(range(K)))])
    status = res.status[:, 0].cpu().numpy()
    rec = res.rec[:, 0, :].cpu().numpy()
    _api.raise_like_reference(status, K)
    return _api.cs_frame(panel.months, rec, status, res.pmax, predictor_cols, date_col)


def newey_west_mean_se(slopes: np.ndarray, lags: int = 4) -> float:
    """Newey-West standard error of the mean with weights 1-k/T (reference
    src/regressions.py:78-100)."""
    x = np.asarray(slopes, dtype=float)
    T = x.size
    if T < 2:
        return np.nan
    if not np.all(np.isfinite(x)):
        return np.nan   # the reference's arithmetic turns any NaN/inf into NaN here
    _, se, _, _ = _api.records_summary(x.reshape(T, 1), nw_lags=int(lags))
    return float(se[0])


def fama_macbeth_summary(cs_results: pd.DataFrame, predictor_cols: list, date_col="mthcaldt",
                         nw_lags=4) -> pd.Series:
    """Time-series means of the monthly slopes with Newey-West t-stats, plus mean R2
    and mean N (reference src/regressions.py:102-131)."""
    predictor_cols = list(predictor_cols)
    cols = [cs_results[f"slope_{c}"] for c in predictor_cols]
    r2 = cs_results["R2"]
    n = cs_results["N"]
    T = len(cs_results)
    if T == 0:
        out = {}
        for c in predictor_cols:
            out[f"{c}_coef"] = np.nan
            out[f"{c}_tstat"] = np.nan
        out["mean_R2"] = np.nan
        out["mean_N"] = np.nan
        return pd.Series(out, dtype=np.float64)
    vals = np.column_stack([_api.as_f64(c) for c in cols] + [_api.as_f64(r2), _api.as_f64(n)])
    mean, se, t, nobs = _api.records_summary(vals, nw_lags=int(nw_lags))
    K = len(predictor_cols)
    return _api.summary_from_device(mean, se, t, nobs, predictor_cols, k_slope0=0, k_r2=K, k_n=K + 1)

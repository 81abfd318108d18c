"""pandas <-> device glue shared by the drop-in modules (fmdrop/regressions.py,
fmdrop/calc_Lewellen_2014.py, mirroring the reference's src/regressions.py and
src/calc_Lewellen_2014.py): panel marshaling, reference-exact error behaviour and
result frames.  Compute happens only in libfm_hip kernels (fmcore.engine)."""
from __future__ import annotations

import numpy as np
import pandas as pd
import torch

from . import _lib as L
from . import engine as E

try:  # the reference raises statsmodels' class; reuse it when statsmodels is importable
    from statsmodels.tools.sm_exceptions import MissingDataError  # type: ignore
except Exception:  # pragma: no cover - statsmodels is not part of this image
    class MissingDataError(ValueError):
        """Mirrors statsmodels.tools.sm_exceptions.MissingDataError."""


def as_f64(s):
    return pd.to_numeric(s, errors="coerce").to_numpy(dtype=np.float64, na_value=np.nan) \
        if not np.issubdtype(np.asarray(s).dtype, np.floating) else np.asarray(s, dtype=np.float64)


def raise_like_reference(status, K, what="exog"):
    """statsmodels/regressions.py failure order within the month loop: the first fitted
    month (ascending) with an inf regressor raises MissingDataError at sm.OLS; with a
    nonzero-constant regressor add_constant skips the intercept and the slope loop raises
    IndexError (reference src/regressions.py:50,57,71)."""
    st = np.asarray(status)
    bad = np.nonzero(((st & L.FM_ST_FITTED) != 0) &
                     ((st & (L.FM_ST_INF_IN_X | L.FM_ST_CONST_COL)) != 0))[0]
    if bad.size == 0:
        return
    s = st[bad[0]]
    if s & L.FM_ST_INF_IN_X:
        raise MissingDataError(f"{what} contains inf or nans")
    raise IndexError(f"index {K - 1} is out of bounds for axis 0 with size {K - 1}")


def cs_frame(months, rec, status, pmax, predictor_cols, date_col):
    """Monthly results frame with the reference's columns: date, N, R2, slope_<x>...
    (src/regressions.py:68-75)."""
    fitted = (np.asarray(status) & L.FM_ST_FITTED) != 0
    if not fitted.any():
        return pd.DataFrame([])
    d = {date_col: np.asarray(months)[fitted],
         "N": rec[fitted, pmax + 1].astype(np.int64),
         "R2": rec[fitted, pmax]}
    for i, c in enumerate(predictor_cols):
        d[f"slope_{c}"] = rec[fitted, 1 + i]
    return pd.DataFrame(d)


def summary_from_device(mean, se, tstat, nobs, predictor_cols, k_slope0=1, k_r2=None, k_n=None,
                        min_obs=10):
    """fama_macbeth_summary's Series (src/regressions.py:110-131) from device summaries of
    one problem's record columns."""
    out = {}
    for i, c in enumerate(predictor_cols):
        k = k_slope0 + i
        if nobs[k] < min_obs:
            out[f"{c}_coef"] = np.nan
            out[f"{c}_tstat"] = np.nan
        else:
            out[f"{c}_coef"] = mean[k]
            out[f"{c}_tstat"] = tstat[k]
    out["mean_R2"] = mean[k_r2] if nobs[k_r2] > 0 else np.nan
    out["mean_N"] = mean[k_n] if nobs[k_n] > 0 else np.nan
    return pd.Series(out, dtype=np.float64)


def records_summary(values, nw_lags=4):
    """Device FM summaries of the columns of a [T, k] host array (all rows present)."""
    dev = E.require_device()
    return records_summary_device(torch.from_numpy(np.ascontiguousarray(values, dtype=np.float64)).to(dev),
                                  nw_lags)


def records_summary_device(vals, nw_lags=0):
    """Device FM summaries (NaN-skipping means) of the columns of a [T, k] device tensor."""
    T, k = vals.shape
    rec = vals.contiguous().view(T, 1, k)
    status = torch.full((T, 1), L.FM_ST_FITTED, dtype=torch.int32, device=vals.device)
    ix = E.ts_compact(status, 1, 1, T, 1)
    s = E.ts_summary(rec, k, k, ix, T, 1, k, nw_lags)
    return (s.mean[0].cpu().numpy(), s.se[0].cpu().numpy(), s.tstat[0].cpu().numpy(),
            s.nobs[0].cpu().numpy())


def sorted_frame(df):
    return df.sort_values(["mthcaldt", "permno"]).copy()

"""Shared tolerances and golden loaders for the parity tests.

Floating-point contract (BASELINE.json north star): FP64 slopes, t-stats and forecasts
within 1e-9 relative error.  Relative to what: SURVEY.md §8(a) 'Tolerance definition' —
|a-b| <= RTOL * max(|b|, s) with s = RMS of that coefficient's series, because a plain
elementwise relative error is meaningless for slopes that happen to sit near zero.
Integer outputs (N, month lists, masks, ranks) and winsorize cuts are compared bit-exact.
"""
import json
import os

import numpy as np

RTOL = 1e-9
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_npz(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def load_json(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def series_close(a, b, rtol=RTOL, scale=None):
    """True if a ~ b under the series-RMS tolerance; NaN/inf must match exactly."""
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    if a.shape != b.shape:
        return False
    fin = np.isfinite(b)
    if not np.array_equal(np.isnan(a), np.isnan(b)):
        return False
    if not np.array_equal(a[~fin & ~np.isnan(b)], b[~fin & ~np.isnan(b)]):
        return False
    if not fin.any():
        return True
    s = scale if scale is not None else float(np.sqrt(np.mean(b[fin] ** 2)))
    tol = rtol * np.maximum(np.abs(b[fin]), s)
    return bool(np.all(np.abs(a[fin] - b[fin]) <= tol))


def assert_series_close(a, b, what="", rtol=RTOL, scale=None):
    if not series_close(a, b, rtol, scale):
        a = np.asarray(a, dtype=np.float64)
        b = np.asarray(b, dtype=np.float64)
        msg = f"{what}: shapes {a.shape} vs {b.shape}"
        if a.shape == b.shape:
            d = np.abs(a - b)
            with np.errstate(invalid="ignore"):
                i = int(np.nanargmax(d)) if np.isfinite(d).any() else 0
            msg += f"; worst |diff|={d.flat[i]!r} at {i}: {a.flat[i]!r} vs {b.flat[i]!r}"
            bad = np.flatnonzero((np.isnan(a) != np.isnan(b)).ravel() |
                                 (np.isinf(b) & (a != b)).ravel())
            if bad.size:
                j = int(bad[0])
                msg += f"; {bad.size} NaN/inf mismatches, first at {j}: {a.flat[j]!r} vs {b.flat[j]!r}"
        raise AssertionError(msg)


def scalar_close(a, b, rtol=RTOL, scale=0.0):
    if b is None:
        return a is None or (isinstance(a, float) and np.isnan(a))
    a = float(a)
    if np.isinf(b) or np.isnan(b):
        return a == b or (np.isnan(a) and np.isnan(b))
    return abs(a - b) <= rtol * max(abs(b), scale)


def frame_from(npz, prefix):
    """Rebuild a DataFrame written by gen_goldens.frame_arrays (index + columns)."""
    import pandas as pd
    keys = [k for k in npz.files if k.startswith(prefix) and k != prefix + "index"]
    data = {}
    for k in keys:
        c = k[len(prefix):]
        v = npz[k]
        if c == "mthcaldt":
            v = v.astype("datetime64[ns]")
        elif c == "primaryexch":
            v = np.where(v == 1, "N", "Q")
        elif c in ("is_all_but_tiny", "is_large"):
            v = v.astype(bool)
        data[c] = v
    return pd.DataFrame(data, index=pd.Index(npz[prefix + "index"]))


def chars_inputs(g):
    """The raw monthly / daily golden input frames of chars.npz (tests/golden/cases.py)."""
    import pandas as pd
    m = pd.DataFrame({"permno": g["in_permno"], "mthcaldt": g["in_mthcaldt"].astype("datetime64[ns]")},
                     index=pd.Index(g["in_index"]))
    for k in ("me", "be", "retx", "accruals", "depreciation", "earnings", "assets", "dvc", "prc",
              "shrout", "total_debt", "sales"):
        m[k] = g["in_" + k]
    m["jdate"] = m["mthcaldt"]
    d = pd.DataFrame({"permno": g["din_permno"], "dlycaldt": g["din_dlycaldt"].astype("datetime64[ns]"),
                      "retx": g["din_retx"]}, index=pd.Index(g["din_index"]))
    return m, d


def beta_inputs(seed=3, nfirms=30):
    """Synthetic daily stock / market returns and a monthly (permno, jdate) frame for the
    156-week rolling beta (tests only): ragged firm date ranges over business days, a firm
    with a > 3-year gap (empty weekly windows), NaN returns, a -100% return (log -> -inf),
    market index days missing (the inner join drops them), months outside every firm's
    range and a permno with no daily data."""
    import pandas as pd
    rng = np.random.default_rng(seed)
    bdays = pd.bdate_range("1990-01-01", "2001-12-31")
    mkt_days = bdays[rng.random(len(bdays)) > 0.01]
    rm = rng.normal(0.0004, 0.01, len(mkt_days))
    crsp_index_d = pd.DataFrame({"caldt": mkt_days, "vwretx": rm})
    rows = []
    for f in range(nfirms):
        a = int(rng.integers(0, len(bdays) - 300))
        b = int(rng.integers(a + 50, len(bdays)))
        d = bdays[a:b]
        if f == 3:   # a gap longer than the 156-week window
            d = d[(d < bdays[a] + pd.Timedelta(days=200)) | (d > bdays[a] + pd.Timedelta(days=1500))]
        beta = rng.normal(1.0, 0.4)
        m = np.interp(d.values.astype("int64"), mkt_days.values.astype("int64"), rm)
        r = beta * m + rng.normal(0, 0.015, len(d))
        if f in (7, 8):
            r[rng.random(len(d)) < 0.002] = np.nan
        if f == 5:
            r[len(r) // 2] = -1.0
        rows.append(pd.DataFrame({"permno": 10000 + f, "dlycaldt": d, "retx": r}))
    crsp_d = pd.concat(rows, ignore_index=True).sample(frac=1.0, random_state=seed).reset_index(drop=True)
    months = pd.date_range("1989-06-30", "2002-06-30", freq="ME")
    comp = [(10000 + f, m) for f in range(nfirms + 1) for m in months[rng.random(len(months)) < 0.7]]
    crsp_comp = pd.DataFrame(comp, columns=["permno", "jdate"])
    crsp_comp["mthcaldt"] = crsp_comp["jdate"]
    return crsp_d, crsp_index_d, crsp_comp

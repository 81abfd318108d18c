"""Deterministic synthetic CRSP/Compustat-style panels for the Fama-MacBeth path.

There is no WRDS data offline, so every workload is a seeded synthetic panel. The
generator is counter based: each cell is a pure function of (seed, month, firm, column),
built only from 64-bit integer mixing and IEEE-754 binary64 +,-,*,/ and sqrt (all
correctly rounded).  The HIP kernel ``fm_gen_panel`` (csrc/fm_gen.hip) evaluates the
identical expression sequence, so a shard generated on any GPU is bit-identical to the
numpy panel built here for the same (seed, month range).

Distribution spec: characteristic j = mu_j + sd_j * t/2 with t a
Student-t(2) draw (closed-form inverse CDF, heavy tails so the 1/99 winsorization is
active), (mu_j, sd_j) = the "All stocks" Avg/Std of Lewellen Table 1 as hard-coded in
the reference fixture ``src/test_calc_Lewellen_2014.py:50-65``.  ``retx`` carries a
linear signal in the standardized characteristics plus t-noise.  ``dy`` has a 30 % mass
at exactly 0.0 (as dividend yields do), which exercises tied order statistics.

Layout matches the reference's long format after ``sort_values(["mthcaldt","permno"])``
(``src/calc_Lewellen_2014.py:69,514``): rows are month-major, permno ascending.
"""
from __future__ import annotations

import numpy as np

# Column order = notebook ``variables_dict`` order (src/get_data.ipynb cell 24).
WINSOR_VARS = [
    "retx", "log_size", "log_bm", "return_12_2", "log_issues_12", "accruals_final",
    "roa", "log_assets_growth", "dy", "log_return_13_36", "log_issues_36", "beta",
    "rolling_std_252", "debt_price", "sales_price",
]
CHAR_VARS = WINSOR_VARS[1:]

# (Avg, Std) "All stocks" from src/test_calc_Lewellen_2014.py:51-65 (retx in decimals).
TABLE1_MOMENTS = {
    "retx": (0.0127, 0.1479),
    "log_size": (4.63, 1.93),
    "log_bm": (-0.51, 0.84),
    "return_12_2": (0.13, 0.48),
    "log_issues_36": (0.11, 0.25),
    "accruals_final": (-0.02, 0.10),
    "roa": (0.01, 0.14),
    "log_assets_growth": (0.12, 0.26),
    "dy": (0.02, 0.02),
    "log_return_13_36": (0.24, 0.58),
    "log_issues_12": (0.04, 0.12),
    "beta": (0.96, 0.55),
    "rolling_std_252": (0.15, 0.08),
    "debt_price": (0.83, 1.59),
    "sales_price": (2.53, 3.56),
}

# Signal loadings of retx on the standardized characteristics (CHAR_VARS order).
RET_LOADINGS = [-0.0030, 0.0035, 0.0040, -0.0010, -0.0025, 0.0020, -0.0015,
                0.0005, 0.0010, -0.0020, 0.0003, -0.0005, 0.0004, 0.0012]

# Column ids used as the RNG "col" key.  Must match csrc/fm_gen.hip.
COL_RET = 0                  # retx noise
COL_CHAR0 = 1                # chars 1..14
COL_NAN0 = 32                # NaN draws per winsor column (32..46)
COL_ME = 64
COL_ME_NAN = 65
COL_EXCH = 66
COL_PRESENT = 67
COL_DY_ZERO = 68

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)
_GOLD = np.uint64(0x9E3779B97F4A7C15)
_GOLD2 = np.uint64(0xD1B54A32D192ED03)


def _mix(z):
    """splitmix64 finalizer on uint64 arrays (wrapping arithmetic)."""
    z = z.astype(np.uint64, copy=True)
    with np.errstate(over="ignore"):
        z ^= z >> np.uint64(30)
        z *= np.uint64(0xBF58476D1CE4E5B9)
        z ^= z >> np.uint64(27)
        z *= np.uint64(0x94D049BB133111EB)
        z ^= z >> np.uint64(31)
    return z


def cell_hash(seed, month, firm, col):
    """64-bit hash of (seed, month, firm, col); broadcasting uint64 arrays."""
    seed = np.asarray(seed, dtype=np.uint64)
    month = np.asarray(month, dtype=np.uint64)
    firm = np.asarray(firm, dtype=np.uint64)
    col = np.asarray(col, dtype=np.uint64)
    with np.errstate(over="ignore"):
        h = _mix(seed ^ (col << np.uint64(40)))
        h = _mix(h + month * _GOLD)
        h = _mix(h + firm * _GOLD2)
    return h


def hash_uniform(h):
    """uint64 hash -> double in (0,1): ((h>>11) + 0.5) * 2^-53 (exact)."""
    return ((h >> np.uint64(11)).astype(np.float64) + 0.5) * (2.0 ** -53)


def t2_from_uniform(u):
    """Student-t(2) inverse CDF: (2u-1)/sqrt(2u(1-u)); IEEE ops only, no FMA."""
    num = 2.0 * u - 1.0
    den = np.sqrt((2.0 * u) * (1.0 - u))
    return num / den


def synth_arrays(T, N, seed, nan_rate=0.02, present_rate=1.0, month0=0, nyse_rate=0.4):
    """Generate the panel as numpy arrays, months [month0, month0+T).

    Returns dict with keys: month (int64 month index, absolute), firm (int64),
    permno (int64), one float64 array per WINSOR_VARS entry, ``me`` (float64),
    ``nyse`` (bool).  Rows are month-major, firm ascending, rows absent with
    probability 1-present_rate removed.
    """
    months = np.arange(month0, month0 + T, dtype=np.uint64)[:, None]
    firms = np.arange(N, dtype=np.uint64)[None, :]
    nan_thr = np.uint64(int(nan_rate * 2.0 ** 64)) if nan_rate > 0 else np.uint64(0)

    def h(col):
        return cell_hash(seed, months, firms, col)

    out = {}
    zsum = None
    chars = {}
    for j, name in enumerate(CHAR_VARS):
        mu, sd = TABLE1_MOMENTS[name]
        t = t2_from_uniform(hash_uniform(h(COL_CHAR0 + j)))
        x = mu + sd * (t * 0.5)
        if name == "dy":
            zero = h(COL_DY_ZERO) < np.uint64(int(0.3 * 2.0 ** 64))
            x = np.where(zero, 0.0, x)
        chars[name] = x
        z = (x - mu) / sd
        term = RET_LOADINGS[j] * z
        zsum = term if zsum is None else zsum + term
    mu_r, sd_r = TABLE1_MOMENTS["retx"]
    tr = t2_from_uniform(hash_uniform(h(COL_RET)))
    ret = (mu_r + zsum) + sd_r * (tr * 0.5)
    cols = {"retx": ret, **chars}
    for k, name in enumerate(WINSOR_VARS):
        v = cols[name]
        if nan_rate > 0:
            v = np.where(h(COL_NAN0 + k) < nan_thr, np.nan, v)
        out[name] = v
    ume = hash_uniform(h(COL_ME))
    me = 10.0 / ume
    if nan_rate > 0:
        me = np.where(h(COL_ME_NAN) < np.uint64(int(0.25 * nan_rate * 2.0 ** 64)), np.nan, me)
    out["me"] = me
    out["nyse"] = h(COL_EXCH) < np.uint64(int(nyse_rate * 2.0 ** 64))
    mgrid = np.broadcast_to(months.astype(np.int64), (T, N))
    fgrid = np.broadcast_to(firms.astype(np.int64), (T, N))
    out["month"] = mgrid
    out["firm"] = fgrid
    if present_rate < 1.0:
        keep = h(COL_PRESENT) < np.uint64(int(present_rate * 2.0 ** 64))
    else:
        keep = np.ones((T, N), dtype=bool)
    flat = keep.reshape(-1)
    res = {k: np.ascontiguousarray(np.broadcast_to(v, (T, N)).reshape(-1)[flat]) for k, v in out.items()}
    res["permno"] = res["firm"] + 10000
    return res


def month_end_dates(month_idx, start="1964-01-31"):
    """Month index -> datetime64[ns] month-end dates starting at ``start``."""
    import pandas as pd
    base = pd.Timestamp(start)
    month_idx = np.asarray(month_idx)
    uniq = np.unique(month_idx)
    dates = pd.DatetimeIndex([base + pd.offsets.MonthEnd(int(m)) for m in uniq])
    return dates.values.astype("datetime64[ns]")[np.searchsorted(uniq, month_idx)]


def synth_frame(T, N, seed, nan_rate=0.02, present_rate=1.0, month0=0, shuffle=False):
    """The panel as a reference-shaped pandas DataFrame.

    Columns: mthcaldt (datetime64 month-end), permno, primaryexch ('N'/'Q'), me, and
    the 15 notebook variables.  ``shuffle=True`` permutes the rows (the reference's
    functions sort internally).
    """
    import pandas as pd
    a = synth_arrays(T, N, seed, nan_rate=nan_rate, present_rate=present_rate, month0=month0)
    df = pd.DataFrame({
        "mthcaldt": month_end_dates(a["month"]),
        "permno": a["permno"],
        "primaryexch": np.where(a["nyse"], "N", "Q"),
        "me": a["me"],
    })
    for name in WINSOR_VARS:
        df[name] = a[name]
    if shuffle:
        rng = np.random.default_rng(seed + 1)
        df = df.iloc[rng.permutation(len(df))].reset_index(drop=True)
    return df

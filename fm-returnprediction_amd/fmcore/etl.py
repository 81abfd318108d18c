"""Panel ETL on the device: the annual -> monthly Compustat expansion.

expand_monthly() plans the output of the reference's expand_compustat_annual_to_monthly
(src/transform_compustat.py:101-172) on the host -- group codes, month codes and each
group's output month range, which need the calendar -- and runs the gather on the device
(fm_ffill_expand): every output row finds its source record by binary search and copies the
FP64 columns; other dtypes are gathered on the host by the returned source indices.
"""
from __future__ import annotations

import numpy as np
import pandas as pd
import torch

from . import _lib as L
from . import engine as E


def month_code(dates) -> np.ndarray:
    """year * 12 + month - 1 of each date (datetime64 input)."""
    d = pd.DatetimeIndex(dates)
    return (d.year.to_numpy().astype(np.int64) * 12 + d.month.to_numpy() - 1).astype(np.int32)


def code_to_month_end(codes) -> np.ndarray:
    codes = np.asarray(codes, dtype=np.int64)
    y, m = codes // 12, codes % 12 + 1
    first = pd.to_datetime({"year": y, "month": m, "day": np.ones_like(y)})
    return (first + pd.offsets.MonthEnd(0)).to_numpy(dtype="datetime64[ns]")


def expand_monthly(group_codes, dates, float_cols, extend_months=12, device=None):
    """Device forward-fill expansion.

    group_codes: int64 [n] group id of each record; dates: datetime64 [n] report dates;
    float_cols: list of float64 [n] arrays.  Records need not be sorted.  Returns
    (out_group_code [m], out_month_end [m] datetime64, out_cols [list of float64 [m]],
    src [m] int64 index into the ORIGINAL records)."""
    device = device or E.require_device()
    g = np.asarray(group_codes)
    # one unit for every date quantity below (Parquet / to_datetime give [us] or [s]; the
    # 12-month clip compares against max_all.value, which is always ns)
    dates = pd.DatetimeIndex(dates).as_unit("ns")
    if dates.hasnans:
        raise ValueError("report dates contain NaT")
    if (g < 0).any():
        raise ValueError("group codes must be >= 0 (drop rows with a missing id first)")
    n = len(g)
    if n == 0:
        return g[:0], np.zeros(0, "datetime64[ns]"), [np.zeros(0) for _ in float_cols], np.zeros(0, np.int64)
    order = np.lexsort((dates.asi8, g))           # sort by (group, date)
    gs = g[order]
    ds = dates[order]
    mc = month_code(ds)
    starts = np.flatnonzero(np.r_[True, gs[1:] != gs[:-1]])
    rec_off = np.r_[starts, n].astype(np.int64)
    last = rec_off[1:] - 1
    # pandas: date_range(first, min(max over all, last + 12 months), freq="M")
    max_all = ds.max()
    ext = ds[last] + pd.DateOffset(months=extend_months)
    ext = pd.DatetimeIndex(np.minimum(ext.asi8, max_all.value))
    end_code = month_code(ext) - (~ext.is_month_end).astype(np.int32)
    start_code = mc[starts]
    counts = np.maximum(end_code.astype(np.int64) - start_code + 1, 0)
    out_off = np.zeros(len(starts) + 1, dtype=np.int64)
    np.cumsum(counts, out=out_off[1:])
    m = int(out_off[-1])
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a, dtype=dt)).to(device)  # noqa: E731
    C = len(float_cols)
    vals = torch.from_numpy(np.stack([np.asarray(c, dtype=np.float64)[order] for c in float_cols])
                            if C else np.zeros((0, n))).to(device)
    out_vals = torch.empty((C, max(m, 1)), dtype=torch.float64, device=device)
    out_month = torch.empty(max(m, 1), dtype=torch.int32, device=device)
    out_src = torch.empty(max(m, 1), dtype=torch.int64, device=device)
    d_rec_off, d_mc, d_out_off = t(rec_off, np.int64), t(mc, np.int32), t(out_off, np.int64)
    L.call("fm_ffill_expand", d_rec_off.data_ptr(), d_mc.data_ptr(), d_out_off.data_ptr(), len(starts), m,
           vals.data_ptr() if C else None, vals.stride(0) if C else 0, C, out_vals.data_ptr(),
           out_vals.stride(0), out_month.data_ptr(), out_src.data_ptr(), E._stream())
    src_sorted = out_src[:m].cpu().numpy()
    months = out_month[:m].cpu().numpy()
    cols = [out_vals[c, :m].cpu().numpy() for c in range(C)]
    out_group = np.repeat(gs[starts], counts)
    return out_group, code_to_month_end(months), cols, order[src_sorted]


def join_pairs(left_keys, right_keys, device=None):
    """Equality join on one- or two-part int64 keys (fm_sorted_join): returns (li, rj) index
    arrays into the left and right frames, in pandas merge order -- left rows in order, each
    with its matches in the right frame's order."""
    device = device or E.require_device()
    lk = [np.ascontiguousarray(k, dtype=np.int64) for k in left_keys]
    rk = [np.ascontiguousarray(k, dtype=np.int64) for k in right_keys]
    nl, nr = len(lk[0]), len(rk[0])
    if nl == 0 or nr == 0:
        return np.zeros(0, np.int64), np.zeros(0, np.int64)
    order = np.lexsort(tuple(reversed(rk)))   # stable: equal keys keep the right order
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)  # noqa: E731
    dl = [t(k) for k in lk]
    dr = [t(k[order]) for k in rk]
    lo = torch.empty(nl, dtype=torch.int64, device=device)
    hi = torch.empty_like(lo)
    two = len(lk) == 2
    L.call("fm_sorted_join", dl[0].data_ptr(), dl[1].data_ptr() if two else None, nl, dr[0].data_ptr(),
           dr[1].data_ptr() if two else None, nr, lo.data_ptr(), hi.data_ptr(), E._stream())
    lo, hi = lo.cpu().numpy(), hi.cpu().numpy()
    cnt = hi - lo
    li = np.repeat(np.arange(nl, dtype=np.int64), cnt)
    start = np.repeat(lo - (np.cumsum(cnt) - cnt), cnt)
    rj = order[start + np.arange(len(li), dtype=np.int64)]
    return li, rj

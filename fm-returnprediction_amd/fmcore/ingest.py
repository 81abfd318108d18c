"""Arrow / Parquet ingest of the month-sorted SoA panel.

The reference loads its CRSP-Compustat panel through pandas (`pd.read_parquet` in the
`pull_*` / `load_*` helpers, then `get_factors`, src/calc_Lewellen_2014.py:531-575) and the
drop-in marshals DataFrame columns into `engine.panel_from_arrays`.  This module builds the
same `DevicePanel` without a DataFrame:

* columns come out of the Arrow buffers directly (zero-copy for null-free float64 chunks;
  float nulls become NaN, as pandas reads them);
* the month segmentation (`engine.month_segments` semantics: sorted factorize, stable
  order, CSR offsets; null dates dropped) runs on the date column's datetime64 view, the
  stable sort as a 16-bit radix sort;
* each column is copied chunk by chunk from the Arrow buffers into one pinned host block
  (one copy per value) and sent with a single H2D copy, then
  permuted month-major on the device (the same gather `panel_from_arrays` does).

The result is bit-identical to `panel_from_arrays` on the equivalent DataFrame columns
(tests/test_host.py, tests/test_gpu_parity.py).
"""
from typing import Optional, Sequence

import numpy as np

from . import engine as E


def _read(source, columns):
    import pyarrow as pa
    if isinstance(source, pa.Table):
        return source
    import pyarrow.parquet as pq
    return pq.read_table(source, columns=list(columns), memory_map=True)


def _f64(col) -> np.ndarray:
    """float64 numpy view of an Arrow column (nulls -> NaN)."""
    import pyarrow as pa
    import pyarrow.compute as pc
    if col.type != pa.float64():
        col = pc.cast(col, pa.float64())
    if isinstance(col, pa.ChunkedArray) and col.num_chunks == 1:
        col = col.chunk(0)
    return np.asarray(col.to_numpy(zero_copy_only=False), dtype=np.float64)


def _fill(dst: np.ndarray, col) -> None:
    """Copy an Arrow column chunk by chunk into `dst` (float64, nulls -> NaN): one copy per
    value, straight from the Arrow buffers into the pinned stage."""
    import pyarrow as pa
    import pyarrow.compute as pc
    if col.type != pa.float64():
        col = pc.cast(col, pa.float64())
    chunks = col.chunks if isinstance(col, pa.ChunkedArray) else [col]
    off = 0
    for ch in chunks:
        m = len(ch)
        dst[off:off + m] = ch.to_numpy(zero_copy_only=False)
        off += m


def month_order(labels):
    """engine.month_segments (its stable sort is a 16-bit radix sort when T < 32767)."""
    return E.month_segments(labels)


def arrow_host_columns(source, value_cols: Sequence[str], date_col: str = "mthcaldt",
                       me_col: Optional[str] = None, exch_col: Optional[str] = None,
                       exch_value: str = "N"):
    """Host half of the ingest: (arrays [original row order], labels, me, nyse).

    `nyse` is `exch_col == exch_value` with nulls False, as
    `(df["primaryexch"] == "N")` is on the pandas side (`get_subsets`, src/calc_Lewellen_2014.py:44-112)."""
    import pyarrow.compute as pc
    need = list(value_cols) + [date_col] + [c for c in (me_col, exch_col) if c]
    tab = _read(source, need)
    arrays = [_f64(tab.column(c)) for c in value_cols]
    labels = tab.column(date_col).to_numpy()
    me = _f64(tab.column(me_col)) if me_col else None
    nyse = None
    if exch_col:
        eq = pc.fill_null(pc.equal(tab.column(exch_col), exch_value), False)
        nyse = np.asarray(eq.to_numpy(zero_copy_only=False), dtype=np.uint8)
    return arrays, labels, me, nyse


def panel_from_arrow(source, value_cols: Sequence[str], date_col: str = "mthcaldt",
                     me_col: Optional[str] = None, exch_col: Optional[str] = None,
                     exch_value: str = "N", device=None, layout="f64") -> "E.DevicePanel":
    """A pyarrow Table or a Parquet path -> month-sorted DevicePanel (one pinned H2D copy),
    in ``layout`` ("f64"; "planes": the split high / low-word layout only, gathered from the
    raw words on the device; "both")."""
    import pyarrow.compute as pc
    import torch
    device = device or E.require_device()
    need = list(value_cols) + [date_col] + [c for c in (me_col, exch_col) if c]
    tab = _read(source, need)
    _, uniq, order, seg_off = month_order(tab.column(date_col).to_numpy())
    n = tab.num_rows
    extra = 1 if me_col else 0
    stage = torch.empty((len(value_cols) + extra, n), dtype=torch.float64, pin_memory=True)
    host = stage.numpy()
    for i, c in enumerate(value_cols):
        _fill(host[i], tab.column(c))
    if me_col:
        _fill(host[len(value_cols)], tab.column(me_col))
    nyse = None
    if exch_col:
        eq = pc.fill_null(pc.equal(tab.column(exch_col), exch_value), False)
        nyse = np.asarray(eq.to_numpy(zero_copy_only=False), dtype=np.uint8)
    C = len(value_cols)
    raw = stage.to(device, non_blocking=True)
    perm = torch.from_numpy(order.astype(np.int64)).to(device, non_blocking=True)
    cols, planes = E.gather_layout(raw[:C], perm, layout)
    me_t = raw[C].index_select(0, perm) if me_col else None
    nyse_t = None
    if nyse is not None:
        nyse_t = torch.from_numpy(nyse).to(device).index_select(0, perm)
    panel = E.DevicePanel(cols=cols, names=list(value_cols),
                          seg_off=torch.from_numpy(seg_off).to(device), seg_off_h=seg_off,
                          months=uniq, me=me_t, nyse=nyse_t, order=order, planes=planes)
    if cols is not None and planes is not None:
        panel.planes_version = cols._version
    torch.cuda.current_stream().synchronize()   # the pinned stage must outlive the copy
    return panel

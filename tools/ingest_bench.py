"""Host->HBM ingest timing at the bench panel size (600 months x 5,000 firms, retx + 14
characteristics + me + primaryexch): a Parquet file written to /tmp,
then (a) pandas: pd.read_parquet -> DataFrame columns -> engine.panel_from_arrays (the
drop-in's path for a frame) and (b) fmcore.ingest.panel_from_arrow on the same file.
Prints one JSON line.  python tools/ingest_bench.py"""
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "fm-returnprediction_amd"), ROOT]

import numpy as np  # noqa: E402
import pandas as pd  # noqa: E402
import pyarrow as pa  # noqa: E402
import pyarrow.parquet as pq  # noqa: E402
import torch  # noqa: E402

from fmcore import engine as E  # noqa: E402
from fmcore import ingest  # noqa: E402


def main(T=600, F=5000, C=15, reps=3):
    dev = E.require_device()
    rng = np.random.default_rng(0)
    n = T * F
    months = pd.date_range("1964-01-31", periods=T, freq="ME")
    cols = ["retx"] + [f"x{k}" for k in range(C - 1)]
    data = {"mthcaldt": np.repeat(months.values, F)}
    for c in cols:
        v = rng.standard_normal(n)
        v[rng.random(n) < 0.02] = np.nan
        data[c] = v
    data["me"] = np.exp(rng.normal(5, 2, n))
    data["primaryexch"] = np.where(rng.random(n) < 0.4, "N", "Q")
    perm = rng.permutation(n)                       # file rows not month-sorted
    tab = pa.table({k: v[perm] for k, v in data.items()})
    path = os.path.join(tempfile.gettempdir(), "fm_ingest_bench.parquet")
    pq.write_table(tab, path, compression=None)
    del tab, data

    def frame_path():
        df = pd.read_parquet(path)
        p = E.panel_from_arrays([df[c].to_numpy(dtype=np.float64) for c in cols], cols,
                                df["mthcaldt"].values, me=df["me"].to_numpy(),
                                nyse=(df["primaryexch"] == "N").to_numpy().astype(np.uint8))
        torch.cuda.synchronize()
        return p

    def arrow_path():
        p = ingest.panel_from_arrow(path, cols, me_col="me", exch_col="primaryexch")
        torch.cuda.synchronize()
        return p

    out = {"rows": n, "cols": C + 2, "file_bytes": os.path.getsize(path)}
    for name, fn in (("pandas_frame", frame_path), ("arrow", arrow_path)):
        fn()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        out[name + "_s"] = min(ts)
        out[name + "_rows_per_s"] = n / min(ts)
    a, b = frame_path(), arrow_path()
    out["identical"] = bool(torch.equal(torch.nan_to_num(a.cols, 7.0), torch.nan_to_num(b.cols, 7.0)))
    os.remove(path)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

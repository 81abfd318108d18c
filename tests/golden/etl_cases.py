"""Input frame for the annual -> monthly Compustat expansion goldens (gen_etl_goldens.py)."""
import numpy as np
import pandas as pd


def comp_annual(seed=31):
    """gvkey groups with 1..12 annual records, multi-year gaps, month-end report dates (the
    reference's add_report_date output) plus one group with mid-month dates, NaN values and
    an int column; rows shuffled (the reference sorts)."""
    rng = np.random.default_rng(seed)
    rows = []
    for k in range(40):
        gv = f"{1000 + 7 * k:06d}"
        nrec = 1 + int(rng.integers(0, 12))
        y0 = 1960 + int(rng.integers(0, 40))
        years = np.sort(rng.choice(np.arange(y0, y0 + 30), size=nrec, replace=False))
        fye = int(rng.integers(1, 13))
        for y in years:
            dd = pd.Timestamp(year=int(y), month=fye, day=1) + pd.offsets.MonthEnd(0)
            rd = dd + pd.offsets.MonthEnd(4)
            if k == 5:                                   # mid-month report dates
                rd = rd - pd.Timedelta(days=10)
            rows.append({"gvkey": gv, "datadate": dd, "fyear": int(y), "report_date": rd,
                         "be": rng.standard_normal() * 100 if rng.random() > 0.1 else np.nan,
                         "at": abs(rng.standard_normal()) * 1000, "sale": rng.standard_normal() * 50,
                         "count": int(rng.integers(0, 40))})
    df = pd.DataFrame(rows)
    return df.iloc[rng.permutation(len(df))].reset_index(drop=True)


def link_inputs(comp_monthly, seed=32):
    """CRSP monthly rows, and a CCM link table for comp_monthly's gvkeys: one or two links per
    gvkey over different windows (some open-ended: NaT linkenddt), one gvkey with no link,
    one permno linked to two gvkeys over time; CRSP carries an overlapping column name
    ('datadate') to exercise the _x / _y suffixes."""
    rng = np.random.default_rng(seed)
    gvs = sorted(comp_monthly["gvkey"].unique())
    links = []
    for k, gv in enumerate(gvs):
        if k == 3:
            continue                                    # no link: dropped by the window filter
        permno = 10000 + k if k != 7 else 10000 + 6     # permno 10006 linked to two gvkeys
        d = comp_monthly.loc[comp_monthly["gvkey"] == gv, "fund_date"]
        lo, hi = d.min(), d.max()
        mid = lo + (hi - lo) / 2
        if rng.random() < 0.5:
            links.append({"gvkey": gv, "permno": permno, "linkdt": lo - pd.Timedelta(days=40),
                          "linkenddt": pd.NaT if rng.random() < 0.5 else mid})
        else:
            links.append({"gvkey": gv, "permno": permno, "linkdt": lo, "linkenddt": mid})
            links.append({"gvkey": gv, "permno": permno + 500, "linkdt": mid + pd.Timedelta(days=1),
                          "linkenddt": pd.NaT})
    ccm = pd.DataFrame(links)
    ccm = ccm.iloc[rng.permutation(len(ccm))].reset_index(drop=True)
    # CRSP months stop before any plausible run date: the reference fills open-ended links
    # with pd.to_datetime("today"), so merged rows past the run date would make the fixture
    # depend on the wall clock (every jdate here is <= 2019-12 < today)
    months = pd.date_range("1959-01-31", "2019-12-31", freq="ME")
    rows = []
    for p in sorted(set(ccm["permno"])):
        sel = months[rng.random(len(months)) < 0.6]
        rows.append(pd.DataFrame({"permno": p, "jdate": sel, "me": rng.random(len(sel)) * 1e3,
                                  "retx": rng.standard_normal(len(sel)) * 0.1,
                                  "datadate": sel - pd.Timedelta(days=1)}))
    crsp = pd.concat(rows, ignore_index=True)
    crsp = crsp.iloc[rng.permutation(len(crsp))].reset_index(drop=True)
    return crsp, ccm


def unit_variants(df):
    """The reference's expansion over inputs pandas 2 produces from Parquet / to_datetime:
    report dates in datetime64[us] and [s], and a frame with missing gvkeys (groupby drops
    them).  {name: frame}."""
    out = {}
    for unit in ("us", "s"):
        d = df.copy()
        d["report_date"] = d["report_date"].astype(f"datetime64[{unit}]")
        out[unit] = d
    d = df.copy()
    d.loc[d.index[::17], "gvkey"] = None
    out["nakey"] = d
    return out


def frame_from_golden(g, prefix, datetime_cols, gvkey=True):
    """Rebuild a frame stored by gen_etl_goldens.arrays (gvkey back to 6-digit strings,
    int64 ns back to datetime64, NaT included)."""
    cols = [k[len(prefix):] for k in g.files if k.startswith(prefix) and k != prefix + "columns"
            and k != prefix + "dtypes"]
    out = {}
    for c in cols:
        v = g[prefix + c]
        if c == "gvkey" and gvkey:
            v = np.array([f"{int(x):06d}" for x in v], dtype=object)
        elif c in datetime_cols:
            v = v.astype("datetime64[ns]")
        out[c] = v
    return pd.DataFrame(out)


def assert_frame_matches(out, g, prefix):
    """Columns, dtypes (when stored) and every value of `out` against a stored frame."""
    assert list(out.columns) == [str(c) for c in g[prefix + "columns"]]
    if prefix + "dtypes" in g.files:
        assert [str(t) for t in out.dtypes] == [str(t) for t in g[prefix + "dtypes"]]
    for c in out.columns:
        a = out[c].to_numpy()
        if c == "gvkey":
            a = np.array([-1 if x is None else int(x) for x in a], dtype=np.int64)
        elif np.issubdtype(out[c].dtype, np.datetime64):
            a = out[c].to_numpy(dtype="datetime64[ns]").astype(np.int64)
        assert np.array_equal(a, g[prefix + c], equal_nan=a.dtype.kind == "f"), c

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

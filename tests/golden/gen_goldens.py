"""Generate golden vectors by running the REFERENCE hot path (this container only).

Run with the oracle interpreter (numpy 1.26.4 = the reference's pin, statsmodels 0.12.2):

    PYTHONDONTWRITEBYTECODE=1 /opt/conda/bin/python3.9 tests/golden/gen_goldens.py

It imports ``/root/reference/src/regressions.py`` and AST-extracts ``winsorize``,
``get_subsets``, ``build_table_2`` and ``create_figure_1`` from
``/root/reference/src/calc_Lewellen_2014.py`` (that module's top-level imports need
polars/decouple/wrds, which are absent), following SURVEY.md Appendix A.  Nothing from the
reference is copied into the repo: only the input panels (tests/golden/cases.py) and the
reference's outputs are written, as .npz/.json fixtures next to this script.  The GPU box
never sees /root/reference; tests read only these fixtures.
"""
import ast
import hashlib
import json
import os
import sys
import types
import warnings

sys.dont_write_bytecode = True
warnings.filterwarnings("ignore")

import numpy as np  # noqa: E402
import pandas as pd  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/src"


# --- compatibility shims --------------------------------------------
class _MachAr:
    eps = np.finfo(float).eps


np.MachAr = _MachAr
for _n in ("Int64Index", "UInt64Index", "Float64Index"):
    setattr(pd, _n, pd.Index)
import statsmodels.api as sm  # noqa: E402
import statsmodels.tsa.tsatools as tt  # noqa: E402

_px = types.SimpleNamespace(**{k: getattr(pd, k) for k in dir(pd) if not k.startswith("__")})
_px.concat = lambda objs, *a, **kw: pd.concat(objs, **({"axis": a[0]} if a else {}), **kw)
tt.pd = _px

sys.path.insert(0, REF)
import regressions as R  # noqa: E402

sys.path.insert(0, HERE)
import cases  # noqa: E402


class _Ax:
    def __init__(self):
        self.lines = []

    def plot(self, x, y, label=None):
        self.lines.append((np.asarray(x), np.asarray(y, dtype=float), label))

    def __getattr__(self, name):
        return lambda *a, **k: None


class RecordingPlt:
    def __init__(self):
        self.axes = None

    def subplots(self, *a, **k):
        self.axes = [_Ax(), _Ax()]
        return None, self.axes

    def tight_layout(self, *a, **k):
        pass


class RecordingSM:
    """sm proxy: records every fitted OLS result's params (create_figure_1 internals)."""

    def __init__(self):
        self.records = []
        self.add_constant = sm.add_constant

    def OLS(self, *a, **k):
        mod = sm.OLS(*a, **k)
        rec = self.records
        fit0 = mod.fit

        def fit(*fa, **fk):
            res = fit0(*fa, **fk)
            rec.append(res.params)
            return res

        mod.fit = fit
        return mod


def load_calc(plt_obj, sm_obj):
    src = open(os.path.join(REF, "calc_Lewellen_2014.py")).read()
    keep = {"winsorize", "get_subsets", "build_table_1", "build_table_2", "create_figure_1"}
    fns = [n for n in ast.parse(src).body if isinstance(n, ast.FunctionDef) and n.name in keep]
    ns = dict(np=np, pd=pd, sm=sm_obj, OUTPUT_DIR=None, Union=__import__("typing").Union,
              Path=__import__("pathlib").Path, plt=plt_obj,
              run_monthly_cs_regressions=R.run_monthly_cs_regressions,
              fama_macbeth_summary=R.fama_macbeth_summary)
    exec(compile(ast.Module(fns, []), "calc_Lewellen_2014.py", "exec"), ns)
    return ns


def frame_arrays(df, prefix):
    out = {prefix + "index": df.index.values.astype(np.int64)}
    for c in df.columns:
        v = df[c].values
        if c == "mthcaldt":
            v = v.astype("datetime64[ns]").astype(np.int64)
        elif c == "primaryexch":
            v = (v == "N").astype(np.int8)
        elif v.dtype == bool:
            v = v.astype(np.int8)
        out[prefix + c] = np.asarray(v)
    return out


def sha(arrs):
    h = hashlib.sha256()
    for a in arrs:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def gen_wins():
    df = cases.wins_panel()
    ns = load_calc(RecordingPlt(), sm)
    out = ns["winsorize"](df, cases.WINSOR_VARS, 1, 99)
    d = {}
    d.update(frame_arrays(df, "in_"))
    d.update(frame_arrays(out, "out_"))
    # per (month, var) cuts with the reference's inner calls (src/calc_Lewellen_2014.py:519-523)
    srt = df.sort_values(["mthcaldt", "permno"])
    months = np.sort(srt["mthcaldt"].unique())
    lo = np.full((len(cases.WINSOR_VARS), len(months)), np.nan)
    hi = np.full_like(lo, np.nan)
    nv = np.zeros(lo.shape, dtype=np.int64)
    for j, v in enumerate(cases.WINSOR_VARS):
        for t, m in enumerate(months):
            vals = srt.loc[srt.mthcaldt == m, v].dropna()
            nv[j, t] = len(vals)
            if len(vals) >= 5:
                lo[j, t] = np.percentile(vals, 1)
                hi[j, t] = np.percentile(vals, 99)
    d.update(cut_lo=lo, cut_hi=hi, cut_n=nv)
    np.savez_compressed(os.path.join(HERE, "wins.npz"), **d)


def fm_results(ns, subsets, models):
    arrs, meta = {}, {}
    for mname, xs in models.items():
        for sname, sdf in subsets.items():
            res = R.run_monthly_cs_regressions(sdf, "retx", xs, "mthcaldt")
            key = f"{mname}|{sname}"
            arrs[key + "|date"] = res["mthcaldt"].values.astype("datetime64[ns]").astype(np.int64) \
                if len(res) else np.zeros(0, np.int64)
            arrs[key + "|N"] = res["N"].values.astype(np.int64) if len(res) else np.zeros(0, np.int64)
            arrs[key + "|R2"] = res["R2"].values if len(res) else np.zeros(0)
            for x in xs:
                arrs[key + "|slope_" + x] = res["slope_" + x].values if len(res) else np.zeros(0)
            summ = R.fama_macbeth_summary(res, xs, "mthcaldt", nw_lags=4) if len(res) else None
            meta[key] = None if summ is None else {k: (None if pd.isna(v) else float(v)) for k, v in summ.items()}
            meta[key + "|columns"] = list(res.columns)
    return arrs, meta


def gen_fm():
    df = cases.fm_panel()
    ns = load_calc(RecordingPlt(), sm)
    w = ns["winsorize"](df, cases.WINSOR_VARS, 1, 99)
    subsets = ns["get_subsets"](w)
    d = frame_arrays(df, "in_")
    allst = subsets["All stocks"]
    d.update(frame_arrays(allst[["mthcaldt", "permno", "me_20", "me_50", "is_all_but_tiny", "is_large"]], "sub_"))
    for s in cases.SUBSETS:
        d["len|" + s] = np.array([len(subsets[s])])
    arrs, meta = fm_results(ns, subsets, cases.MODELS)
    d.update(arrs)
    t2 = ns["build_table_2"](subsets, cases.VARIABLES_DICT)
    meta["table2"] = {
        "index": [list(i) for i in t2.index],
        "columns": [list(c) for c in t2.columns],
        "values": [[str(x) for x in row] for row in t2.values.tolist()],
    }
    np.savez_compressed(os.path.join(HERE, "fm.npz"), **d)
    json.dump(meta, open(os.path.join(HERE, "fm.json"), "w"), indent=1)


def gen_fig1(df=None, out="fig1.npz"):
    df = cases.fig1_panel() if df is None else df
    plt_obj, sm_obj = RecordingPlt(), RecordingSM()
    ns = load_calc(plt_obj, sm_obj)
    w = ns["winsorize"](df, cases.WINSOR_VARS, 1, 99)
    subsets = ns["get_subsets"](w)
    # monthly params: recreate the same loop grouping to know which months/subsets they belong to
    ns["create_figure_1"](subsets, save_plot=False, output_dir=None)
    d = {"in_sha": np.frombuffer(sha([df[c].values for c in cases.WINSOR_VARS + ["me"]]).encode(), dtype=np.uint8)}
    recs = sm_obj.records
    k = 0
    for si, sname in enumerate(["All stocks", "Large stocks"]):
        sub = subsets[sname].sort_values(["mthcaldt", "permno"]).dropna(subset=["retx"] + cases.FIG1_VARS)
        months = []
        for mth, grp in sub.groupby("mthcaldt"):
            if len(grp) < len(cases.FIG1_VARS) + 1:
                continue
            months.append(mth)
        params = np.array([np.asarray(recs[k + i][["const"] + cases.FIG1_VARS], dtype=float)
                           for i in range(len(months))])
        k += len(months)
        tag = "all" if si == 0 else "large"
        d[tag + "|date"] = np.array(months, dtype="datetime64[ns]").astype(np.int64)
        d[tag + "|params"] = params
        ax = plt_obj.axes[si]
        d[tag + "|rolling_plotted"] = np.stack([ln[1] for ln in ax.lines], axis=1)
        d[tag + "|plot_x"] = np.asarray(ax.lines[0][0]).astype("datetime64[ns]").astype(np.int64)
    np.savez_compressed(os.path.join(HERE, out), **d)


def gen_mid():
    df = cases.mid_panel()
    d = {"in_sha": np.frombuffer(sha([df[c].values for c in cases.WINSOR_VARS + ["me"]]).encode(), dtype=np.uint8)}
    meta = {}
    for mname in ("M2", "M3"):
        xs = cases.MODELS[mname]
        res = R.run_monthly_cs_regressions(df, "retx", xs, "mthcaldt")
        d[mname + "|N"] = res["N"].values.astype(np.int64)
        d[mname + "|R2"] = res["R2"].values
        d[mname + "|slopes"] = res[["slope_" + x for x in xs]].values
        d[mname + "|date"] = res["mthcaldt"].values.astype("datetime64[ns]").astype(np.int64)
        s = R.fama_macbeth_summary(res, xs, "mthcaldt", nw_lags=4)
        meta[mname] = {k: float(v) for k, v in s.items()}
    np.savez_compressed(os.path.join(HERE, "mid.npz"), **d)
    json.dump(meta, open(os.path.join(HERE, "mid.json"), "w"), indent=1)


def gen_edge(case_list=None, out="edge"):
    d, meta = {}, {}
    for name, df, xs in (cases.edge_cases() if case_list is None else case_list):
        d.update(frame_arrays(df, name + "|in_"))
        try:
            res = R.run_monthly_cs_regressions(df, "retx", xs, "mthcaldt")
            meta[name] = {"error": None, "columns": list(res.columns)}
            d.update(frame_arrays(res, name + "|out_"))
            try:
                s = R.fama_macbeth_summary(res, xs, "mthcaldt", nw_lags=4)
                meta[name]["summary"] = {k: (None if pd.isna(v) else float(v)) for k, v in s.items()}
                meta[name]["summary_keys"] = list(s.index)
            except Exception as e:  # pragma: no cover
                meta[name]["summary_error"] = type(e).__name__
        except Exception as e:
            meta[name] = {"error": type(e).__name__, "message": str(e)}
    np.savez_compressed(os.path.join(HERE, out + ".npz"), **d)
    json.dump(meta, open(os.path.join(HERE, out + ".json"), "w"), indent=1)


def gen_nw():
    out = []
    for x in cases.nw_series():
        for lags in (0, 1, 2, 4, 6):
            v = R.newey_west_mean_se(x, lags)
            out.append({"x": [float(a) for a in x], "lags": lags,
                        "se": None if np.isnan(v) else float(v)})
    json.dump(out, open(os.path.join(HERE, "nw.json"), "w"))


def gen_table1():
    """build_table_1 (src/calc_Lewellen_2014.py:577-670) on the winsorize panel, whose
    inf values survive winsorizing (NaN cuts) and exercise the inf->NaN replacement."""
    df = cases.wins_panel()
    ns = load_calc(RecordingPlt(), sm)
    w = ns["winsorize"](df, cases.WINSOR_VARS, 1, 99)
    subsets = ns["get_subsets"](w)
    vd = dict(cases.VARIABLES_DICT)
    vd["Missing column"] = "not_a_column"
    t1 = ns["build_table_1"](subsets, vd)
    meta = {"index": list(t1.index), "columns": [list(c) for c in t1.columns],
            "values": [[None if pd.isna(x) else float(x) for x in row] for row in t1.values.tolist()],
            "dtypes": [str(t) for t in t1.dtypes]}
    json.dump(meta, open(os.path.join(HERE, "table1.json"), "w"), indent=1)


def gen_pct():
    arrs = cases.percentile_arrays()
    qs = [1, 99, 20, 50, 0, 100, 37.5]
    off = np.cumsum([0] + [len(a) for a in arrs])
    res = np.array([[np.percentile(a, q) for q in qs] for a in arrs])
    # pandas groupby.quantile lerp (src/calc_Lewellen_2014.py:74-82)
    g = np.repeat(np.arange(len(arrs)), [len(a) for a in arrs])
    s = pd.Series(np.concatenate(arrs))
    fin = np.isfinite(s.values)   # groupby.quantile with inf can produce inf-inf; keep finite
    pq = s[fin].groupby(g[fin]).quantile([0.2, 0.5]).unstack(level=1)
    pdq = np.full((len(arrs), 2), np.nan)
    pdq[pq.index.values] = pq.values
    np.savez_compressed(os.path.join(HERE, "pct.npz"), values=np.concatenate(arrs), offsets=off,
                        qs=np.array(qs, dtype=float), np_percentile=res, pd_quantile=pdq)


CHAR_FUNCS = ["calc_log_size", "calc_log_bm", "calc_return_12_2", "calc_accruals", "calc_roa",
              "calc_log_assets_growth", "calc_dy", "calc_log_return_13_36", "calc_log_issues_12",
              "calc_log_issues_36", "calc_debt_price", "calc_sales_price"]


def load_chars():
    """The firm-axis characteristic functions of get_factors (src/calc_Lewellen_2014.py:137-466),
    AST-extracted like load_calc (the module's polars/wrds imports are absent here)."""
    src = open(os.path.join(REF, "calc_Lewellen_2014.py")).read()
    keep = set(CHAR_FUNCS) | {"calc_std_12"}
    fns = [n for n in ast.parse(src).body if isinstance(n, ast.FunctionDef) and n.name in keep]
    ns = dict(np=np, pd=pd)
    exec(compile(ast.Module(fns, []), "calc_Lewellen_2014.py", "exec"), ns)
    return ns


def gen_chars():
    """Each calc_* on a scrambled raw panel (groupby order = frame order), the get_factors
    chain (sorted by permno, date; :531-548 without the polars beta), and calc_std_12."""
    ns = load_chars()
    d = {}
    base = cases.raw_monthly_panel()
    daily = cases.raw_daily_panel()
    d["in_index"] = base.index.values.astype(np.int64)
    d["in_permno"] = base["permno"].values.astype(np.int64)
    d["in_mthcaldt"] = base["mthcaldt"].values.astype("datetime64[ns]").astype(np.int64)
    for k in cases.RAW_FIELDS:
        d["in_" + k] = base[k].values.astype(np.float64)
    d["din_index"] = daily.index.values.astype(np.int64)
    d["din_permno"] = daily["permno"].values.astype(np.int64)
    d["din_dlycaldt"] = daily["dlycaldt"].values.astype("datetime64[ns]").astype(np.int64)
    d["din_retx"] = daily["retx"].values.astype(np.float64)
    for fn, col in zip(CHAR_FUNCS, cases.CHAR_NAMES):
        out = ns[fn](base.copy())
        d[f"single_{col}_index"] = out.index.values.astype(np.int64)
        d[f"single_{col}"] = out[col].values.astype(np.float64)
        d[f"single_{col}_columns"] = np.array(list(out.columns))
    # get_factors order (:533-548)
    cc = base.sort_values(["permno", "mthcaldt"])
    dd = daily.sort_values(["permno", "dlycaldt"])
    for fn in CHAR_FUNCS:
        cc = ns[fn](cc)
    cc = ns["calc_std_12"](dd, cc)
    d["chain_index"] = cc.index.values.astype(np.int64)
    d["chain_columns"] = np.array(list(cc.columns))
    d["chain_permno"] = cc["permno"].values.astype(np.int64)
    d["chain_mthcaldt"] = cc["mthcaldt"].values.astype("datetime64[ns]").astype(np.int64)
    for col in cases.CHAR_NAMES + ["rolling_std_252"]:
        d["chain_" + col] = cc[col].values.astype(np.float64)
    # calc_std_12 on scrambled inputs (rolling in frame order within permno; left merge)
    s12 = ns["calc_std_12"](daily.copy(), base.copy())
    d["std_index"] = s12.index.values.astype(np.int64)
    d["std_permno"] = s12["permno"].values.astype(np.int64)
    d["std_mthcaldt"] = s12["mthcaldt"].values.astype("datetime64[ns]").astype(np.int64)
    d["std_rolling_std_252"] = s12["rolling_std_252"].values.astype(np.float64)
    # the per-day rolling std itself (before the month-end pick and the merge)
    dsort = daily.sort_values(["permno", "dlycaldt"])
    r = dsort.groupby("permno")["retx"].rolling(window=252, min_periods=100).std()
    d["daily_std_sorted"] = r.reset_index(level=0, drop=True).reindex(dsort.index).values * np.sqrt(252)
    np.savez_compressed(os.path.join(HERE, "chars.npz"), **d)


if __name__ == "__main__":
    print("numpy", np.__version__, "pandas", pd.__version__, "statsmodels", sm.__version__ if hasattr(sm, "__version__") else "?")
    gen_pct()
    gen_nw()
    gen_edge()
    gen_wins()
    gen_fm()
    gen_fig1()
    gen_fig1(cases.fig1_const_panel(), "fig1c.npz")
    gen_edge(cases.divergence_cases(), "diverge")
    gen_mid()
    gen_table1()
    gen_chars()
    print("ok")

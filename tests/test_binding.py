"""The documented drop-in binding (fmdrop.bind) keeps the reference
notebook runnable: every name its cells call still resolves, the hot-path names resolve to
the engine, and nothing else of the reference modules is shadowed.

The reference modules cannot all be imported here (polars, wrds, decouple and statsmodels
are absent), so the notebook is checked by simulating Python's name resolution over the
AST of src/get_data.ipynb and of the reference modules; the import hook itself is checked
on stand-in modules and on the reference's own transform_compustat.py (pandas/numpy only).
"""
import ast
import builtins
import inspect
import json
import os
import subprocess
import sys
import textwrap
import warnings

import pytest

REF_SRC = "/root/reference/src"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "fm-returnprediction_amd")

needs_ref = pytest.mark.skipif(not os.path.isdir(REF_SRC), reason="reference not mounted")


def _module_exports(name, seen=None):
    """Names `from <name> import *` binds, for a module of the reference's src/ (AST only):
    public top-level defs, classes, assignments and imported names, recursively through the
    module's own star imports.  Third-party modules (not in src/) export nothing known."""
    seen = set() if seen is None else seen
    path = os.path.join(REF_SRC, name + ".py")
    if name in seen or not os.path.exists(path):
        return {}
    seen.add(name)
    tree = _parse(path)
    out = {}
    for node in tree.body:
        if isinstance(node, (ast.FunctionDef, ast.AsyncFunctionDef, ast.ClassDef)):
            out[node.name] = name
        elif isinstance(node, ast.Assign):
            for t in node.targets:
                for n in ast.walk(t):
                    if isinstance(n, ast.Name):
                        out[n.id] = name
        elif isinstance(node, ast.Import):
            for a in node.names:
                out[(a.asname or a.name).split(".")[0]] = name
        elif isinstance(node, ast.ImportFrom):
            for a in node.names:
                if a.name == "*":
                    out.update(_module_exports(node.module, seen))
                else:
                    # a name imported from another src/ module keeps that module as origin
                    origin = node.module if os.path.exists(os.path.join(REF_SRC, f"{node.module}.py")) else name
                    out[a.asname or a.name] = origin
    return {k: v for k, v in out.items() if not k.startswith("_")}


def _parse(path):
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", DeprecationWarning)   # escape sequences in reference strings
        return ast.parse(open(path).read())


def _defs(name):
    tree = _parse(os.path.join(REF_SRC, name + ".py"))
    return {n.name: n for n in tree.body if isinstance(n, ast.FunctionDef)}


def _notebook_cells():
    nb = json.load(open(os.path.join(REF_SRC, "get_data.ipynb")))
    return ["".join(c["source"]) for c in nb["cells"] if c["cell_type"] == "code"]


BINDING_CELL = 'import sys; sys.path.insert(0, "<repo>/fm-returnprediction_amd")\n' \
               "from fmdrop import bind; bind.install()\n"


@needs_ref
def test_integration_md_shows_this_binding():
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    for line in BINDING_CELL.strip().splitlines():
        assert line in doc, line


@needs_ref
def test_hot_names_exist_in_reference_modules_with_same_parameters():
    """Every re-bound name is a def of the reference module it replaces (or a name that
    module imports from one), and the engine's parameters start with the reference's."""
    from fmdrop import bind
    for mod, names in bind.HOT.items():
        exports = _module_exports(mod)
        eng = bind.engine_functions(mod)
        for n in names:
            assert n in exports, (mod, n)
            origin = exports[n]
            ref_def = _defs(origin)[n]
            ref_params = [a.arg for a in ref_def.args.args]
            got = list(inspect.signature(eng[n]).parameters)
            assert got[:len(ref_params)] == ref_params, (mod, n, got, ref_params)
            # extra engine parameters must have defaults (callers pass the reference's)
            sig = inspect.signature(eng[n])
            for p in got[len(ref_params):]:
                assert sig.parameters[p].default is not inspect.Parameter.empty, (n, p)


@needs_ref
def test_notebook_names_resolve_under_binding():
    """Run the notebook's cells symbolically with the binding cell prepended: every called
    name resolves when called, and every hot-path name the notebook calls resolves to a
    module the binding patches (so to the engine)."""
    from fmdrop import bind
    ns = {n: "builtins" for n in dir(builtins)}
    called_hot = set()
    cells = [BINDING_CELL] + _notebook_cells()
    for cell in cells:
        tree = ast.parse(cell)
        for stmt in tree.body:
            for node in ast.walk(stmt):
                if isinstance(node, ast.Call) and isinstance(node.func, ast.Name):
                    name = node.func.id
                    assert name in ns, f"notebook calls {name!r} before anything binds it"
                    origin = ns[name]
                    if origin in bind.HOT and name in bind.HOT[origin]:
                        called_hot.add(name)
            if isinstance(stmt, ast.ImportFrom):
                for a in stmt.names:
                    if a.name == "*":
                        ex = _module_exports(stmt.module)
                        if stmt.module in bind.HOT:
                            # bound through the patched module: origin = that module
                            ex = {k: (stmt.module if k in bind.HOT[stmt.module] else v) for k, v in ex.items()}
                        ns.update(ex)
                    else:
                        ns[a.asname or a.name] = stmt.module
            elif isinstance(stmt, ast.Import):
                for a in stmt.names:
                    ns[(a.asname or a.name).split(".")[0]] = a.name
            else:
                for node in ast.walk(stmt):
                    if isinstance(node, ast.Name) and isinstance(node.ctx, ast.Store):
                        ns[node.id] = "<cell>"
    # what VERDICT r02 found unresolvable under the old shadowing recipe
    for n in ("add_report_date", "calc_book_equity", "save_data", "create_latex_document_from_pkl",
              "compile_latex_document"):
        assert n in ns and ns[n] not in ("<cell>",), n
    # the hot path the notebook drives is the engine's
    for n in ("expand_compustat_annual_to_monthly", "merge_CRSP_and_Compustat", "winsorize", "get_subsets",
              "build_table_1", "build_table_2", "create_figure_1", "calc_std_12", "calculate_rolling_beta",
              "calc_log_size", "calc_sales_price"):
        assert n in called_hot, n


def _run_py(code, extra_path):
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1",
               PYTHONPATH=os.pathsep.join([PKG, extra_path, os.environ.get("PYTHONPATH", "")]))
    r = subprocess.run([sys.executable, "-c", textwrap.dedent(code)], env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


def test_install_patches_only_hot_names(tmp_path):
    """Stand-in reference modules (same module names, hot and non-hot defs): after
    install(), star imports give the engine's hot-path functions and the reference's
    other functions; the originals stay in __fm_reference__."""
    (tmp_path / "regressions.py").write_text(
        "def run_monthly_cs_regressions(df, return_col, predictor_cols, date_col='mthcaldt'): return 'ref'\n"
        "def newey_west_mean_se(slopes, lags=4): return 'ref'\n"
        "def fama_macbeth_summary(cs_results, predictor_cols, date_col='mthcaldt', nw_lags=4): return 'ref'\n")
    (tmp_path / "transform_compustat.py").write_text(
        "def add_report_date(comp): return 'ref'\n"
        "def calc_book_equity(comp): return 'ref'\n"
        "def expand_compustat_annual_to_monthly(comp_annual, id_col='gvkey', report_date_col='report_date'): "
        "return 'ref'\n"
        "def merge_CRSP_and_Compustat(crsp, comp, ccm): return 'ref'\n")
    hot = "\n".join(f"def {n}(*a, **k): return 'ref'" for n in
                    ("get_subsets", "calc_log_size", "calc_log_bm", "calc_return_12_2", "calc_accruals",
                     "calc_log_issues_36", "calc_log_issues_12", "calc_roa", "calc_log_assets_growth",
                     "calc_dy", "calc_log_return_13_36", "calc_debt_price", "calc_sales_price",
                     "calculate_rolling_beta", "calc_std_12", "winsorize", "build_table_1", "build_table_2",
                     "create_figure_1"))
    (tmp_path / "calc_Lewellen_2014.py").write_text(
        "from transform_compustat import expand_compustat_annual_to_monthly, merge_CRSP_and_Compustat\n"
        "from regressions import run_monthly_cs_regressions, fama_macbeth_summary\n" + hot + "\n"
        "def save_data(table_1, table_2, figure_1): return 'ref'\n"
        "def create_latex_document_from_pkl(): return 'ref'\n"
        "def compile_latex_document(tex_file_path=None): return 'ref'\n"
        "def get_factors(crsp_comp, crsp_d, crsp_index_d): return winsorize(crsp_comp, [])\n")
    out = _run_py("""
        from fmdrop import bind; bind.install()
        from transform_compustat import *
        from calc_Lewellen_2014 import *
        import calc_Lewellen_2014 as CL, regressions as R, transform_compustat as TC
        for mod, names in bind.HOT.items():
            m = {"regressions": R, "transform_compustat": TC, "calc_Lewellen_2014": CL}[mod]
            for n in names:
                assert getattr(m, n).__module__.startswith("fmdrop."), (mod, n)
                assert n in m.__fm_reference__ or mod == "calc_Lewellen_2014", (mod, n)
        assert add_report_date(None) == "ref" and calc_book_equity(None) == "ref"
        assert save_data(1, 2, 3) == "ref" and create_latex_document_from_pkl() == "ref"
        assert compile_latex_document() == "ref"
        assert winsorize.__module__ == "fmdrop.calc_Lewellen_2014"
        assert expand_compustat_annual_to_monthly.__module__ == "fmdrop.transform_compustat"
        assert run_monthly_cs_regressions.__module__ == "fmdrop.regressions"
        assert CL.__fm_reference__["winsorize"](None) == "ref"
        # the reference's own callers inside the module reach the engine too
        import inspect
        assert CL.get_factors.__globals__["winsorize"] is winsorize
        print("ok")
    """, str(tmp_path))
    assert out.strip().endswith("ok")


@needs_ref
def test_install_on_reference_transform_compustat():
    """The reference's real transform_compustat.py (it imports pandas / numpy only): the
    expansion and the CCM merge become the engine's, add_report_date / calc_book_equity stay
    the reference's own code."""
    out = _run_py("""
        import sys; sys.dont_write_bytecode = True
        from fmdrop import bind; bind.install()
        from transform_compustat import *
        import transform_compustat as TC
        assert TC.__file__.startswith("/root/reference/src/"), TC.__file__
        assert add_report_date.__code__.co_filename.startswith("/root/reference/src/")
        assert calc_book_equity.__code__.co_filename.startswith("/root/reference/src/")
        assert expand_compustat_annual_to_monthly.__module__ == "fmdrop.transform_compustat"
        assert merge_CRSP_and_Compustat.__module__ == "fmdrop.transform_compustat"
        assert TC.__fm_reference__["merge_CRSP_and_Compustat"].__code__.co_filename.startswith("/root/reference")
        print("ok")
    """, REF_SRC)
    assert out.strip().endswith("ok")

"""Bind the MI355X engine into the reference's own modules, hot-path names only.

The reference notebook (src/get_data.ipynb) reaches the hot path through star imports of
the reference modules: ``from transform_compustat import *`` (cell 0), ``from
calc_Lewellen_2014 import *`` (cell 9), and calc_Lewellen_2014 itself does ``from regressions
import run_monthly_cs_regressions, fama_macbeth_summary`` (reference
src/calc_Lewellen_2014.py:30).  ``install()`` puts an import hook in front of those three
modules: each is loaded from the reference's own file as usual, and right after it executes,
the names in ``HOT`` are replaced by the engine's functions (fmdrop.*).  Nothing else in the
module changes, so ``add_report_date``, ``calc_book_equity``, ``save_data``,
``create_latex_document_from_pkl``, ``compile_latex_document`` and the WRDS pulls keep
resolving to the reference code.  The reference's originals stay reachable as
``module.__fm_reference__[name]``.

Usage (first lines of the notebook's first cell, before its star imports):

    import sys; sys.path.insert(0, "<repo>/fm-returnprediction_amd")
    from fmdrop import bind; bind.install()
"""
from __future__ import annotations

import importlib
import importlib.abc
import sys

# reference module -> the names the engine replaces in it (reference file:line of each def)
HOT = {
    "regressions": (
        "run_monthly_cs_regressions",            # src/regressions.py:9
        "newey_west_mean_se",                    # :78
        "fama_macbeth_summary",                  # :102
    ),
    "transform_compustat": (
        "expand_compustat_annual_to_monthly",    # src/transform_compustat.py:101
        "merge_CRSP_and_Compustat",              # :184
    ),
    "calc_Lewellen_2014": (
        "get_subsets",                           # src/calc_Lewellen_2014.py:44
        "calc_log_size",                         # :137
        "calc_log_bm",                           # :150
        "calc_return_12_2",                      # :166
        "calc_accruals",                         # :195
        "calc_log_issues_36",                    # :207
        "calc_log_issues_12",                    # :224
        "calc_roa",                              # :241
        "calc_log_assets_growth",                # :252
        "calc_dy",                               # :265
        "calc_log_return_13_36",                 # :290
        "calc_debt_price",                       # :316
        "calc_sales_price",                      # :330
        "calculate_rolling_beta",                # :344
        "calc_std_12",                           # :438
        "winsorize",                             # :505
        "build_table_1",                         # :577
        "build_table_2",                         # :674
        "create_figure_1",                       # :871
        # names the reference module imports from the two modules above (:24-30): re-bound
        # here too so `from calc_Lewellen_2014 import *` can never re-export an original
        "run_monthly_cs_regressions",
        "fama_macbeth_summary",
        "expand_compustat_annual_to_monthly",
        "merge_CRSP_and_Compustat",
    ),
}


def engine_functions(module_name: str) -> dict:
    """{name: engine function} for one reference module name."""
    eng = importlib.import_module(f"fmdrop.{module_name}")
    out = {}
    for name in HOT[module_name]:
        if hasattr(eng, name):
            out[name] = getattr(eng, name)
        else:   # re-exported names (the calc_Lewellen_2014 tail of HOT) live in a sibling
            for other in ("regressions", "transform_compustat"):
                mod = importlib.import_module(f"fmdrop.{other}")
                if hasattr(mod, name):
                    out[name] = getattr(mod, name)
                    break
            else:
                raise AttributeError(f"fmdrop has no engine function {name!r}")
    return out


def patch_module(module) -> dict:
    """Replace the HOT names of an already executed reference module in place; returns the
    originals it replaced (also kept as module.__fm_reference__)."""
    name = module.__name__
    repl = engine_functions(name)
    orig = dict(getattr(module, "__fm_reference__", {}))
    for k, fn in repl.items():
        cur = module.__dict__.get(k)
        if cur is not None and cur is not fn and k not in orig:
            orig[k] = cur
        setattr(module, k, fn)
    module.__fm_reference__ = orig
    return orig


class _OverlayLoader(importlib.abc.Loader):
    def __init__(self, inner):
        self.inner = inner

    def create_module(self, spec):
        return self.inner.create_module(spec)

    def exec_module(self, module):
        self.inner.exec_module(module)
        patch_module(module)


class _OverlayFinder(importlib.abc.MetaPathFinder):
    """Finds HOT modules with the remaining finders and wraps their loader."""

    def find_spec(self, fullname, path, target=None):
        if fullname not in HOT:
            return None
        for finder in sys.meta_path:
            if finder is self or not hasattr(finder, "find_spec"):
                continue
            spec = finder.find_spec(fullname, path, target)
            if spec is not None:
                break
        else:
            return None
        if spec.loader is not None:
            spec.loader = _OverlayLoader(spec.loader)
        return spec


_FINDER = _OverlayFinder()


def install(namespace: dict = None) -> None:
    """Activate the binding: reference modules imported from now on get the engine's
    hot-path functions; ones already imported are patched now.  ``namespace`` (e.g. a
    notebook's ``globals()`` after its star imports already ran) has the same names
    re-bound where they are present."""
    # the engine modules import first, so a failure (no libfm_hip, no torch) surfaces here
    engines = {m: engine_functions(m) for m in HOT}
    if _FINDER not in sys.meta_path:
        sys.meta_path.insert(0, _FINDER)
    for m in HOT:
        if m in sys.modules:
            patch_module(sys.modules[m])
    if namespace is not None:
        for fns in engines.values():
            for k, fn in fns.items():
                if k in namespace:
                    namespace[k] = fn


def uninstall() -> None:
    """Remove the import hook (modules already patched stay patched)."""
    while _FINDER in sys.meta_path:
        sys.meta_path.remove(_FINDER)

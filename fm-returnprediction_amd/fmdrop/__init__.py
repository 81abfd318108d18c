"""Drop-in replacements for the reference's hot-path functions, backed by libfm_hip.

The submodules mirror the reference modules they replace, function by function:

  fmdrop.regressions          <- src/regressions.py:9-131
  fmdrop.calc_Lewellen_2014   <- src/calc_Lewellen_2014.py (winsorize, get_subsets, Tables 1/2,
                                  Figure 1, firm characteristics)
  fmdrop.transform_compustat  <- src/transform_compustat.py:101-226 (expansion, CCM merge)

They live in this package, not under the reference's module names, so they never shadow the
reference modules: ``fmdrop.bind.install()`` re-binds only the hot-path names inside the
reference's own modules, and every other name the notebook uses
(``add_report_date``, ``save_data``, the LaTeX helpers, the WRDS pulls) stays the
reference's.
"""

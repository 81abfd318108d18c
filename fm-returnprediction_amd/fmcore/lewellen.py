"""The Lewellen (2015) Table-2 / Figure-1 pass as one device-resident pipeline.

winsorize (1/99, every column, reference src/calc_Lewellen_2014.py:505-529)
 -> NYSE 20th/50th me breakpoints and nested universe levels (:44-112)
 -> Models 1/2/3 x {All, All-but-tiny, Large} and the Figure-1 5-variable model x {All,
    Large} in ONE batched Gram pass (:714-770, :882-921)
 -> Fama-MacBeth means + Newey-West(4) t-stats (src/regressions.py:102-131)
 -> 120-month rolling coefficient means (:926)
 -> lagged-rolling forecasts and predictive-slope FM summaries (build-defined A7/A8)
All stages are libfm_hip kernels; the panel is read from HBM twice (cuts, Gram).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np
import torch

from . import engine as E

# Model definitions: reference src/calc_Lewellen_2014.py:714-745 (labels) and the notebook's
# variables_dict (src/get_data.ipynb cell 24).
MODELS_PREDICTORS = {
    "Model 1: Three Predictors": [
        "Log Size (-1)", "Log B/M (-1)", "Return (-2, -12)"],
    "Model 2: Seven Predictors": [
        "Log Size (-1)", "Log B/M (-1)", "Return (-2, -12)", "Log Issues (-1,-36)",
        "Accruals (-1)", "ROA (-1)", "Log Assets Growth (-1)"],
    "Model 3: Fourteen Predictors": [
        "Log Size (-1)", "Log B/M (-1)", "Return (-2, -12)", "Log Issues (-1,-12)",
        "Accruals (-1)", "ROA (-1)", "Log Assets Growth (-1)", "Dividend Yield (-1,-12)",
        "Log Return (-13,-36)", "Log Issues (-1,-36)", "Beta (-1,-36)", "Std Dev (-1,-12)",
        "Debt/Price (-1)", "Sales/Price (-1)"],
}
VARIABLES_DICT = {
    "Return (%)": "retx", "Log Size (-1)": "log_size", "Log B/M (-1)": "log_bm",
    "Return (-2, -12)": "return_12_2", "Log Issues (-1,-12)": "log_issues_12",
    "Accruals (-1)": "accruals_final", "ROA (-1)": "roa",
    "Log Assets Growth (-1)": "log_assets_growth", "Dividend Yield (-1,-12)": "dy",
    "Log Return (-13,-36)": "log_return_13_36", "Log Issues (-1,-36)": "log_issues_36",
    "Beta (-1,-36)": "beta", "Std Dev (-1,-12)": "rolling_std_252", "Debt/Price (-1)": "debt_price",
    "Sales/Price (-1)": "sales_price",
}
FIG1_VARS = ["log_bm", "return_12_2", "log_issues_36", "accruals_final", "log_assets_growth"]
SUBSET_NAMES = ["All stocks", "All-but-tiny stocks", "Large stocks"]


def table2_models(variables_dict=None):
    vd = variables_dict or VARIABLES_DICT
    out = {}
    for name, labels in MODELS_PREDICTORS.items():
        cols = []
        for lbl in labels:
            if lbl not in vd:
                raise ValueError(f"'{lbl}' not found in variables_dict!")
            cols.append(vd[lbl])
        out[name] = cols
    return out


@dataclass
class PipelineConfig:
    lower_percentile: float = 1
    upper_percentile: float = 99
    winsorize: bool = True
    standardize: bool = False      # north-star extension; OFF on the parity path
    universes: bool = True
    nw_lags: int = 4
    window: int = 120
    min_periods: int = 60
    lag: int = 1
    forecasts: bool = True
    fig1: bool = True


@dataclass
class PipelineResult:
    model_names: List[str]
    model_cols: Dict[str, List[str]]
    res: E.FMResult
    ix: E.TSIndex
    summary: E.Summary
    rolling: Optional[torch.Tensor] = None
    pred: Optional[torch.Tensor] = None
    pred_status: Optional[torch.Tensor] = None
    pred_summary: Optional[E.Summary] = None
    cuts: Optional[E.Cuts] = None
    level: Optional[torch.Tensor] = None
    breakpoints: Optional[tuple] = None


def build_models(panel: E.DevicePanel, model_cols: Dict[str, List[str]], y="retx", fig1=True,
                 universes=True):
    levels = (0, 1, 2) if universes else (0,)
    models, names = [], []
    for name, cols in model_cols.items():
        models.append(E.Model(name, y=panel.col(y), xs=[panel.col(c) for c in cols], levels=levels))
        names.append(name)
    if fig1:
        # create_figure_1: has_constant='add' (no constant-column error), All & Large only
        models.append(E.Model("Figure 1", y=panel.col(y), xs=[panel.col(c) for c in FIG1_VARS],
                              levels=(0, 2) if universes else (0,), const_check=False))
        names.append("Figure 1")
    return models, names


def _standardize_params(panel: E.DevicePanel, cuts: E.Cuts, yi: int):
    """A9 (build-defined): the Gram sees z = (clip(x) - mean_t) / sd_t for every predictor
    column (shift = mean, inv_scale = 1/sd, nothing added back: the regressors ARE the
    z-scores), while the dependent column keeps its units (shift = its pivot, scale 1,
    added back to the intercept).  All [C, T] month tables, built on the device."""
    shift = cuts.mean.clone()
    inv_scale = 1.0 / cuts.sd
    add_back = torch.zeros_like(shift)
    shift[yi] = cuts.center[yi]
    inv_scale[yi] = 1.0
    add_back[yi] = cuts.center[yi]
    return shift, inv_scale, add_back


def local_stage(panel: E.DevicePanel, cfg: PipelineConfig, model_cols, y="retx"):
    """Panel-sized work for one shard of months: cuts, universes, batched Gram + solve."""
    cuts = None
    shift = None
    inv_scale = None
    level, bp = None, None
    nlevels = 1
    models, names = build_models(panel, model_cols, y=y, fig1=cfg.fig1, universes=cfg.universes)
    select = cfg.winsorize or cfg.standardize
    # get_subsets' NYSE breakpoints + level bytes come with the winsorize call
    # (fm_select_universe): on the bench's short months they share the select fix-up's launch
    # (the universe no longer needs a launch of its own), on C5's long months they ride the
    # long-month kernel's launch (one more grid column); other paths launch fm_universe first
    fused_universe = cfg.universes and select and not cfg.standardize
    if cfg.universes and not fused_universe:
        a, b, level = E.universe(panel)
        nlevels = 3
        bp = (a, b)
    add_back = None
    if select:
        mc = 5 if cfg.winsorize else 2 ** 31 - 1
        # standardize needs the exact clipped moments; otherwise the Gram pivot is the
        # select kernel's free center (midpoint of the cuts), and no moments pass runs
        cuts = E.select_cuts(panel, cfg.lower_percentile / 100, cfg.upper_percentile / 100, mc,
                             E.LERP_NUMPY, moments=cfg.standardize, center=True,
                             universe=(0.2, 0.5) if fused_universe else None)
        if fused_universe:
            cuts, (a, b, level) = cuts
            nlevels = 3
            bp = (a, b)
        shift = cuts.center
        if cfg.standardize:
            shift, inv_scale, add_back = _standardize_params(panel, cuts, panel.col(y))
        if not cfg.winsorize:
            cuts = E.Cuts(torch.full_like(cuts.lo, float("nan")), torch.full_like(cuts.hi, float("nan")),
                          cuts.nvalid, cuts.mean, cuts.sd, cuts.center)
    res = E.fm_pass(panel, models, level=level, nlevels=nlevels, cuts=cuts, shift=shift,
                    inv_scale=inv_scale, add_back=add_back if cfg.standardize else shift,
                    moments=cfg.forecasts)
    if cfg.standardize:
        E.drop_degenerate_months(res, models, cuts.sd)
    return res, names, cuts, level, bp


def time_series_stage(res: E.FMResult, cfg: PipelineConfig, moments=None, seg_lo=0, seg_hi=None,
                      sum_range=None, roll_own=False):
    """One launch (fm_ts_fused): compaction, FM summaries, rolling means, predictive slopes.
    Their FM summary follows in summarize_predictive.  Returns (ix, summ, roll, pred, pst).
    Month-sharded ranks pass their problem block (``sum_range``) and ``roll_own`` (rolling
    means only where their own months' predictive records read them); the summaries are then
    SUM-combined across ranks (fmcore.step.ShardedStep)."""
    return E.time_series_result(
        res, cfg.nw_lags, cfg.window, cfg.min_periods, cfg.lag, seg_lo=seg_lo, seg_hi=seg_hi,
        moments=moments, rolling=cfg.forecasts or cfg.fig1, predictive=cfg.forecasts,
        sum_range=sum_range, roll_own=roll_own)


def run_pipeline(panel: E.DevicePanel, cfg: PipelineConfig = None, model_cols=None, y="retx"):
    cfg = cfg or PipelineConfig()
    model_cols = model_cols or table2_models()
    res, names, cuts, level, bp = local_stage(panel, cfg, model_cols, y)
    ix, summ, roll, pred, pst = time_series_stage(res, cfg)
    psumm = None
    if cfg.forecasts:
        psumm, _ = E.summarize_predictive(pred, pst, cfg.nw_lags)
    return PipelineResult(model_names=names, model_cols=dict(model_cols, **({"Figure 1": FIG1_VARS} if cfg.fig1 else {})),
                          res=res, ix=ix, summary=summ, rolling=roll, pred=pred, pred_status=pst,
                          pred_summary=psumm, cuts=cuts, level=level, breakpoints=bp)


def problem_index(res: E.FMResult, names, model_name, level):
    mi = names.index(model_name)
    for k, p in enumerate(res.problems):
        if p.model == mi and p.level == level:
            return k
    raise KeyError((model_name, level))

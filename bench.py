"""Benchmark: the full Fama-MacBeth pass (BASELINE.json metric) on MI355X.

Workload per GPU (BASELINE configs C3+C4): a 600-month x 5,000-firm synthetic panel with
15 characteristics (retx + the 14 Lewellen predictors), generated in HBM by fm_gen_panel.
One step = winsorize all 15 columns (1/99) -> NYSE me breakpoints + nested universes ->
Models 1/2/3 x {All, All-but-tiny, Large} + the Figure-1 model x {All, Large} (11
cross-sectional problems per month) in one batched Gram pass -> solves -> all-gather of
the monthly records -> Fama-MacBeth means + Newey-West(4) -> 120/60 rolling means ->
lagged-rolling forecasts + predictive-slope FM summaries.  Inputs are HBM-resident when
the timed region starts.  With N GPUs (torchrun) each rank owns 600 months of a 600*N-month
panel (weak scaling); value = all ranks' firm-month rows / max-over-ranks time.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "fm-returnprediction_amd")
for _p in (PKG, ROOT):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "firm-month rows/sec (and % HBM roofline) for full FM pass at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s; 6.29 measured copy)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--months", type=int, default=600, help="months per GPU")
    ap.add_argument("--firms", type=int, default=5000)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--cpu-months", type=int, default=240, help="oracle CPU-baseline sample")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-chars", action="store_true", help="skip the firm-characteristic stage")
    ap.add_argument("--check", action="store_true", help="verify one step against the oracle")
    ap.add_argument("--no-graph", action="store_true", help="eager launches instead of HIP graphs")
    ap.add_argument("--no-c5", action="store_true", help="skip the C5 per-rank shard measurement")
    return ap.parse_args()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)
    from fmcore import dist as D
    from fmcore import engine as E
    from fmcore import lewellen as LW
    from fmcore.step import ShardedStep

    cfg = LW.PipelineConfig()
    model_cols = LW.table2_models()
    T_loc, N = args.months, args.firms
    T_glob = T_loc * world
    panel = E.panel_synthetic(T_loc, N, args.seed, month0=rank * T_loc, device=dev)
    # chunk the Gram by the GLOBAL panel so per-month sums are identical for any rank count
    panel.chunk_rows = E.default_chunk_rows(T_glob * N, T_glob, N)
    rows_local = T_loc * N
    step = ShardedStep(panel, cfg, model_cols, world=world, rank=rank, seg_lo=rank * T_loc,
                       seg_hi=(rank + 1) * T_loc, global_months=T_glob, counts=[T_loc] * world)
    for _ in range(max(1, args.warmup)):   # >= 1: allocates the static exchange buffers
        step.eager()
    torch.cuda.synchronize()
    if not args.no_graph:
        # capture (on a side stream, as torch.cuda.graph requires); the eager warm-up has
        # filled every host-side cache, so the captured launches are exactly a step's kernels
        step.capture()
    for _ in range(2):
        step.replay()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = step.replay()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        dt = D.max_over_ranks(dt, dev)
    # per-kernel device times (HIP events on the launch stream), from eager steps outside
    # the timed region: they feed the roofline of the dominant kernel
    timer = E.KernelTimer()
    with timer:
        for _ in range(max(3, min(args.steps, 10))):
            step.eager()
    torch.cuda.synchronize()
    gres, summ, psumm = out
    nfit = int(((gres.status & 1) != 0).sum().item())

    # roofline of the dominant kernel: per-launch algorithmic bytes / its device time, the
    # latter from the latest launch re-issued back to back (E.time_launch: no launch gaps)
    C = panel.ncols
    kern = {}
    for tag in timer.names():
        kern[tag] = timer.avg_ms(tag)   # events around each eager launch (incl. launch gaps)
    tags = ("fm_select_cuts", "fm_gram", "fm_universe", "fm_solve", "fm_ts_fused", "fm_ts_fused[pred]")
    dev_ms = {t: E.time_launch(t) for t in tags if t in E.LAST_LAUNCH}
    # algorithmic HBM bytes per launch: every panel column once (8 B per
    # value), the universe level byte, and the month tables written (cuts, pivots, Gram
    # partials); fm_select alone reads the columns only
    cand = {"fm_select_cuts": rows_local * C * 8, "fm_gram": rows_local * (C * 8 + 1)}
    dom = max((t for t in cand if t in dev_ms), key=lambda k: dev_ms[k])
    dom_ms = dev_ms[dom]
    achieved = cand[dom] / (dom_ms * 1e-3) / 1e9
    traffic = _pmc_traffic(dom)
    # whole pass: every input byte of a firm-month row -- the C FP64 columns,
    # me (FP64) and the NYSE flag -- over the measured step time
    b_row = C * 8 + 8 + 1
    ms_step = dt / args.steps * 1e3
    whole = rows_local * b_row / (ms_step * 1e-3) / 1e9

    stream = _stream_copy_gbs(dev)
    result = {
        "metric": METRIC,
        "value": rows_local * world * args.steps / dt,
        "unit": "firm-month rows/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (counter-hash panel generated in HBM, Table-1 moments, t2 tails, 2% NaN)",
        "config": {
            "workload": "C3+C4 full pass per GPU: 600 months x 5000 firms x 15 chars; winsorize 1/99 -> "
                        "NYSE universes -> M1/M2/M3 x 3 universes + Fig-1 x 2 -> NW(4) -> rolling 120/60 -> "
                        "lagged-rolling forecasts + predictive-slope FM",
            "months_per_gpu": T_loc, "firms": N, "chars": C, "problems_per_month": gres.nprob,
            "global_months": T_glob, "parallelism": f"month-sharded x{world}, RCCL all-gather of records",
        },
        "regressions_per_s": nfit * args.steps / dt,
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                     "traffic": traffic["bytes"] if traffic else None,
                     "traffic_ratio": traffic["bytes"] / cand[dom] if traffic else None,
                     "traffic_source": traffic["source"] if traffic else None,
                     "bytes_per_launch": cand[dom], "avg_launch_ms": dom_ms,
                     "measured_copy_peak": stream, "frac_of_measured_copy": achieved / stream,
                     "whole_pass": {"bytes_per_row": b_row, "achieved": whole, "frac": whole / HBM_PEAK_GBS,
                                    "ms_per_step": ms_step}},
        "kernel_ms": {k: round(v, 4) for k, v in dev_ms.items()},
        "lib_sha16": _lib_sha(),
        "kernel_ms_eager_events": {k: round(v, 4) for k, v in kern.items()},
        "graph": not args.no_graph,
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        result["cpu_baseline"] = cpu_baseline(panel, args, LW)
    if rank == 0 and world == 1 and not args.no_chars:
        result["firm_chars"] = firm_chars_stage(args, E)
    if args.check and rank == 0 and world == 1:
        result["check"] = check_against_oracle(panel, gres, summ, args, LW)
    if rank == 0 and world == 1 and not args.no_c5:
        del panel
        torch.cuda.empty_cache()
        result["c5_rank_shard"] = c5_shard_stage(args, E, LW)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


def c5_shard_stage(args, E, LW, reps=3):
    """C5 (BASELINE configs[4]: 100,000 months x 20,000 firms x 15 chars over 8 GPUs) at one
    rank's size, as rank 4 of 8 runs it: its 12,500 months x 20,000 firms = 250M rows (30 GB
    of FP64 columns) generated in HBM, the local pass (winsorize, universes, 11 problems per
    month), then the time-series stage on the GATHERED 100,000-month series (FM means, NW,
    rolling means, the predictive slopes of its own months + their summary).  The gathered
    records are this pass's records tiled 8 times; the all-gather itself is replaced by one
    device copy of the rank's rows.  Eager launches, HIP events around each stage."""
    T, N, world, rank = 12500, 20000, 8, 4
    p = E.panel_synthetic(T, N, 20150101, month0=rank * T)
    cfg = LW.PipelineConfig()
    mc = LW.table2_models()
    lo, hi = rank * T, (rank + 1) * T
    res = LW.local_stage(p, cfg, mc)[0]   # warm-up (plans, workspaces)
    rec_g = res.rec.repeat(world, 1, 1).contiguous()
    st_g = res.status.repeat(world, 1).contiguous()

    def ts(r):
        rec_g[lo:hi].copy_(r.rec)   # stand-in for the all-gather of the ranks' records
        st_g[lo:hi].copy_(r.status)
        g = E.FMResult(problems=r.problems, rec=rec_g, status=st_g, pmax=r.pmax, moments=r.moments,
                       mom_stride=r.mom_stride)
        ix, summ, roll, pred, pst = LW.time_series_stage(g, cfg, moments=r.moments, seg_lo=lo, seg_hi=hi)
        E.summarize_predictive(pred, pst, cfg.nw_lags)

    ts(res)
    torch.cuda.synchronize()
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(reps)]
    for e in ev:
        e[0].record()
        r = LW.local_stage(p, cfg, mc)[0]
        e[1].record()
        ts(r)
        e[2].record()
    ev[-1][2].synchronize()
    loc = sum(e[0].elapsed_time(e[1]) for e in ev) / reps
    tsm = sum(e[1].elapsed_time(e[2]) for e in ev) / reps
    ms = loc + tsm
    rows = T * N
    return {"rows": rows, "months": T, "gathered_months": T * world, "firms": N, "ms_per_pass": ms,
            "ms_local": loc, "ms_ts_100k": tsm, "rows_per_s": rows / (ms * 1e-3),
            "whole_pass_frac": rows * (15 * 8 + 8 + 1) / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "note": "eager launches; rank 4 of the 8-GPU C5 split (local pass + time series on the "
                    "100,000-month gathered series; the all-gather is not timed)"}


def _stream_copy_gbs(dev, nbytes=1 << 30, reps=10):
    """The achievable HBM rate on this box: a 1 GiB device-to-device copy (read + write
    bytes) timed with HIP events -- reported beside the 8 TB/s spec peak."""
    a = torch.empty(nbytes // 8, dtype=torch.float64, device=dev)
    b = torch.empty_like(a)
    b.copy_(a)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        b.copy_(a)
    e1.record()
    e1.synchronize()
    ms = e0.elapsed_time(e1) / reps
    del a, b
    torch.cuda.empty_cache()
    return 2 * nbytes / (ms * 1e-3) / 1e9


def _lib_sha():
    import hashlib
    path = os.path.join(PKG, "lib", "libfm_hip.so")
    try:
        return hashlib.sha256(open(path, "rb").read()).hexdigest()[:16]
    except OSError:
        return None


def _pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 counter summary
    (profiles/pmc_traffic.json, tools/pmc_traffic.py: FETCH_SIZE x the gfx950 calibration +
    WRITE_SIZE, separate --pmc passes).  Used only if it was collected on the SAME library
    build (sha256 of libfm_hip.so): a stale file is refused, not reported."""
    tf = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        d = json.load(open(tf))
    except Exception:
        return None
    if d.get("lib_sha16") != _lib_sha() or kernel not in d:
        return None
    return {"bytes": d[kernel], "source": f"profiles/pmc_traffic.json (lib {d['lib_sha16']})"}


def firm_chars_stage(args, E):
    """SURVEY.md §8(f) row 2, measured beside the headline (not part of `value`): the twelve
    get_factors characteristics (fm_firm_chars) on a firm-major 5,000-firm x 600-month panel
    and calc_std_12's rolling std (fm_rolling_std) on 5,000 firms x 2,520 trading days, both
    resident in HBM; device time = the launch re-issued back to back (HIP events on the
    launch stream).  Algorithmic bytes: 12 fields + id read, 12 outputs written = 200 B per
    monthly row; id + retx read, std written = 24 B per daily row."""
    from fmcore import synth_chars
    res = {}
    ids, flds = synth_chars.device_raw_panel(args.firms, 600, seed=args.seed)
    E.firm_chars(ids, flds)
    torch.cuda.synchronize()
    ms = E.time_launch("fm_firm_chars", 20)
    rows = int(ids.shape[0])
    gbs = rows * 200 / (ms * 1e-3) / 1e9
    res["monthly"] = {"rows": rows, "ms": ms, "rows_per_s": rows / (ms * 1e-3),
                      "roofline": {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                   "frac": gbs / HBM_PEAK_GBS, "bytes_per_launch": rows * 200}}
    del flds
    dids, x = synth_chars.device_daily_returns(args.firms, 2520, seed=args.seed)
    out = torch.empty_like(x)
    E.rolling_std(dids, x, out=out)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        E.rolling_std(dids, x, out=out)
    e1.record()
    e1.synchronize()
    ms = e0.elapsed_time(e1) / 10
    drows = int(x.shape[0])
    gbs = drows * 24 / (ms * 1e-3) / 1e9
    res["daily_std"] = {"rows": drows, "ms": ms, "rows_per_s": drows / (ms * 1e-3),
                        "roofline": {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                     "frac": gbs / HBM_PEAK_GBS, "bytes_per_launch": drows * 24}}
    if not args.no_cpu:
        from oracle import chars_oracle as CO
        nf = 200
        ids2, fl2 = synth_chars.device_raw_panel(nf, 600, seed=args.seed + 1)
        fh = {k: v.cpu().numpy() for k, v in fl2.items()}
        ih = ids2.cpu().numpy()
        t0 = time.perf_counter()
        CO.firm_chars(ih, fh)
        dt = time.perf_counter() - t0
        res["monthly"]["cpu_baseline"] = {"value": len(ih) / dt, "unit": "firm-month rows/s", "cores": 1,
                                          "kind": "port", "sample": f"{nf} firms x 600 months, "
                                          "oracle/chars_oracle.py firm_chars (vectorized numpy)"}
        nd = 20
        di, dx = synth_chars.device_daily_returns(nd, 2520, seed=args.seed + 1)
        di, dx = di.cpu().numpy(), dx.cpu().numpy()
        t0 = time.perf_counter()
        CO.rolling_std(di, dx)
        dt = time.perf_counter() - t0
        res["daily_std"]["cpu_baseline"] = {"value": len(dx) / dt, "unit": "firm-day rows/s", "cores": 1,
                                            "kind": "port", "sample": f"{nd} firms x 2520 days, "
                                            "oracle/chars_oracle.py rolling_std (per-row window)"}
    return res


def cpu_baseline(panel, args, LW):
    """The CPU oracle (numpy restatement of the reference path; per-month SVD-pinv OLS,
    numpy percentiles, NW, rolling) timed on a bounded month sample of the same panel."""
    from oracle import fm_oracle as O
    try:
        from threadpoolctl import threadpool_limits
    except Exception:  # pragma: no cover
        threadpool_limits = None
    S = min(args.cpu_months, panel.nseg)
    n = S * args.firms
    cols = {name: panel.cols[i, :n].cpu().numpy() for i, name in enumerate(panel.names)}
    me = panel.me[:n].cpu().numpy()
    nyse = panel.nyse[:n].cpu().numpy().astype(bool)
    seg = panel.seg_off_h[: S + 1]
    models = {k: ("retx", v, (0, 1, 2)) for k, v in LW.table2_models().items()}
    models["Figure 1"] = ("retx", LW.FIG1_VARS, (0, 2))
    ctx = threadpool_limits(1) if threadpool_limits else None
    t0 = time.perf_counter()
    if ctx:
        with ctx:
            O.pipeline_arrays(cols, seg, me, nyse, models, None)
    else:
        O.pipeline_arrays(cols, seg, me, nyse, models, None)
    dt = time.perf_counter() - t0
    out = {"value": n / dt, "unit": "firm-month rows/s", "cores": 1, "kind": "port",
           "seconds": dt,
            "sample": f"first {S} months x {args.firms} firms of the same panel, full pass "
                      f"(11 problems/month, rolling, forecasts), oracle/fm_oracle.py, 1 BLAS thread"}
    # the port vs the reference itself, timed side by side in the build container
    # (tools/ref_vs_port_timing.py -> profiles/ref_vs_port.json; the reference never travels)
    rp = os.path.join(ROOT, "profiles", "ref_vs_port.json")
    if os.path.exists(rp):
        d = json.load(open(rp))
        out["ref_over_port"] = d["ref_over_port"]
        out["reference_value_est"] = out["value"] * d["ref_over_port"]
        out["ref_over_port_sample"] = d["sample"] + f", python {d['interpreter']}, profiles/ref_vs_port.json"
        out["ref_over_port_host"] = ("the 8-core build container (the reference cannot travel to the GPU box); "
                                     "reference_value_est = this host's port rate x that ratio")
    return out


def check_against_oracle(panel, gres, summ, args, LW):
    """Spot check: monthly records of 3 months against the oracle on those months."""
    from oracle import fm_oracle as O
    S = 3
    n = S * args.firms
    cols = {name: panel.cols[i, :n].cpu().numpy() for i, name in enumerate(panel.names)}
    models = {k: ("retx", v, (0, 1, 2)) for k, v in LW.table2_models().items()}
    ref = O.pipeline_arrays(cols, panel.seg_off_h[: S + 1], panel.me[:n].cpu().numpy(),
                            panel.nyse[:n].cpu().numpy().astype(bool), models, None)
    rec = gres.rec.cpu().numpy()
    worst = 0.0
    for k, p in enumerate(gres.problems):
        if p.model >= 3:
            continue
        name = list(models)[p.model]
        r = ref[(name, p.level)]
        for i, t in enumerate(r["month"]):
            a = rec[t, k, : p.K + 1]
            b = r["params"][i]
            worst = max(worst, float(np.max(np.abs(a - b) / np.maximum(np.abs(b), 1e-3))))
    return {"months": S, "worst_rel_param_err": worst}


if __name__ == "__main__":
    main()

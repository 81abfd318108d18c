"""Benchmark: the full Fama-MacBeth pass (BASELINE.json metric) on MI355X.

Workloads (one step = one pass of the hot path over the rank's months, inputs HBM-resident):

* headline (default at N=1; BASELINE configs C3+C4): a 600-month x 5,000-firm synthetic
  panel with 15 characteristics (retx + the 14 Lewellen predictors), generated in HBM by
  fm_gen_panel.  One step = winsorize all 15 columns (1/99) -> NYSE me breakpoints + nested
  universes -> Models 1/2/3 x {All, All-but-tiny, Large} + the Figure-1 model x {All, Large}
  (11 cross-sectional problems per month) in one batched Gram pass -> solves -> Fama-MacBeth
  means + Newey-West(4) -> 120/60 rolling means -> lagged-rolling forecasts +
  predictive-slope FM summaries.
* c5 (default at N>1; BASELINE configs[4]): every rank owns 12,500 months x 20,000 firms x 15
  characteristics of a 12,500*N-month panel (at N=8 exactly C5's 100,000 x 20,000 x 15), the
  same pass through fmcore.step.ShardedStep: local pass -> RCCL all-gather of the monthly
  records -> time-series stage on the gathered series -> RCCL SUM all-reduce of the
  predictive records -> predictive summary.  Both collectives are inside the timed region.

value = all ranks' firm-month rows / max-over-ranks time (weak scaling).  At N=1 the line
also carries the C5 per-rank shard through ShardedStep (`c5_rank_shard`, the N=1 point of
the C5 scaling curve); at N>1 it also carries the headline panel weak-scaled
(`headline_weak`, 600 months x 5,000 firms per rank, same exchanges).
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
C5_MONTHS, C5_FIRMS, C5_SEED = 12500, 20000, 20150101   # per rank (C5 = 100,000 months at N=8)
B_ROW = 15 * 8 + 8 + 1   # input bytes of a firm-month row: 15 FP64 columns, me, the NYSE flag


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); without WORLD_SIZE in the environment, N > 1 starts "
                         "N worker processes itself through torch.distributed.run (default: "
                         "WORLD_SIZE, else 1)")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", choices=("headline", "c5"), default=None,
                    help="default: headline at N=1, c5 at N>1")
    ap.add_argument("--months", type=int, default=600, help="headline months per GPU")
    ap.add_argument("--firms", type=int, default=5000, help="headline firms")
    ap.add_argument("--c5-months", type=int, default=C5_MONTHS, help="c5 months per GPU")
    ap.add_argument("--c5-firms", type=int, default=C5_FIRMS)
    ap.add_argument("--c5-steps", type=int, default=5, help="timed steps of the N=1 C5 shard")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--cpu-months", type=int, default=240, help="oracle CPU-baseline sample")
    ap.add_argument("--cpu-procs", type=int, default=8, help="month-parallel CPU baseline processes")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-chars", action="store_true", help="skip the firm-characteristic stage")
    ap.add_argument("--check", action="store_true", help="verify one step against the oracle")
    ap.add_argument("--no-graph", action="store_true", help="eager launches instead of HIP graphs")
    ap.add_argument("--no-planes", action="store_true",
                    help="generate the panel as FP64 columns (default: the split high/low-word planes only)")
    ap.add_argument("--no-c5", action="store_true", help="skip the C5 per-rank shard at N=1")
    ap.add_argument("--no-standardize", action="store_true",
                    help="skip the C3 winsorize/standardize variant timed beside the headline")
    ap.add_argument("--no-headline", action="store_true", help="skip headline_weak at N>1")
    ap.add_argument("--dist-backend", default="nccl",
                    help="N>1 process group backend (nccl = RCCL; gloo only to rehearse on one GPU)")
    ap.add_argument("--one-device", action="store_true",
                    help="rehearsal: every rank on cuda:0 (with --dist-backend gloo)")
    ap.add_argument("--launch-probe", action="store_true",
                    help="test aid: start the ranks as for --gpus N, join a gloo group on the CPU, "
                         "print rank 0's {n_gpus, dist_world} and exit (no GPU call)")
    return ap.parse_args(argv)


class LaunchError(SystemExit):
    """--gpus disagrees with the rank count the launcher gave this process."""

    def __init__(self, msg):
        print(f"bench.py: {msg}", file=sys.stderr, flush=True)
        super().__init__(2)


def launch_plan(gpus, env, argv, port=None):
    """How `bench.py --gpus N` gets N ranks (decided before anything touches the GPU).

    * Under a launcher (WORLD_SIZE set, e.g. the driver's torch.distributed.run line), this
      process IS one rank: returns None, and a --gpus that differs from WORLD_SIZE is an
      error (LaunchError, exit 2), never a silent one-rank run.
    * Without one and N > 1: the command that starts N fresh worker processes, one per GPU,
      through torch.distributed.run on 127.0.0.1 with the same arguments; this process only
      waits for them (rank 0 prints the JSON line).
    * Otherwise (N = 1): None, one in-process rank."""
    ws = env.get("WORLD_SIZE")
    if ws is not None:
        ws = int(ws)
        if gpus is not None and gpus != ws:
            raise LaunchError(f"--gpus {gpus} but the launcher started WORLD_SIZE={ws} ranks")
        return None
    if gpus is None or gpus <= 1:
        if gpus is not None and gpus < 1:
            raise LaunchError(f"--gpus {gpus}: need at least one GPU")
        return None
    if port is None:
        port = env.get("MASTER_PORT") or _free_port()
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def _launch_probe(world):
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo")
    out = {"n_gpus": world, "dist_backend": dist.get_backend() if world > 1 else None,
           "dist_world": dist.get_world_size() if world > 1 else 1,
           "rank": int(os.environ.get("RANK", "0"))}
    if out["rank"] == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def timed_steps(step, steps, warmup, graph, world, dev):
    """W untimed warm-up steps (>= 1: the static exchange buffers), HIP-graph capture, then
    exactly `steps` replays bracketed by barrier + synchronize; max over ranks."""
    for _ in range(max(1, warmup)):
        step.eager()
    torch.cuda.synchronize()
    if graph:
        step.capture()
    for _ in range(2):
        step.replay()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        out = step.replay()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        from fmcore import dist as D
        dt = D.max_over_ranks(dt, dev)
    return dt, out


def gen_panel(T, N, seed, month0, dev, E, planes=True):
    """The rank's panel generated in HBM (outside the timed step, like a real panel's ingest):
    by default in the split layout only -- fm_gen_panel_planes writes the values' high / low
    32-bit planes, which the selects (high plane) and the Gram (both) read; no FP64 columns, no
    separate layout pass.  --no-planes: FP64 columns only.  Returns (panel, device ms)."""
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    panel = E.panel_synthetic(T, N, seed, month0=month0, device=dev, layout="planes" if planes else "f64")
    e1.record()
    e1.synchronize()
    return panel, e0.elapsed_time(e1)


def make_step(T_loc, N, seed, world, rank, dev, E, LW, planes=True):
    from fmcore.step import ShardedStep
    panel, panel.gen_ms = gen_panel(T_loc, N, seed, rank * T_loc, dev, E, planes)
    T_glob = T_loc * world
    # one Gram plan for every rank, made from the GLOBAL panel's sizes and cut in global row
    # space, so a month's partial sums (and their order) do not depend on the rank count
    panel.chunk_policy = E.chunk_policy(T_glob * N, T_glob, N)
    panel.row_origin = rank * T_loc * N
    step = ShardedStep(panel, LW.PipelineConfig(), LW.table2_models(), world=world, rank=rank,
                       seg_lo=rank * T_loc, seg_hi=(rank + 1) * T_loc, global_months=T_glob,
                       counts=[T_loc] * world)
    return panel, step


def kernel_roofline(step, panel, E, steps):
    """Per-kernel device times and the roofline of the dominant kernel.  Eager steps outside
    the timed region fill engine.LAST_LAUNCH; each panel-sized launch is then re-issued back
    to back on its stream (E.time_launch, HIP events: no launch gaps)."""
    timer = E.KernelTimer()
    with timer:
        for _ in range(steps):
            step.eager()
    torch.cuda.synchronize()
    kern = {tag: timer.avg_ms(tag) for tag in timer.names()}
    tags = ("fm_select_cuts", "fm_select_cuts[nyse]", "fm_gram", "fm_universe", "fm_solve", "fm_ts_fused",
            "fm_ts_fused[pred]")
    reps = 20 if panel.nrows <= 10_000_000 else 3
    dev_ms = {t: E.time_launch(t, reps) for t in tags if t in E.LAST_LAUNCH}
    rows, C = panel.nrows, panel.ncols
    # algorithmic HBM bytes per launch: the Gram reads every panel column once
    # (8 B per value, from the two 32-bit planes or the FP64 columns) and the universe level
    # byte.  The roofline is priced on the Gram: it is one kernel, while the select tag is two
    # launches (the two-wave select, then the fix-up that also computes the universe); the
    # select's own figure (high plane: 4 B per value; + me, NYSE and level bytes when the
    # universe comes with it) is reported beside it
    gram_bytes = rows * (C * 8 + 1)
    sel_bytes = rows * C * (4 if panel.planes is not None else 8)
    if E.LAST_LAUNCH.get("fm_select_cuts", ("",))[0] == "fm_select_universe":
        sel_bytes += rows * (8 + 1 + 1)
    dom = "fm_gram"
    dom_ms = dev_ms[dom]
    achieved = gram_bytes / (dom_ms * 1e-3) / 1e9
    sel = None
    if "fm_select_cuts" in dev_ms:
        sel = {"launches": "select + fix-up/universe", "bytes_per_launch": sel_bytes, "ms": dev_ms["fm_select_cuts"],
               "achieved": sel_bytes / (dev_ms["fm_select_cuts"] * 1e-3) / 1e9}
        sel["frac"] = sel["achieved"] / HBM_PEAK_GBS
    return dom, dom_ms, gram_bytes, achieved, dev_ms, kern, sel


def main():
    argv = sys.argv[1:]
    args = parse(argv)
    cmd = launch_plan(args.gpus, os.environ, argv)
    if cmd is not None:
        # N worker ranks as child processes (this process never touched the GPU); their
        # stdout is ours, rank 0 prints the line; exit with the launcher's status
        import subprocess
        sys.exit(subprocess.run(cmd).returncode)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.launch_probe:
        return _launch_probe(world)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.one_device:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.dist_backend)
    from fmcore import engine as E
    from fmcore import lewellen as LW

    workload = args.workload or ("headline" if world == 1 else "c5")
    if workload == "headline":
        T_loc, N, seed = args.months, args.firms, args.seed
        wl = ("C3+C4 full pass per GPU: 600 months x 5000 firms x 15 chars; winsorize 1/99 -> "
              "NYSE universes -> M1/M2/M3 x 3 universes + Fig-1 x 2 -> NW(4) -> rolling 120/60 -> "
              "lagged-rolling forecasts + predictive-slope FM")
    else:
        T_loc, N, seed = args.c5_months, args.c5_firms, C5_SEED
        wl = (f"C5 month-sharded: {T_loc} months x {N} firms x 15 chars per GPU of a {T_loc * world}-month "
              f"panel (N=8: 100,000 x 20,000 x 15); local pass -> RCCL all-gather of records -> "
              f"time series on the gathered series -> RCCL all-reduce of predictive records")
    panel, step = make_step(T_loc, N, seed, world, rank, dev, E, LW, planes=not args.no_planes)
    T_glob = T_loc * world
    rows_local = T_loc * N
    dt, out = timed_steps(step, args.steps, args.warmup, not args.no_graph, world, dev)
    gres, summ, psumm = out
    nfit = int(((gres.status & 1) != 0).sum().item())   # fitted (month, problem) pairs, all ranks
    ksteps = max(3, min(args.steps, 10)) if workload == "headline" else 2
    dom, dom_ms, dom_bytes, achieved, dev_ms, kern, sel_roof = kernel_roofline(step, panel, E, ksteps)
    traffic = _pmc_traffic(dom) if workload == "headline" else None
    ms_step = dt / args.steps * 1e3
    whole = rows_local * B_ROW / (ms_step * 1e-3) / 1e9   # per rank (each rank reads its shard)

    read_peak = _stream_read_gbs(E, dev)
    copy_peak = _stream_copy_gbs(E, dev)
    result = {
        "metric": METRIC,
        "value": rows_local * world * args.steps / dt,
        "unit": "firm-month rows/s",
        "n_gpus": world,
        "dist_backend": torch.distributed.get_backend() if world > 1 else None,
        "dist_world": torch.distributed.get_world_size() if world > 1 else 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (counter-hash panel generated in HBM, Table-1 moments, t2 tails, 2% NaN)",
        "config": {
            "workload": wl, "months_per_gpu": T_loc, "firms": N, "chars": panel.ncols,
            "problems_per_month": gres.nprob, "global_months": T_glob, "seed": seed,
            "parallelism": f"month-sharded x{world}" + (", RCCL all-gather of records + all-reduce of "
                                                        "predictive records (timed)" if world > 1 else ""),
        },
        "regressions_per_s": nfit * args.steps / dt,
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                     "traffic": traffic["bytes"] if traffic else None,
                     "traffic_ratio": traffic["bytes"] / dom_bytes if traffic else None,
                     "traffic_source": traffic["source"] if traffic else None,
                     "bytes_per_launch": dom_bytes, "avg_launch_ms": dom_ms,
                     "measured_read_peak": read_peak, "frac_of_measured_read": achieved / read_peak,
                     "measured_read_peak_source": "fm_stream_probe, 1 GiB, 16-B loads (bench._stream_read_gbs)",
                     "measured_copy_peak": copy_peak, "frac_of_measured_copy": achieved / copy_peak,
                     "measured_copy_peak_source": "fm_stream_copy_probe, 1 GiB read + 1 GiB written, 16-B accesses (bench._stream_copy_gbs)",
                     "whole_pass": {"bytes_per_row": B_ROW, "achieved": whole, "frac": whole / HBM_PEAK_GBS,
                                    "ms_per_step": ms_step, "per": "rank"},
                     "select": sel_roof},
        "kernel_ms": {k: round(v, 4) for k, v in dev_ms.items()},
        "lib_sha16": _lib_sha(),
        "kernel_ms_eager_events": {k: round(v, 4) for k, v in kern.items()},
        "graph": not args.no_graph,
        "ingest": {"gen_ms": panel.gen_ms, "layout": "planes" if panel.cols is None else "f64",
                   "panel_hbm_bytes": _panel_bytes(panel),
                   "note": "the panel generated in HBM directly in its layout (fm_gen_panel_planes: high / low "
                           "32-bit planes, no FP64 columns, no separate layout pass), outside the timed step"},
    }
    if world > 1:
        result["scaling_note"] = ("value at N>1 is the C5 workload; its N=1 point is the N=1 line's "
                                  "c5_rank_shard.rows_per_s (same per-rank shard), the headline's "
                                  "weak-scaled rate is headline_weak.value")
    if world == 1 and workload == "headline" and not args.no_standardize:
        result["standardize"] = standardize_stage(panel, args, E, LW, dev)
    if args.check and rank == 0 and world == 1 and workload == "headline":
        result["check"] = check_against_oracle(panel, gres, summ, args, LW)
    if rank == 0 and world == 1 and workload == "headline" and not args.no_cpu:
        result["cpu_baseline"] = cpu_baseline(panel, args, LW)
    del step, panel, out, gres, summ, psumm
    E.LAST_LAUNCH.clear()
    torch.cuda.empty_cache()
    if rank == 0 and world == 1 and not args.no_chars:
        result["firm_chars"] = firm_chars_stage(args, E)
        E.LAST_LAUNCH.clear()
        torch.cuda.empty_cache()
    if world == 1 and workload == "headline" and not args.no_c5:
        result["c5_rank_shard"] = c5_shard_stage(args, E, LW, dev)
    if world > 1 and workload == "c5" and not args.no_headline:
        p2, s2 = make_step(args.months, args.firms, args.seed, world, rank, dev, E, LW, planes=not args.no_planes)
        d2, o2 = timed_steps(s2, args.steps, args.warmup, not args.no_graph, world, dev)
        rows2 = args.months * args.firms
        result["headline_weak"] = {"value": rows2 * world * args.steps / d2, "unit": "firm-month rows/s",
                                   "ms_per_step": d2 / args.steps * 1e3, "months_per_gpu": args.months,
                                   "firms": args.firms, "steps": args.steps,
                                   "whole_pass_frac": rows2 * B_ROW / (d2 / args.steps) / 1e9 / HBM_PEAK_GBS}
        del s2, p2, o2
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


def standardize_stage(panel, args, E, LW, dev):
    """BASELINE configs[2]'s "per-month winsorize/standardize" variant on the headline panel
    (reported beside the headline, not part of `value`): PipelineConfig(standardize=True) --
    the select kernels also return the clipped moments (the workgroup select path: moments
    need every value), the Gram sees z-scores (shift = mean, inv_scale = 1/sd), degenerate
    months are dropped -- replayed from a HIP graph and timed like the headline step."""
    from fmcore.step import ShardedStep
    cfg = LW.PipelineConfig(standardize=True)
    step = ShardedStep(panel, cfg, LW.table2_models())
    dt, out = timed_steps(step, args.steps, args.warmup, not args.no_graph, 1, dev)
    ms = dt / args.steps * 1e3
    rows = panel.nrows
    timer = E.KernelTimer()
    E.LAST_LAUNCH.clear()
    with timer:
        step.eager()
    torch.cuda.synchronize()
    kms = {t: round(E.time_launch(t, 10), 4) for t in ("fm_select_cuts", "fm_universe", "fm_gram", "fm_solve")
           if t in E.LAST_LAUNCH}
    res = {"ms_per_step": ms, "rows_per_s": rows / (ms * 1e-3), "steps": args.steps, "kernel_ms": kms,
           "whole_pass_frac": rows * B_ROW / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
           "note": "PipelineConfig(standardize=True) on the headline panel: winsorize + per-month z-scores "
                   "(A9) -> the same universes / models / time series; HIP graph replay"}
    del step, out
    E.LAST_LAUNCH.clear()
    torch.cuda.empty_cache()
    return res


def c5_shard_stage(args, E, LW, dev):
    """C5 (BASELINE configs[4]: 100,000 months x 20,000 firms x 15 chars over 8 GPUs) at one
    rank's size through the same ShardedStep the N>1 c5 workload runs: 12,500 months x 20,000
    firms = 250M rows (30 GB of FP64 columns) generated in HBM as rank 4 of 8 would, the local
    pass and the time-series stage on its months, replayed from a HIP graph and timed like the
    headline (the N=1 point of the c5 scaling curve).  Beside it, the time-series stage on the
    100,000-month series the 8-rank all-gather assembles (this pass's records tiled 8 times),
    which every rank of the 8-GPU run executes replicated."""
    T, N, world8, rank8 = args.c5_months, args.c5_firms, 8, 4
    from fmcore.step import ShardedStep
    p, gen_ms = gen_panel(T, N, C5_SEED, rank8 * T, dev, E, not args.no_planes)
    step = ShardedStep(p, LW.PipelineConfig(), LW.table2_models(), seg_lo=rank8 * T, seg_hi=(rank8 + 1) * T)
    dt, out = timed_steps(step, args.c5_steps, 1, not args.no_graph, 1, dev)
    ms = dt / args.c5_steps * 1e3
    rows = T * N
    gres = out[0]
    nfit = int(((gres.status & 1) != 0).sum().item())
    # per-kernel device times of the C5 shard (eager step, launches re-issued back to back)
    timer = E.KernelTimer()
    with timer:
        step.eager()
    torch.cuda.synchronize()
    kms = {t: round(E.time_launch(t, 3), 4) for t in ("fm_select_cuts", "fm_select_cuts[nyse]", "fm_gram",
                                                        "fm_solve") if t in E.LAST_LAUNCH}
    # the 100,000-month gathered series' time-series stage (replicated on every rank at N=8)
    res = gres
    lo, hi = rank8 * T, (rank8 + 1) * T
    rec_g = res.rec.repeat(world8, 1, 1).contiguous()
    st_g = res.status.repeat(world8, 1).contiguous()
    g = E.FMResult(problems=res.problems, rec=rec_g, status=st_g, pmax=res.pmax, moments=res.moments,
                   mom_stride=res.mom_stride)
    cfg = LW.PipelineConfig()

    from fmcore import dist as D
    prange = D.problem_block(res.nprob, world8, rank8)

    def ts(sharded):
        # sharded (what ShardedStep runs at N = 8): this rank's problem block of the summaries,
        # rolling means only where its own months' predictive records read them
        ix, summ, roll, pred, pst = LW.time_series_stage(g, cfg, moments=res.moments, seg_lo=lo, seg_hi=hi,
                                                         sum_range=prange if sharded else None,
                                                         roll_own=sharded)
        E.summarize_predictive(pred, pst, cfg.nw_lags, sum_range=prange if sharded else None)

    tsm = {}
    for sharded in (True, False):
        ts(sharded)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            ts(sharded)
        e1.record()
        e1.synchronize()
        tsm[sharded] = e0.elapsed_time(e1) / 3
    out_d = {"rows": rows, "months": T, "firms": N, "seed": C5_SEED, "steps": args.c5_steps,
             "ms_per_pass": ms, "rows_per_s": rows / (ms * 1e-3), "regressions_per_s": nfit / (ms * 1e-3),
             "whole_pass_frac": rows * B_ROW / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, "kernel_ms": kms,
             "ms_ts_gathered_100k": tsm[True], "ms_ts_gathered_100k_replicated": tsm[False],
             "gen_ms": gen_ms, "panel_hbm_bytes": _panel_bytes(p),
             "note": "fmcore.step.ShardedStep at world 1 (HIP graph replay, timed like the headline): the "
                     "N=1 point of the c5 workload; ms_ts_gathered_100k = rank 4's share of the time-series "
                     "stage on the 100,000-month series an 8-rank all-gather assembles (its problem block's "
                     "summaries, rolling means / predictive records of its own months; _replicated: the "
                     "whole stage, as every rank ran it before round 6)"}
    del step, p, out, gres, res, rec_g, st_g, g
    E.LAST_LAUNCH.clear()
    torch.cuda.empty_cache()
    return out_d


def _stream_read_gbs(E, dev, nbytes=1 << 30, reps=10):
    """The achievable HBM READ rate on this box: the library's own fm_stream_probe (16-byte
    loads, four in flight per thread, 2,048 workgroups) over a 1 GiB buffer, HIP events on
    the launch stream.  The Gram is a read stream (its partials are < 1 % of its bytes), so
    this -- not the 8 TB/s spec -- is the ceiling its roofline fraction is also quoted
    against (MI355X_MICROARCH.md: 6.29 TB/s measured)."""
    a = torch.ones(nbytes // 8, dtype=torch.float64, device=dev)
    E.stream_probe(a)
    torch.cuda.synchronize()
    ms = E.time_launch("fm_stream_probe", reps)
    del a
    E.LAST_LAUNCH.pop("fm_stream_probe", None)
    torch.cuda.empty_cache()
    return nbytes / (ms * 1e-3) / 1e9


def _stream_copy_gbs(E, dev, nbytes=1 << 30, reps=10):
    """The achievable HBM COPY rate (read + write bytes) on this box: the library's own
    fm_stream_copy_probe (the read probe's 16-byte stream, each pair stored) over 1 GiB,
    HIP events on the launch stream via time_launch."""
    a = torch.ones(nbytes // 8, dtype=torch.float64, device=dev)
    b = torch.empty_like(a)
    E.stream_copy_probe(a, b)
    torch.cuda.synchronize()
    ms = E.time_launch("fm_stream_copy_probe", reps)
    del a, b
    E.LAST_LAUNCH.pop("fm_stream_copy_probe", None)
    torch.cuda.empty_cache()
    return 2 * nbytes / (ms * 1e-3) / 1e9


def _panel_bytes(panel):
    """HBM bytes the panel holds (values in their layout, me, NYSE flags, month offsets)."""
    n = 0
    for t in (panel.cols, panel.planes, panel.me, panel.nyse, panel.seg_off):
        if t is not None:
            n += t.numel() * t.element_size()
    return n


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
    ms = E.time_launch("fm_rolling_std", 20)
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
    cols = {name: panel.column_host(i, n) for i, name in enumerate(panel.names)}
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
    # optional month-parallel variant: all months of the panel, one contiguous
    # month block per worker process, 1 BLAS thread each
    if args.cpu_procs > 1:
        from oracle import month_parallel as MP
        try:
            avail = len(os.sched_getaffinity(0))
        except AttributeError:  # pragma: no cover
            avail = os.cpu_count() or 1
        procs = max(1, min(args.cpu_procs, avail, 16))
        n_all = panel.nrows
        cols_all = {name: panel.column_host(i) for i, name in enumerate(panel.names)}
        sec, _ = MP.run(cols_all, panel.seg_off_h, panel.me.cpu().numpy(),
                        panel.nyse.cpu().numpy().astype(bool), models, procs)
        out["month_parallel"] = {"value": n_all / sec, "unit": "firm-month rows/s", "cores": procs,
                                 "kind": "port", "seconds": sec,
                                 "sample": f"all {panel.nseg} months x {args.firms} firms, {procs} processes x "
                                           f"1 BLAS thread, one contiguous month block each "
                                           f"(oracle/month_parallel.py)"}
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
    cols = {name: panel.column_host(i, n) for i, name in enumerate(panel.names)}
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

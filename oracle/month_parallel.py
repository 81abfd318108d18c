"""Month-parallel CPU baseline (TEST / BENCH INFRASTRUCTURE ONLY -- never imported by the
product path; bench.py's cpu_baseline leg uses it beside the 1-core timing).

The reference is a single-process loop over months (src/regressions.py:43,
src/calc_Lewellen_2014.py:516-527); SURVEY.md §8(d) allows an optional, clearly labeled
multi-process month-parallel variant of the CPU path.  Every worker process runs
fm_oracle.pipeline_arrays (winsorize -> universes -> 11 monthly pinv regressions per month
-> summaries, rolling means and forecasts of its block) on one contiguous block of months;
the blocks' cross-sections are exactly the single-process ones (months are independent),
the per-block time-series work is the negligible remainder."""
from __future__ import annotations

import multiprocessing as mp
import time

import numpy as np


def _block(job):
    from threadpoolctl import threadpool_limits

    from oracle import fm_oracle as O
    cols, seg, me, nyse, models = job
    with threadpool_limits(1):
        out = O.pipeline_arrays(cols, seg, me, nyse, models, None)
    return sum(len(v["month"]) for v in out.values())


def _warm(_):
    from oracle import fm_oracle  # noqa: F401
    return 0


def run(cols, seg_off, me, nyse, models, nprocs):
    """Time the full pass over all months of the month-sorted arrays with `nprocs` worker
    processes (spawned; pool start-up and imports are outside the timed region, handing
    each worker its block's arrays is inside it).  Returns (seconds, fitted problems)."""
    T = len(seg_off) - 1
    edges = np.linspace(0, T, nprocs + 1).astype(np.int64)
    jobs = []
    for b in range(nprocs):
        t0, t1 = int(edges[b]), int(edges[b + 1])
        if t1 <= t0:
            continue
        r0, r1 = int(seg_off[t0]), int(seg_off[t1])
        jobs.append(({k: v[r0:r1] for k, v in cols.items()}, seg_off[t0:t1 + 1] - r0, me[r0:r1],
                     nyse[r0:r1], models))
    ctx = mp.get_context("spawn")
    with ctx.Pool(len(jobs)) as pool:
        pool.map(_warm, range(len(jobs)))
        t = time.perf_counter()
        fitted = sum(pool.map(_block, jobs, chunksize=1))
        dt = time.perf_counter() - t
    return dt, fitted

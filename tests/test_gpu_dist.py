"""The month-sharded step bench.py times (fmcore.step.ShardedStep: three graph-replayed
phases with the record all-gather and the predictive SUM all-reduce between them), run as
two processes on cuda:0 over gloo (RCCL refuses two ranks on one device), against the
single-process step on the concatenated panel: monthly records, status, FM summaries and
predictive summaries bit for bit (sharding does not change the per-month
arithmetic)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
T_LOC, FIRMS, SEED = 96, 700, 11


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _host(out):
    gres, summ, psumm = out
    d = {"rec": gres.rec, "status": gres.status, "mean": summ.mean, "se": summ.se, "t": summ.tstat,
         "nobs": summ.nobs, "pmean": psumm.mean, "pse": psumm.se, "pt": psumm.tstat, "pnobs": psumm.nobs}
    return {k: v.cpu().numpy() for k, v in d.items()}


# Gram plans of the GLOBAL panel (as bench.make_step): the default policy (whole months at
# this size) and a balanced plan (R-row blocks of the global row space that straddle the
# ranks' month ranges), each identical on every rank and in the 1-rank run
PLANS = {
    "default": lambda T_glob: None,
    "balanced": lambda T_glob: ("balanced", -(-T_glob * FIRMS // 61)),   # R = 2,204 at 2 x 96 months
}


def _plan(name, T_glob):
    from fmcore import engine as E
    pol = PLANS[name](T_glob)
    return pol if pol is not None else E.chunk_policy(T_glob * FIRMS, T_glob, FIRMS)


def _run(world, rank, T_loc, plan="default"):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "fm-returnprediction_amd"))
    from fmcore import engine as E
    from fmcore import lewellen as LW
    from fmcore.step import ShardedStep
    dev = E.require_device()
    T_glob = T_loc * world
    panel = E.panel_synthetic(T_loc, FIRMS, SEED, month0=rank * T_loc, device=dev)
    panel.chunk_policy = _plan(plan, T_glob)   # the GLOBAL panel's plan, as bench.make_step
    panel.row_origin = rank * T_loc * FIRMS
    step = ShardedStep(panel, LW.PipelineConfig(), LW.table2_models(), world=world, rank=rank,
                       seg_lo=rank * T_loc, seg_hi=(rank + 1) * T_loc, global_months=T_glob,
                       counts=[T_loc] * world)
    eager = _host(step.eager())
    step.capture()
    step.replay()
    graph = _host(step.replay())
    torch.cuda.synchronize()
    return eager, graph


def _worker(rank, world, port, q, plan):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q.put((rank, _run(world, rank, T_LOC, plan)))
    except Exception as e:   # surface the failure in the parent
        q.put((rank, repr(e)))
    dist.destroy_process_group()


@pytest.mark.parametrize("plan", sorted(PLANS))
def test_two_ranks_one_gpu_bit_identical_to_single_process(plan):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, plan)) for r in range(2)]
    for p in procs:
        p.start()
    outs = dict(q.get(timeout=300) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(2):
        assert not isinstance(outs[r], str), outs[r]
    ref_eager, ref_graph = _run(1, 0, 2 * T_LOC, plan)
    for k, v in ref_graph.items():
        assert np.array_equal(v, ref_eager[k], equal_nan=v.dtype.kind == "f"), ("graph vs eager", k)
    for r in range(2):
        for mode in (0, 1):
            got = outs[r][mode]
            for k, v in ref_graph.items():
                assert np.array_equal(got[k], v, equal_nan=v.dtype.kind == "f"), (r, mode, k)

"""The RCCL device path of the month-sharded step, executed on one GPU (SURVEY.md §8(e)
exchange steps 1-2): a 1-rank `nccl` process group on cuda:0 (RCCL refuses two ranks on one
device, so the multi-rank runs use gloo; see tests/test_gpu_dist.py).

* fmcore.dist.gather_records_into takes its all_gather_into_tensor branch and
  combine_predictive its device all_reduce on HIP tensors;
* ShardedStep with the exchanges forced at world size 1 (three HIP graphs, the collectives
  between their replays) returns records, status, FM summaries and predictive summaries bit
  for bit equal to the single-graph step without exchanges, eager and replayed.
The group lives in a spawned child process, so a failing RCCL init cannot leave a process
group behind in the test runner."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


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


def _same(a, b):
    return a.shape == b.shape and np.array_equal(a, b, equal_nan=a.dtype.kind == "f")


def _worker(port, q):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "fm-returnprediction_amd"))
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    try:
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
        from fmcore import dist as D
        from fmcore import engine as E
        from fmcore import lewellen as LW
        from fmcore.step import ShardedStep
        checks = {"backend": dist.get_backend()}
        # the exchange helpers on device tensors (no host staging on nccl)
        rng = np.random.default_rng(3)
        rec = torch.from_numpy(rng.standard_normal((37, 11, 18))).to(dev)
        st = torch.from_numpy(rng.integers(0, 4, (37, 11)).astype(np.int32)).to(dev)
        checks["host_staged"] = D._host_staged(rec, None)
        r_out = torch.full_like(rec, float("nan"))
        s_out = torch.full_like(st, -7)
        D.gather_records_into(rec, st, r_out, s_out)                 # counts None: into_tensor
        D.gather_records_into(rec, st, r_out, s_out, counts=[37])    # equal counts: into_tensor
        checks["gather"] = bool(torch.equal(r_out, rec) and torch.equal(s_out, st))
        pred = torch.from_numpy(rng.standard_normal((11, 37, 4))).to(dev)
        pst = torch.from_numpy(rng.integers(0, 2, (11, 37)).astype(np.int32)).to(dev)
        p0, s0 = pred.clone(), pst.clone()
        D.combine_predictive(pred, pst)
        checks["combine"] = bool(torch.equal(pred, p0) and torch.equal(pst, s0))
        # the three-graph sharded step with the collectives, vs the single-graph step
        panel = E.panel_synthetic(96, 700, 11, device=dev)
        cfg, mc = LW.PipelineConfig(), LW.table2_models()
        ref = ShardedStep(panel, cfg, mc)
        ref_eager = _host(ref.eager())
        ref.capture()
        ref.replay()
        ref_graph = _host(ref.replay())
        xs = ShardedStep(panel, cfg, mc, world=1, rank=0, counts=[panel.nseg], exchange=True)
        x_eager = _host(xs.eager())
        xs.capture()
        assert len(xs.graphs) == 3
        xs.replay()
        x_graph = _host(xs.replay())
        torch.cuda.synchronize()
        for k in ref_graph:
            checks[f"ref:{k}"] = _same(ref_graph[k], ref_eager[k])
            checks[f"eager:{k}"] = _same(x_eager[k], ref_eager[k])
            checks[f"graph:{k}"] = _same(x_graph[k], ref_eager[k])
        q.put(checks)
        dist.destroy_process_group()
    except Exception as e:   # surface the failure in the parent
        import traceback
        q.put("".join(traceback.format_exception(e)))


def test_rccl_exchanges_one_rank_bit_identical():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(_free_port(), q))
    p.start()
    try:
        out = q.get(timeout=240)
    finally:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
    assert not isinstance(out, str), out
    assert p.exitcode == 0
    assert out.pop("backend") == "nccl"
    assert out.pop("host_staged") is False
    bad = [k for k, v in out.items() if not v]
    assert not bad, bad

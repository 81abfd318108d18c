"""World-size-2 gloo tests (CPU) of the month-sharded path: record all-gather with uneven
shards, the predictive sum-combine and max-over-ranks timing.  The per-rank records are
seeded random arrays (the exchange code is data-agnostic); the gathered / combined result
must equal the single-process arrays bit for bit.  That the real device pipeline, split by
shard_bounds and run per range with the global chunk policy, is bit-identical to the
unsharded run is tested on the GPU (tests/test_gpu_parity.py::test_sharded_pipeline_bit_identical)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _records(T, P, rs, seed):
    rng = np.random.default_rng(seed)
    rec = rng.standard_normal((T, P, rs))
    st = (rng.random((T, P)) < 0.9).astype(np.int32)
    return rec, st


def _worker(rank, world, port, T, P, rs, q):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "fm-returnprediction_amd"))
    from fmcore import dist as D
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rec, st = _records(T, P, rs, 5)
    rows = np.r_[np.full(T // 3, 10), np.full(T - T // 3, 30)]       # uneven month sizes
    bounds = D.shard_bounds(rows, world)
    s0, s1 = bounds[rank]
    counts = [e - s for s, e in bounds]
    g_rec, g_st = D.gather_records(torch.from_numpy(rec[s0:s1]), torch.from_numpy(st[s0:s1]), counts)
    ok_gather = bool(np.array_equal(g_rec.numpy(), rec) and np.array_equal(g_st.numpy(), st))
    # predictive rows: compact index i owned by the rank whose month range holds it; other
    # ranks' rows hold the -0.0 record the device kernels write there (fm_ts.hip), so the SUM
    # returns the owner's bits, signed zeros, infinities and NaNs included
    months = np.nonzero(st[:, 0])[0]
    pred_full = np.random.default_rng(9).standard_normal((1, len(months), 4))
    pred_full[0, ::5, 0] = -0.0
    pred_full[0, 1::5, 1] = 0.0
    pred_full[0, 2::7, 2] = -np.inf
    pred_full[0, 3::7, 0] = np.nan
    mine = (months >= s0) & (months < s1)
    pred = np.where(mine[None, :, None], pred_full, -0.0)
    pst = mine.astype(np.int32)[None, :]
    tp, ts = D.combine_predictive(torch.from_numpy(pred.copy()), torch.from_numpy(pst.copy()))
    ok_pred = bool(np.array_equal(tp.numpy().view(np.int64), pred_full.view(np.int64)) and (ts.numpy() == 1).all())
    mx = D.max_over_ranks(float(rank + 1), torch.device("cpu"))
    # gather_records_into (the call bench.py makes, into static global buffers): uneven
    # counts take the padded all_gather, equal counts all_gather_into_tensor
    r_out = torch.full((T, P, rs), np.nan, dtype=torch.float64)
    s_out = torch.full((T, P), -7, dtype=torch.int32)
    D.gather_records_into(torch.from_numpy(rec[s0:s1]), torch.from_numpy(st[s0:s1]), r_out, s_out, counts)
    ok_into = bool(np.array_equal(r_out.numpy(), rec) and np.array_equal(s_out.numpy(), st))
    Te = (T // world) * world
    per = Te // world
    r_eq = torch.full((Te, P, rs), np.nan, dtype=torch.float64)
    s_eq = torch.full((Te, P), -7, dtype=torch.int32)
    D.gather_records_into(torch.from_numpy(rec[rank * per:(rank + 1) * per]),
                          torch.from_numpy(st[rank * per:(rank + 1) * per]), r_eq, s_eq)
    ok_into_eq = bool(np.array_equal(r_eq.numpy(), rec[:Te]) and np.array_equal(s_eq.numpy(), st[:Te]))
    q.put((rank, ok_gather and ok_into and ok_into_eq, ok_pred, mx, counts))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_records_equal_single_process(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, 37, 3, 7, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok_gather, ok_pred, mx, counts in out:
        assert ok_gather and ok_pred, rank
        assert mx == float(world)
        assert sum(counts) == 37


FIXTURE = os.path.join(ROOT, "tests", "golden", "shard_pred.npz")


def _pred_worker(rank, world, port, q):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "fm-returnprediction_amd"))
    from fmcore import dist as D
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = np.load(FIXTURE)
    # world 2: rank 0 holds shards 0 and 1 (their rows are disjoint), rank 1 shard 2
    mine = [0, 1] if (world == 2 and rank == 0) else [2] if world == 2 else [rank]
    pred = sum(g[f"pred{i}"] for i in mine)
    pst = sum(g[f"pst{i}"] for i in mine)
    tp, ts = D.combine_predictive(torch.from_numpy(pred.copy()), torch.from_numpy(pst.copy()))
    tp, ts = tp.numpy(), ts.numpy()
    keep = (g["full_pst"] & 1) != 0
    same_st = bool(np.array_equal(ts, g["full_pst"]))
    a, b = tp[keep], g["full_pred"][keep]
    same_pred = bool(np.array_equal(np.isnan(a), np.isnan(b)) and np.array_equal(a[~np.isnan(a)], b[~np.isnan(b)]))
    q.put((rank, same_st, same_pred))
    dist.destroy_process_group()


@pytest.mark.skipif(not os.path.exists(FIXTURE), reason="tools/dump_shard_pred.py fixture not generated")
@pytest.mark.parametrize("world", [2, 3])
def test_combine_predictive_real_shard_outputs(world):
    """combine_predictive on the real device pipeline's per-shard predictive records
    (tests/golden/shard_pred.npz, written by tools/dump_shard_pred.py on the GPU: a ragged
    96-month panel in 3 shard_bounds ranges, each shard's time-series stage with its own
    moments).  The SUM all-reduce relies on every row of another shard's months being
    a zero record (-0.0 since round 6, +0.0 in fixtures dumped before; status 0); the combined
    result must equal the unsharded run bit for bit on every fitted row, and the status words
    exactly."""
    g = np.load(FIXTURE)
    for i in range(3):   # the fixture's premise: the shards' fitted rows are disjoint
        for j in range(i + 1, 3):
            assert not ((g[f"pst{i}"] & 1) & (g[f"pst{j}"] & 1)).any()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pred_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, same_st, same_pred in out:
        assert same_st and same_pred, rank


# ------------------------------------------------------------ bench.py --gpus N launcher
def _bench():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_bench_launch_plan():
    """--gpus N without a launcher spawns N ranks through torch.distributed.run on
    127.0.0.1; under a launcher (WORLD_SIZE set) the process is one rank; a disagreeing
    --gpus exits non-zero instead of measuring one rank."""
    B = _bench()
    argv = ["--gpus", "8", "--steps", "5"]
    cmd = B.launch_plan(8, {}, argv, port=29511)
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--master-addr=127.0.0.1" in cmd and "--master-port=29511" in cmd
    assert cmd[-len(argv):] == argv and cmd[-len(argv) - 1].endswith("bench.py")
    assert B.launch_plan(8, {"WORLD_SIZE": "8"}, argv) is None
    assert B.launch_plan(None, {"WORLD_SIZE": "4"}, []) is None
    assert B.launch_plan(1, {}, ["--gpus", "1"]) is None
    assert B.launch_plan(None, {}, []) is None
    with pytest.raises(SystemExit) as e:
        B.launch_plan(8, {"WORLD_SIZE": "1"}, argv)
    assert e.value.code == 2
    with pytest.raises(SystemExit) as e:
        B.launch_plan(2, {"WORLD_SIZE": "4"}, argv)
    assert e.value.code == 2


def _run_bench(args, extra_env=None):
    import json
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK",
                                                           "MASTER_ADDR", "MASTER_PORT")}
    env.update(extra_env or {})
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True,
                       text=True, env=env, timeout=240)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    return p.returncode, (json.loads(lines[-1]) if lines else None), p.stderr


def test_bench_spawns_n_ranks_itself():
    """The real launch path, no wrapper: `bench.py --gpus 2` starts two ranks that join one
    gloo group (--launch-probe stops before any GPU call); rank 0's line says so."""
    rc, out, err = _run_bench(["--gpus", "2", "--launch-probe"])
    assert rc == 0, err[-2000:]
    assert out == {"n_gpus": 2, "dist_backend": "gloo", "dist_world": 2, "rank": 0}
    rc, out, err = _run_bench(["--gpus", "1", "--launch-probe"])
    assert rc == 0 and out["n_gpus"] == 1 and out["dist_world"] == 1


def test_bench_rejects_gpus_world_mismatch():
    rc, out, err = _run_bench(["--gpus", "4", "--launch-probe"], {"WORLD_SIZE": "2"})
    assert rc == 2 and out is None and "WORLD_SIZE=2" in err

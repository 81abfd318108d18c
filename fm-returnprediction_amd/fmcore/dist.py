"""Month sharding across GPUs (one process per GPU, torch.distributed over RCCL/xGMI).

Every panel-sized step is independent per month (cuts, universes, Gram, solve), so each
rank owns a contiguous month range, balanced by row count, and never exchanges panel rows.
The only exchanges:
  1. all-gather of the per-(month, problem) records {intercept, slopes, R2, N} and status
     (a few KB per month) before the time-series stage, which every rank then runs on the
     full series, each doing only its share: the FM means / Newey-West summaries of its
     block of problems (problem_block) and the 120-month rolling means and predictive-slope
     records of its own months (the gathered series supplies the window halo);
  2. a SUM all-reduce of the predictive-slope records and the summaries (every entry has
     exactly one owner; the others hold -0.0 / 0, so the sum is the owner's value bit for
     bit, signed zeros included);
  3. a SUM all-reduce of the predictive summaries (again one owner per problem).
The helpers are device-agnostic so the same code runs under gloo on CPU in the tests.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist


def shard_bounds(seg_rows, world):
    """Contiguous month ranges [s0, s1) per rank, balanced by cumulative row count."""
    seg_rows = np.asarray(seg_rows, dtype=np.int64)
    T = len(seg_rows)
    cum = np.concatenate([[0], np.cumsum(seg_rows)])
    total = cum[-1]
    bounds = [0]
    for r in range(1, world):
        target = total * r / world
        s = int(np.searchsorted(cum, target, side="left"))
        s = min(max(s, bounds[-1]), T)
        bounds.append(s)
    bounds.append(T)
    return [(bounds[r], bounds[r + 1]) for r in range(world)]


def _host_staged(t, group):
    """gloo moves host memory: device tensors are staged through host copies (the tests run
    the sharded step as several processes on one GPU over gloo; RCCL takes device memory)."""
    return t.is_cuda and dist.get_backend(group) == "gloo"


def _gather_rows(t, counts, group=None):
    """All-gather a [T_local, ...] tensor whose first dim differs per rank."""
    world = dist.get_world_size(group)
    tmax = max(counts)
    pad = torch.zeros((tmax,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    pad[: t.shape[0]] = t
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad, group=group)
    return torch.cat([parts[r][: counts[r]] for r in range(world)], dim=0)


def gather_records(rec, status, counts, group=None):
    """Global [T, P, rs] records and [T, P] status from each rank's local months."""
    return _gather_rows(rec, counts, group), _gather_rows(status, counts, group)


def gather_records_into(rec, status, rec_out, status_out, counts=None, group=None):
    """gather_records into preallocated global buffers (static addresses, so the stages
    around the exchange can be replayed from HIP graphs).  Equal month counts per rank use
    one all_gather_into_tensor per buffer."""
    world = dist.get_world_size(group)
    if _host_staged(rec, group):
        r, s = gather_records(rec.cpu(), status.cpu(), counts or [rec.shape[0]] * world, group)
        rec_out.copy_(r)
        status_out.copy_(s)
    elif counts is None or len(set(counts)) == 1:
        dist.all_gather_into_tensor(rec_out, rec.contiguous(), group=group)
        dist.all_gather_into_tensor(status_out, status.contiguous(), group=group)
    else:
        r, s = gather_records(rec, status, counts, group)
        rec_out.copy_(r)
        status_out.copy_(s)
    assert rec_out.shape[0] == (rec.shape[0] * world if counts is None else sum(counts))
    return rec_out, status_out


def problem_block(nprob, world, rank):
    """Contiguous problem range [p0, p1) of a rank for the sharded FM summaries (blocks
    differ in size by at most one; empty when there are more ranks than problems)."""
    return (nprob * rank) // world, (nprob * (rank + 1)) // world


def combine_sum(tensors, group=None):
    """SUM all-reduce of each tensor in place.  Every entry has one owner rank; the others
    hold -0.0 (floats) or 0 (integers), so the result is the owner's value bit for bit:
    v + (-0.0) == v for every v, signed zeros, infinities and NaNs included, in any order."""
    for t in tensors:
        if _host_staged(t, group):
            h = t.cpu()
            dist.all_reduce(h, op=dist.ReduceOp.SUM, group=group)
            t.copy_(h)
        else:
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return tensors


def combine_predictive(pred, pst, group=None):
    """Rows of other ranks' months are -0.0 records / status 0 in `pred`/`pst` (fm_ts.hip):
    a SUM all-reduce merges them exactly (each compact row has exactly one owner)."""
    combine_sum((pred, pst), group)
    return pred, pst


def max_over_ranks(x, device, group=None):
    if dist.get_backend(group) == "gloo":
        device = torch.device("cpu")
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())

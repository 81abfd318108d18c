"""One step of the month-sharded full Fama-MacBeth pass (what bench.py times).

A step is three device phases with the exchanges of SURVEY.md §8(e) between them:

  phase_local   cuts, universes, batched Gram + solve of this rank's months
  exchange 1    all-gather of the monthly records into static global buffers
  phase_ts      time-series stage on the gathered series, this rank's share only: the FM
                means / NW of its problem block (dist.problem_block), the rolling means and
                predictive records of its own months
  exchange 2    SUM all-reduce of the predictive records and the summaries (one owner each;
                the others hold -0.0 / 0)
  phase_pred    FM summary of the predictive slopes of its problem block
  exchange 3    SUM all-reduce of the predictive summaries

Without exchanges (world size 1, no process group) the whole step can be replayed from ONE
HIP graph; otherwise each phase is its own graph (static buffers), with the collectives
between replays.  ``exchange=True`` at world size 1 (a 1-rank process group) runs the
three-graph path with the collectives anyway -- the RCCL device path, executed on one GPU.
"""
from __future__ import annotations

import torch

from . import dist as D
from . import engine as E
from . import lewellen as LW


class ShardedStep:
    def __init__(self, panel: E.DevicePanel, cfg: LW.PipelineConfig, model_cols, world=1, rank=0,
                 seg_lo=0, seg_hi=None, global_months=None, counts=None, group=None, exchange=None,
                 shard_ts=None):
        self.panel, self.cfg, self.model_cols = panel, cfg, model_cols
        self.world, self.rank, self.group = world, rank, group
        self.seg_lo = seg_lo
        self.seg_hi = seg_lo + panel.nseg if seg_hi is None else seg_hi
        if counts is not None and len(counts) != world:
            raise ValueError("counts needs one month count per rank")
        if global_months is None:
            global_months = sum(counts) if counts is not None else panel.nseg * world
        if counts is not None and global_months != sum(counts):
            raise ValueError("global_months must equal sum(counts)")
        self.global_months = global_months
        self.counts = counts
        self.exchange = world > 1 if exchange is None else bool(exchange)
        if world > 1 and not self.exchange:
            raise ValueError("a sharded step (world > 1) needs its exchanges")
        # the time-series stage split across the ranks (problem blocks, own-month rolling);
        # False: every rank runs all of it on the gathered series (round-5 behaviour)
        self.shard_ts = self.exchange if shard_ts is None else bool(shard_ts) and self.exchange
        self.rec_g = self.st_g = None
        self.graphs = None
        self._out = None

    def _sum_range(self, nprob):
        return D.problem_block(nprob, self.world, self.rank) if self.shard_ts else None

    # ---- phases ------------------------------------------------------------------------
    def phase_local(self):
        res, names, cuts, level, bp = LW.local_stage(self.panel, self.cfg, self.model_cols)
        if self.exchange and self.rec_g is None:
            dev = res.rec.device
            self.rec_g = torch.empty((self.global_months,) + tuple(res.rec.shape[1:]), dtype=res.rec.dtype,
                                     device=dev)
            self.st_g = torch.empty((self.global_months,) + tuple(res.status.shape[1:]), dtype=res.status.dtype,
                                    device=dev)
        return res

    def exchange_records(self, res):
        if self.exchange:
            D.gather_records_into(res.rec, res.status, self.rec_g, self.st_g, self.counts, self.group)

    def phase_ts(self, res):
        gres = res
        if self.exchange:
            gres = E.FMResult(problems=res.problems, rec=self.rec_g, status=self.st_g, pmax=res.pmax,
                              moments=res.moments, mom_stride=res.mom_stride)
        ix, summ, roll, pred, pst = LW.time_series_stage(gres, self.cfg, moments=res.moments,
                                                         seg_lo=self.seg_lo, seg_hi=self.seg_hi,
                                                         sum_range=self._sum_range(res.nprob),
                                                         roll_own=self.shard_ts)
        self._summ = summ
        return gres, summ, pred, pst

    def exchange_pred(self, pred, pst):
        if not self.exchange:
            return
        ts = []
        if pred is not None:
            ts += [pred, pst]
        if self.shard_ts:
            sm = self._summ
            ts += [sm.mean, sm.se, sm.tstat, sm.nobs]
        D.combine_sum(ts, self.group)

    def phase_pred(self, pred, pst):
        if pred is None:
            return None
        psumm, _ = E.summarize_predictive(pred, pst, self.cfg.nw_lags, sum_range=self._sum_range(pred.shape[0]))
        return psumm

    def exchange_psumm(self, psumm):
        if self.shard_ts and psumm is not None:
            D.combine_sum((psumm.mean, psumm.se, psumm.tstat, psumm.nobs), self.group)

    # ---- whole step --------------------------------------------------------------------
    def eager(self):
        """(global FMResult, Summary, predictive Summary) with eager launches."""
        res = self.phase_local()
        self.exchange_records(res)
        gres, summ, pred, pst = self.phase_ts(res)
        self.exchange_pred(pred, pst)
        psumm = self.phase_pred(pred, pst)
        self.exchange_psumm(psumm)
        return gres, summ, psumm

    def capture(self):
        """Capture the phases as HIP graphs.  Every host-side cache (chunk plans, model
        plans) and the static exchange buffers must exist before capture: without a prior
        eager() step, one is run here first."""
        warmed = getattr(self.panel, "_chunk_cache", None) is not None and \
            bool(getattr(self.panel, "_group_cache", None))
        if not warmed or (self.exchange and self.rec_g is None):
            # host-side plans upload with host-to-device copies, which must not be captured
            self.eager()
            torch.cuda.synchronize()
        if not self.exchange:
            g1 = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g1):
                res = self.phase_local()
                gres, summ, pred, pst = self.phase_ts(res)
                psumm = self.phase_pred(pred, pst)
            self.graphs = (g1,)
            self._out = (gres, summ, psumm)
            self._static = None
            return
        assert self.rec_g is not None and self.st_g is not None
        ga, gb = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        with torch.cuda.graph(ga):
            res = self.phase_local()
        self.exchange_records(res)
        with torch.cuda.graph(gb):
            gres, summ, pred, pst = self.phase_ts(res)
        self.exchange_pred(pred, pst)
        gc, psumm = None, None
        if pred is not None:   # no forecasts: no predictive phase to capture
            gc = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gc):
                psumm = self.phase_pred(pred, pst)
            self.exchange_psumm(psumm)
        self.graphs = (ga, gb, gc)
        self._psumm = psumm
        self._static = (res, pred, pst)
        self._out = (gres, summ, psumm)

    def replay(self):
        if self.graphs is None:
            return self.eager()
        if not self.exchange:
            self.graphs[0].replay()
            return self._out
        res, pred, pst = self._static
        ga, gb, gc = self.graphs
        ga.replay()
        self.exchange_records(res)
        gb.replay()
        self.exchange_pred(pred, pst)
        if gc is not None:
            gc.replay()
            self.exchange_psumm(self._psumm)
        return self._out

"""Device-resident Fama-MacBeth engine: host orchestration of libfm_hip kernels.

torch (ROCm) only provides device buffers and the stream; every computation on the hot
path is a libfm_hip kernel.  There is no CPU fallback: without a HIP device the
functions raise.

Layout in HBM (``DevicePanel``): the panel's C columns with rows sorted by (month, input
order) -- month segments are CSR ``seg_off[T+1]`` -- as an FP64 SoA block ``cols[C, n]``
and/or the split layout ``planes[2, C, n]`` (uint32 high / low words: the selects read the
high plane, the Gram both), plus optional ``me`` (FP64) and ``nyse`` (uint8) rows and a
uint8 universe ``level`` per row.  A panel built with ``layout="planes"`` holds no FP64
columns at all (half the HBM): the whole Table-2 pass reads the planes, and consumers of
FP64 columns (clip, forecasts, moments) get them from ``values()``.
"""
from __future__ import annotations

import itertools
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np
import torch

from . import _lib as L

# statsmodels/numpy quantile modes
LERP_NUMPY = 0
LERP_PANDAS = 1


def require_device():
    if not torch.cuda.is_available():
        raise RuntimeError("fmcore needs a HIP device (MI355X); none is visible and there is "
                           "no CPU fallback")
    L.load()
    return torch.device("cuda", torch.cuda.current_device())


def _ptr(t):
    return None if t is None else t.data_ptr()


class KernelTimer:
    """Records HIP events on the current stream around every libfm_hip launch made by
    this module while active (bench.py uses it for the per-kernel roofline)."""

    def __init__(self):
        self.events = {}

    def __enter__(self):
        global _TIMER
        _TIMER = self
        return self

    def __exit__(self, *exc):
        global _TIMER
        _TIMER = None

    def avg_ms(self, name):
        torch.cuda.synchronize()
        ev = self.events.get(name, [])
        if not ev:
            return float("nan")
        return float(np.mean([a.elapsed_time(b) for a, b in ev]))

    def names(self):
        return list(self.events)


_TIMER = None

# The latest argument struct of each struct-taking entry point, with the tensors it points
# to kept alive, so one kernel can be re-issued in isolation (time_launch).
LAST_LAUNCH = {}


def _remember(tag, name, struct, *keep):
    LAST_LAUNCH[tag] = (name, struct, keep)


def time_launch(tag, reps=20):
    """Average device milliseconds of the latest `tag` launch, re-issued `reps` times back
    to back on the current stream.  The host stays ahead of the device, so unlike events
    around single launches of a host-bound pipeline this excludes launch gaps.  The
    re-issued launches rewrite the same outputs with the same values."""
    name, struct, keep = LAST_LAUNCH[tag]
    st = _stream()
    args = (L.C.byref(struct),) if struct is not None else keep[1]
    L.call(name, *args, st)
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        L.call(name, *args, st)
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def _kcall(tag, name, *args):
    t = _TIMER
    if t is not None:
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
    L.call(name, *args)
    if t is not None:
        e1.record()
        t.events.setdefault(tag, []).append((e0, e1))


def _stream():
    return torch.cuda.current_stream().cuda_stream


# ------------------------------------------------------------------------------------------
# Panel
# ------------------------------------------------------------------------------------------
@dataclass
class DevicePanel:
    cols: Optional[torch.Tensor]       # [C, n] float64, contiguous (None: a planes-only panel)
    names: List[str]
    seg_off: torch.Tensor              # [T+1] int64 (device)
    seg_off_h: np.ndarray              # [T+1] int64 (host)
    months: object = None              # segment labels (host)
    me: Optional[torch.Tensor] = None  # [n] float64
    nyse: Optional[torch.Tensor] = None  # [n] uint8
    order: Optional[np.ndarray] = None   # sorted row -> original positional row
    chunk_rows: Optional[int] = None     # Gram chunking override (sharded runs: global policy)
    chunk_split: Optional[bool] = None   # split-month Gram plan (make_chunks_split) override
    planes: Optional[torch.Tensor] = None   # [2, C, n] int32: the values' high / low words
    chunk_policy: Optional[tuple] = None    # Gram plan of the GLOBAL panel (chunk_policy()), sharded runs
    row_origin: int = 0                     # global row of this panel's row 0 (balanced plans)
    planes_version: int = -1                # cols._version when the planes were made from cols

    @property
    def device(self):
        return (self.cols if self.cols is not None else self.planes).device

    def values(self):
        """The FP64 columns [C, n]: ``cols``, or for a planes-only panel a device merge of the
        planes (fm_merge_planes), made once and kept.  Off the Table-2 hot path (clip,
        forecasts, moments, the standardize variant)."""
        if self.cols is not None:
            return self.cols
        m = self.__dict__.get("_merged")
        if m is None:
            C, n = self.planes.shape[1], self.planes.shape[2]
            m = torch.empty((C, n), dtype=torch.float64, device=self.planes.device)
            _kcall("fm_merge_planes", "fm_merge_planes", self.planes[0].data_ptr(), self.planes[1].data_ptr(),
                   self.planes.stride(1), C, n, m.data_ptr(), m.stride(0), _stream())
            self.__dict__["_merged"] = m
        return m

    def column_host(self, i, n=None):
        """Column i (its first n rows) as a host float64 array, from the planes without an
        FP64 device copy when the panel has none."""
        n = self.nrows if n is None else n
        if self.cols is not None:
            return self.cols[i, :n].cpu().numpy()
        hi = self.planes[0, i, :n].cpu().numpy().astype(np.uint32).astype(np.uint64)
        lo = self.planes[1, i, :n].cpu().numpy().astype(np.uint32).astype(np.uint64)
        return ((hi << np.uint64(32)) | lo).view(np.float64)

    def check_planes(self):
        """The planes must still be the FP64 columns' words: an in-place write to ``cols``
        after the planes were made (torch bumps the tensor's version counter) is refused."""
        if self.planes is not None and self.cols is not None and self.planes_version >= 0 and \
                self.cols._version != self.planes_version:
            raise RuntimeError("panel.cols was modified in place after its planes were made: call "
                               "split_planes(panel) again (or build a new panel)")

    @property
    def nrows(self):
        return int(self.seg_off_h[-1])

    @property
    def nseg(self):
        return len(self.seg_off_h) - 1

    @property
    def ncols(self):
        return self.cols.shape[0] if self.cols is not None else self.planes.shape[1]

    @property
    def stride(self):
        return self.values().stride(0)

    @property
    def max_seg_len(self):
        return int(np.diff(self.seg_off_h).max()) if self.nseg else 0

    def col(self, name):
        return self.names.index(name)


def month_segments(labels):
    """Factorize month labels (sorted) -> (codes, uniques, stable order of valid rows,
    seg_off).  Rows with a missing label are excluded (pandas groupby/dropna drop them)."""
    import pandas as pd
    codes, uniq = pd.factorize(labels, sort=True)
    codes = np.asarray(codes)
    if len(uniq) < 32767:
        # numpy sorts 16-bit keys stably by radix (vs a merge sort on int64): ~4x at 3M rows
        codes = codes.astype(np.int16)
    order = np.argsort(codes, kind="stable")
    order = order[codes[order] >= 0]
    counts = np.bincount(codes[codes >= 0], minlength=len(uniq))
    seg_off = np.zeros(len(uniq) + 1, dtype=np.int64)
    np.cumsum(counts, out=seg_off[1:])
    return codes, uniq, order, seg_off


def gather_layout(raw, perm, layout="f64"):
    """The device gather of an ingest: FP64 columns ``raw`` [C, n_in] (input row order) ->
    month-major rows in the panel's layout, (cols, planes): "f64" the FP64 columns, "planes"
    the high / low 32-bit words gathered straight from the raw words (no FP64 panel copy),
    "both"."""
    if layout not in PANEL_LAYOUTS:
        raise ValueError(f"layout must be one of {PANEL_LAYOUTS}")
    cols = planes = None
    if layout != "planes":
        cols = raw.index_select(1, perm).contiguous()
    if layout != "f64":
        C = raw.shape[0]
        words = raw.contiguous().view(torch.int32).view(C, -1, 2)   # little-endian: [..., 1] = high word
        planes = torch.empty((2, C, max(perm.numel(), 1)), dtype=torch.int32, device=raw.device)
        planes[0, :, :perm.numel()] = words[:, :, 1].index_select(1, perm)
        planes[1, :, :perm.numel()] = words[:, :, 0].index_select(1, perm)
    return cols, planes


def panel_from_arrays(arrays: Sequence[np.ndarray], names, labels, me=None, nyse=None,
                      device=None, layout="f64"):
    """Upload host columns (original row order) and permute them month-major on device, into
    the panel's ``layout`` ("f64", "planes": the split layout only, "both")."""
    device = device or require_device()
    _, uniq, order, seg_off = month_segments(labels)
    n_in = len(labels)
    host = np.empty((len(arrays), n_in), dtype=np.float64)
    for i, a in enumerate(arrays):
        host[i] = np.asarray(a, dtype=np.float64)
    raw = torch.from_numpy(host).to(device, non_blocking=False)
    perm = torch.from_numpy(order.astype(np.int64)).to(device)
    cols, planes = gather_layout(raw, perm, layout)
    me_t = nyse_t = None
    if me is not None:
        me_t = torch.from_numpy(np.asarray(me, dtype=np.float64)).to(device).index_select(0, perm)
    if nyse is not None:
        nyse_t = torch.from_numpy(np.asarray(nyse, dtype=np.uint8)).to(device).index_select(0, perm)
    p = DevicePanel(cols=cols, names=list(names), seg_off=torch.from_numpy(seg_off).to(device),
                    seg_off_h=seg_off, months=uniq, me=me_t, nyse=nyse_t, order=order, planes=planes)
    if cols is not None and planes is not None:
        p.planes_version = cols._version
    return p


def split_planes(panel: DevicePanel):
    """The panel's FP64 columns as two 32-bit planes (fm_split_planes), kept beside cols:
    the selects then order values by their high words (half the bytes) and the Gram reads
    both planes (the high plane the select just streamed is still in the Infinity Cache).
    A device pass over the panel, done once at ingest."""
    C, n = panel.cols.shape
    planes = torch.empty((2, C, max(n, 1)), dtype=torch.int32, device=panel.cols.device)
    _kcall("fm_split_planes", "fm_split_planes", panel.cols.data_ptr(), panel.stride, C, n, planes[0].data_ptr(),
           planes[1].data_ptr(), planes.stride(1), _stream())
    panel.planes = planes
    panel.planes_version = panel.cols._version
    return panel


@dataclass
class _Src:
    """What a panel kernel reads: FP64 columns (``f64``) and/or the panel's planes."""
    f64: Optional[torch.Tensor]
    hp: Optional[int]
    lp: Optional[int]
    pstride: int
    ncols: int
    device: object

    @property
    def ptr(self):
        return None if self.f64 is None else self.f64.data_ptr()

    @property
    def stride(self):
        return self.f64.stride(0) if self.f64 is not None else self.pstride


def _source(panel: DevicePanel, cols=None):
    """``cols`` given: those FP64 columns only.  Else the panel's own values: its FP64
    columns, its planes, or both (a planes-only panel: no FP64 pointer at all)."""
    if cols is not None:
        cols = cols.view(1, -1) if cols.dim() == 1 else cols
        return _Src(cols, None, None, 0, cols.shape[0], cols.device)
    panel.check_planes()
    hp = lp = None
    ps = 0
    if panel.planes is not None:
        hp, lp, ps = panel.planes[0].data_ptr(), panel.planes[1].data_ptr(), panel.planes.stride(1)
    return _Src(panel.cols, hp, lp, ps, panel.ncols, panel.device)


PANEL_LAYOUTS = ("f64", "planes", "both")


def panel_synthetic(nmonths, nfirms, seed, month0=0, nan_rate=0.02, nyse_rate=0.4, device=None, layout="f64"):
    """Generate a balanced synthetic panel directly in HBM (fm_gen_panel; identical to
    fmcore.synth.synth_arrays with present_rate=1).  ``layout``: "f64" the FP64 columns,
    "planes" only the split layout (fm_gen_panel_planes writes the high / low words itself:
    no FP64 columns, no layout pass), "both"."""
    from .synth import WINSOR_VARS
    if layout not in PANEL_LAYOUTS:
        raise ValueError(f"layout must be one of {PANEL_LAYOUTS}")
    device = device or require_device()
    n = nmonths * nfirms
    C = len(WINSOR_VARS)
    cols = planes = None
    if layout != "planes":
        cols = torch.empty((C, n), dtype=torch.float64, device=device)
    if layout != "f64":
        planes = torch.empty((2, C, max(n, 1)), dtype=torch.int32, device=device)
    me = torch.empty(n, dtype=torch.float64, device=device)
    nyse = torch.empty(n, dtype=torch.uint8, device=device)
    if planes is None:
        _kcall("fm_gen_panel", "fm_gen_panel", seed, month0, nmonths, nfirms, nan_rate, nyse_rate, cols.data_ptr(),
               cols.stride(0), me.data_ptr(), nyse.data_ptr(), _stream())
    else:
        _kcall("fm_gen_panel", "fm_gen_panel_planes", seed, month0, nmonths, nfirms, nan_rate, nyse_rate, _ptr(cols),
               cols.stride(0) if cols is not None else 0, planes[0].data_ptr(), planes[1].data_ptr(),
               planes.stride(1), me.data_ptr(), nyse.data_ptr(), _stream())
    seg_off = np.arange(nmonths + 1, dtype=np.int64) * nfirms
    p = DevicePanel(cols=cols, names=list(WINSOR_VARS), seg_off=torch.from_numpy(seg_off).to(device),
                    seg_off_h=seg_off, months=np.arange(month0, month0 + nmonths), me=me, nyse=nyse,
                    planes=planes)
    if cols is not None and planes is not None:
        p.planes_version = cols._version
    return p


# ------------------------------------------------------------------------------------------
# Order statistics, clipping, universes
# ------------------------------------------------------------------------------------------
@dataclass
class Cuts:
    lo: torch.Tensor      # [C, T]
    hi: torch.Tensor
    nvalid: torch.Tensor  # [C, T] int32
    mean: Optional[torch.Tensor] = None
    sd: Optional[torch.Tensor] = None
    center: Optional[torch.Tensor] = None   # Gram pivot (midpoint of the cuts)


_SELECT_WS = {}   # device -> the zeroed fm_select work buffer (the library leaves it zeroed)
_SELECT_WS_OLD = []   # outgrown buffers stay alive: captured HIP graphs may still use them


def select_ws(nseg, ncols, max_seg_len, device):
    """fm_select_args.ws: the fix-up worklist (+ zero-sign replay slots for > 6,144-row
    months), zeroed once; every fm_select call leaves it zeroed, so one buffer per device
    serves all calls on the stream (grown on demand, never freed while graphs may use it)."""
    need = int(L.load().fm_select_ws_bytes(int(nseg), int(ncols), int(max_seg_len)))
    if need < 0:
        raise ValueError("fm_select_ws_bytes: bad sizes")
    key = str(device)
    buf = _SELECT_WS.get(key)
    if buf is None or buf.numel() < need:
        if buf is not None:
            _SELECT_WS_OLD.append(buf)
        buf = torch.zeros(max(need, 1 << 16), dtype=torch.uint8, device=device)
        _SELECT_WS[key] = buf
    return buf


def select_cuts(panel: DevicePanel, q_lo, q_hi, min_count, mode=LERP_NUMPY, cols=None,
                row_mask=None, moments=False, center=False, level=None, tag="fm_select_cuts",
                universe=None):
    """Per (column, month) quantile cuts.  ``cols`` defaults to panel.cols.  ``moments``:
    also the clipped mean / sd; ``center``: also a Gram pivot inside the data; ``level``
    (uint8 [rows], one column): every row's (x >= lo) + (x >= hi) (fm_select).
    ``universe`` = (q_a, q_b): also get_subsets' NYSE breakpoints and level bytes of the
    panel's me / nyse rows in the same call (fm_select_universe: sharing the select fix-up's
    launch for months of <= 5,120 rows, riding the long-month kernel's launch for
    6,145-20,480-row months without the histogram (MID) variant, its own launch first
    otherwise); returns (Cuts, (cut_a, cut_b, level)) then."""
    if cols is not None:
        src = _source(panel, cols)
    elif row_mask is not None or moments:   # the row-masked and moments paths read FP64 columns
        src = _source(panel, panel.values())
    else:
        src = _source(panel)
    C, T = src.ncols, panel.nseg
    dev = src.device
    lo = torch.empty((C, T), dtype=torch.float64, device=dev)
    hi = torch.empty_like(lo)
    nv = torch.empty((C, T), dtype=torch.int32, device=dev)
    mean = sd = cen = None
    if moments:
        mean = torch.empty_like(lo)
        sd = torch.empty_like(lo)
    if center:
        cen = torch.empty_like(lo)
    msl = max(panel.max_seg_len, 1)
    ws = select_ws(T, C, msl, dev)
    sa = L.SelectArgs(cols=src.ptr, col_stride=src.stride if src.f64 is not None else 0, ncols=C,
                      seg_off=panel.seg_off.data_ptr(),
                      nseg=T, max_seg_len=msl, row_mask=_ptr(row_mask), q_lo=float(q_lo),
                      q_hi=float(q_hi), min_count=int(min_count), lerp_mode=int(mode), lo=lo.data_ptr(),
                      hi=hi.data_ptr(), nvalid=nv.data_ptr(), mean=_ptr(mean), sd=_ptr(sd), center=_ptr(cen),
                      level=_ptr(level), ws=ws.data_ptr(), hi_plane=src.hp, plane_stride=src.pstride,
                      lo_plane=src.lp)
    if universe is None:
        _kcall(tag, "fm_select", L.C.byref(sa), _stream())
        _remember(tag, "fm_select", sa, src, panel.planes, lo, hi, nv, mean, sd, cen, row_mask, panel.seg_off, level)
        return Cuts(lo, hi, nv, mean, sd, cen)
    ca = torch.empty(T, dtype=torch.float64, device=dev)
    cb = torch.empty_like(ca)
    ulev = torch.empty(panel.nrows, dtype=torch.uint8, device=dev)
    ua = L.UniverseArgs(me=panel.me.data_ptr(), nyse=panel.nyse.data_ptr(), q_a=float(universe[0]),
                        q_b=float(universe[1]), cut_a=ca.data_ptr(), cut_b=cb.data_ptr(), level=ulev.data_ptr())
    _kcall(tag, "fm_select_universe", L.C.byref(sa), L.C.byref(ua), _stream())
    # re-issued by time_launch with both structs (keep[1] holds the argument tuple)
    LAST_LAUNCH[tag] = ("fm_select_universe", None,
                        ((sa, ua, src, panel.planes, lo, hi, nv, mean, sd, cen, row_mask, panel.seg_off, panel.me, panel.nyse,
                          ca, cb, ulev), (L.C.byref(sa), L.C.byref(ua))))
    return Cuts(lo, hi, nv, mean, sd, cen), (ca, cb, ulev)


def clip(panel: DevicePanel, cuts: Cuts, out=None):
    v = panel.values()
    out = torch.empty_like(v) if out is None else out
    _kcall("fm_clip", "fm_clip", v.data_ptr(), out.data_ptr(), v.stride(0), panel.ncols,
           panel.seg_off.data_ptr(), panel.nseg, panel.nrows, cuts.lo.data_ptr(), cuts.hi.data_ptr(),
           _stream())
    return out


def standardize(panel: DevicePanel, mean, sd, src=None, out=None):
    src = panel.values() if src is None else src
    out = torch.empty_like(src) if out is None else out
    _kcall("fm_standardize", "fm_standardize", src.data_ptr(), out.data_ptr(), src.stride(0), src.shape[0],
           panel.seg_off.data_ptr(), panel.nseg, panel.nrows, mean.data_ptr(), sd.data_ptr(),
           _stream())
    return out


def nyse_breakpoints(panel: DevicePanel, q_a=0.2, q_b=0.5, level=None):
    """me_20 / me_50 per month over NYSE rows (pandas groupby.quantile lerp); with ``level``
    (uint8 [rows]) also every row's universe level from them, in the same call."""
    cuts = select_cuts(panel, q_a, q_b, 1, LERP_PANDAS, cols=panel.me.view(1, -1), row_mask=panel.nyse,
                       level=level, tag="fm_select_cuts[nyse]")
    return cuts.lo[0], cuts.hi[0]


def universe_level(panel: DevicePanel, cut_a, cut_b):
    level = torch.empty(panel.nrows, dtype=torch.uint8, device=panel.device)
    _kcall("fm_universe_level", "fm_universe_level", panel.me.data_ptr(), panel.seg_off.data_ptr(), panel.nseg,
           panel.nrows, cut_a.data_ptr(), cut_b.data_ptr(), level.data_ptr(), _stream())
    return level


def universe(panel: DevicePanel, q_a=0.2, q_b=0.5):
    """get_subsets on the device (reference src/calc_Lewellen_2014.py:69-105): the NYSE
    me_20 / me_50 breakpoints and the nested universe level byte of every row, one launch
    (fm_universe); months longer than its register budget take fm_select (row mask, the
    level bytes written by the same call).  Returns (cut_a [T], cut_b [T], level [rows] uint8)."""
    if panel.max_seg_len > UNIVERSE_MAX_ROWS:
        level = torch.empty(panel.nrows, dtype=torch.uint8, device=panel.device)
        a, b = nyse_breakpoints(panel, q_a, q_b, level=level)
        return a, b, level
    dev = panel.device
    a = torch.empty(panel.nseg, dtype=torch.float64, device=dev)
    b = torch.empty_like(a)
    level = torch.empty(panel.nrows, dtype=torch.uint8, device=dev)
    args = (panel.me.data_ptr(), panel.nyse.data_ptr(), panel.seg_off.data_ptr(), panel.nseg,
            max(panel.max_seg_len, 0), float(q_a), float(q_b), a.data_ptr(), b.data_ptr(), level.data_ptr())
    _kcall("fm_universe", "fm_universe", *args, _stream())
    _remember("fm_universe", "fm_universe", None, (panel.me, panel.nyse, panel.seg_off, a, b, level), args)
    return a, b, level


UNIVERSE_MAX_ROWS = 64 * 256   # fm_universe's register budget (one workgroup per month)
# fm_select's long-month kernel: months of SELECT_LONG_MIN + 1 .. SELECT_LONG_MAX rows (no row
# mask, no moments); fm_select_universe puts the universe months into its launch
SELECT_LONG_MIN, SELECT_LONG_MAX = 24 * 256, 40 * 512


def pilot_shift(panel: DevicePanel, cols=None):
    src = panel.values() if cols is None else cols
    sh = torch.empty((src.shape[0], panel.nseg), dtype=torch.float64, device=src.device)
    _kcall("fm_pilot_shift", "fm_pilot_shift", src.data_ptr(), src.stride(0), src.shape[0], panel.seg_off.data_ptr(),
           panel.nseg, sh.data_ptr(), _stream())
    return sh


# ------------------------------------------------------------------------------------------
# Models, problems, the batched Gram pass
# ------------------------------------------------------------------------------------------
@dataclass
class Model:
    name: str
    y: int                       # panel column of the dependent variable
    xs: List[int]                # panel columns of the regressors (order = output order)
    levels: Sequence[int] = (0,)  # universe levels to solve (0 all, 1 all-but-tiny, 2 large)
    const_check: bool = True     # add_constant(has_constant='skip') semantics (regressions.py)

    @property
    def mask(self):
        m = 1 << self.y
        for x in self.xs:
            m |= 1 << x
        return m


@dataclass
class Problem:
    model: int
    level: int
    K: int


@dataclass
class FMResult:
    problems: List[Problem]
    rec: torch.Tensor            # [T, nprob, pmax+2]
    status: torch.Tensor         # [T, nprob] int32 (FM_ST_* bits)
    pmax: int
    moments: Optional[torch.Tensor] = None   # [T, nprob, mom_stride]
    mom_stride: int = 0

    @property
    def nprob(self):
        return len(self.problems)


def plan_patterns(models: Sequence[Model]):
    """Validity patterns that can occur: if model a's columns are a subset of model b's,
    every row valid for b is valid for a.  Returns (lut[1<<M] uint8, pattern_models)."""
    M = len(models)
    masks = [m.mask for m in models]
    pats = []
    for P in range(1, 1 << M):
        ok = True
        for a, b in itertools.permutations(range(M), 2):
            if (masks[a] & masks[b]) == masks[a] and (P >> b) & 1 and not (P >> a) & 1:
                ok = False
                break
        if ok:
            pats.append(P)
    lut = np.full(1 << M, 255, dtype=np.uint8)
    for i, P in enumerate(pats):
        lut[P] = i
    return lut, pats


def group_models(models: Sequence[Model], nlevels, cap):
    """Split models into groups whose bucket count (patterns x levels) fits ``cap``."""
    groups, cur = [], []
    for i, m in enumerate(models):
        trial = cur + [i]
        if len(trial) > L.FM_MAX_MODELS or len(plan_patterns([models[j] for j in trial])[1]) * nlevels > cap:
            if not cur:
                raise ValueError("a single model exceeds the bucket budget")
            groups.append(cur)
            cur = [i]
        else:
            cur = trial
    if cur:
        groups.append(cur)
    return groups


def default_chunk_rows(total_rows, nseg, max_seg_len, target_chunks=512):
    """Rows per Gram workgroup: whole months when there are enough months to fill the chip
    (fm_gram keeps 3 workgroups per CU resident, 768 slots: one month per workgroup means one
    prologue and one cross-wave epilogue per month), else months split into
    ~target_chunks/nseg pieces.  Callers that shard months across ranks pass the GLOBAL sizes
    so every rank chunks (and sums) identically."""
    if nseg == 0:
        return 256
    per = max(1, -(-target_chunks // nseg))
    ch = -(-max(int(max_seg_len), 1) // per)
    return max(256, ((ch + 255) // 256) * 256)


GRAM_SLOTS_PER_CU = 3   # fm_gram workgroups resident per CU (3 waves / SIMD)
# The plan's slot count is a constant of the plan, not a query of the local device: a plan
# (and so every month's FP64 partial-sum order) must not change with the GPU a rank runs on.
GRAM_PLAN_SLOTS = 256 * GRAM_SLOTS_PER_CU   # MI355X: 256 CUs


def chunk_policy(total_rows, nseg, max_seg_len, slots=None, min_rows=2048):
    """The Gram's chunk plan for a panel of these GLOBAL sizes (sharded callers pass the
    global panel's, so every rank cuts, and sums, every month identically):

    * ("balanced", R): when the months are too few to even out over the resident workgroup
      slots (fewer than 4 rounds of them), every workgroup takes R consecutive rows of the
      global row space, cut at month boundaries into chunks (a workgroup can end one month and
      start the next), so every CU gets the same rows.  At the bench's 600 x 5,000 panel a
      grid of whole months leaves 88 CUs a third month to finish while the rest idle
      (profiles/r04/v1_size_scan.log: 600 months cost what 768 do).
    * ("months", chunk_rows): otherwise months split into ceil(L / chunk_rows) chunks
      (default_chunk_rows), one per workgroup.

    ``slots`` defaults to GRAM_PLAN_SLOTS (a constant, never the local device's CU count)."""
    slots = slots or GRAM_PLAN_SLOTS
    if nseg > 0 and nseg < 4 * slots:
        R = -(-int(total_rows) // slots)
        if R >= min_rows:
            return ("balanced", int(R))
    return ("months", default_chunk_rows(total_rows, nseg, max_seg_len))


def make_chunks_balanced(seg_off_h, rows_per_wg, row_origin=0):
    """Chunks = the row space cut at month boundaries and at global row multiples of
    rows_per_wg (row_origin = global row of local row 0); the chunks of one R-block go to one
    workgroup.  Returns (seg, rows, off, wg_off): chunk month, (r0, r1) pairs, a month's chunk
    range (fm_solve sums them in order) and each workgroup's chunk range.  A function of the
    global row space only, so a month's chunks (and sums) do not depend on the sharding."""
    so = np.asarray(seg_off_h, dtype=np.int64)
    T = len(so) - 1
    total = int(so[-1])
    R = int(rows_per_wg)
    first = (-int(row_origin)) % R
    blk = np.arange(first, total, R, dtype=np.int64)
    cuts = np.unique(np.concatenate([so, blk[blk > 0]]))
    starts, ends = cuts[:-1], cuts[1:]
    seg_of = np.searchsorted(so, starts, side="right") - 1
    # empty months keep one empty chunk (fm_solve then sums nothing for them)
    empty = np.nonzero(np.diff(so) == 0)[0]
    if len(empty):
        starts = np.concatenate([starts, so[empty]])
        ends = np.concatenate([ends, so[empty]])
        seg_of = np.concatenate([seg_of, empty])
        order = np.lexsort((seg_of, starts))   # by row, then month (an empty month before the next)
        starts, ends, seg_of = starts[order], ends[order], seg_of[order]
    seg = seg_of.astype(np.int32)
    rows = np.stack([starts, ends], axis=1).reshape(-1).astype(np.int64)
    off = np.zeros(T + 1, dtype=np.int32)
    np.cumsum(np.bincount(seg, minlength=T), out=off[1:])
    blk_of = (int(row_origin) + starts) // R
    brk = np.nonzero(np.diff(blk_of))[0] + 1
    wg_off = np.concatenate([[0], brk, [len(seg)]]).astype(np.int32)
    return seg, rows, off, wg_off


def split_policy(nseg):
    """Whether the Gram takes the split-month plan (make_chunks_split) by default.  A grid of
    whole months that is a few rounds of the chip's resident workgroup slots leaves the CUs
    unevenly loaded (600 months cost as much as 768: profiles/r04/v1_size_scan.log), but the
    3/4 + 1/4 split with the big chunks launched first measured -2 us on the Gram and +2 us on
    the solve at the bench's 600 months (profiles/r04/v3_split_scan.log: -10 us at 512
    months, +5 us at 768), so it is off; callers opt in with panel.chunk_split = True.
    Callers that shard months pass the GLOBAL month count, like default_chunk_rows, so every
    rank plans (and sums) identically."""
    return False


def make_chunks_split(seg_off_h, num=3, den=4, min_rows=256):
    """Every month of >= min_rows rows as two chunks, rows [0, L*num/den) and the rest (a
    function of the month's own length only, so sharding does not change its sums), else one.
    Returns (seg, rows, off, order): the chunk arrays in month order (fm_solve sums a month's
    chunks from seg_chunk_off) and the launch order for fm_gram's chunk_order -- every big
    chunk first (last month first), then the small ones, which fill the slots the big ones
    leave (longest-first scheduling evens the per-CU load)."""
    T = len(seg_off_h) - 1
    lens = np.diff(seg_off_h).astype(np.int64)
    two = lens >= min_rows
    nch = np.where(two, 2, 1).astype(np.int64)
    off = np.zeros(T + 1, dtype=np.int32)
    np.cumsum(nch, out=off[1:])
    n = int(off[-1])
    seg = np.repeat(np.arange(T, dtype=np.int32), nch)
    rows = np.empty((n, 2), dtype=np.int64)
    first = off[:-1].astype(np.int64)
    cut = seg_off_h[:-1] + (lens * num) // den
    rows[first, 0] = seg_off_h[:-1]
    rows[first, 1] = np.where(two, cut, seg_off_h[1:])
    sec = first[two] + 1
    rows[sec, 0] = cut[two]
    rows[sec, 1] = seg_off_h[1:][two]
    order = np.concatenate([first[::-1], sec[::-1]]).astype(np.int32)
    return seg, rows.reshape(-1), off, order


def make_chunks(seg_off_h, chunk_rows):
    """Split every month into ceil(L / chunk_rows) near-equal chunks (depends only on the
    month's own length, so per-month arithmetic is independent of sharding)."""
    T = len(seg_off_h) - 1
    lens = np.diff(seg_off_h).astype(np.int64)
    nch = np.maximum(1, -(-lens // chunk_rows)).astype(np.int64)
    seg = np.repeat(np.arange(T, dtype=np.int32), nch)
    k = np.arange(len(seg)) - np.repeat(np.cumsum(nch) - nch, nch)
    L = lens[seg]
    n = nch[seg]
    r0 = seg_off_h[seg] + (k * L) // n
    r1 = seg_off_h[seg] + ((k + 1) * L) // n
    rows = np.stack([r0, r1], axis=1).reshape(-1).astype(np.int64)
    off = np.zeros(T + 1, dtype=np.int32)
    np.cumsum(nch, out=off[1:])
    return seg, rows, off


@dataclass
class _Plan:
    chunk_seg: torch.Tensor
    chunk_row: torch.Tensor
    seg_chunk_off: torch.Tensor
    nchunks: int
    order: Optional[torch.Tensor] = None   # fm_gram launch order (split plan) or None
    wg_off: Optional[torch.Tensor] = None  # balanced plan: each workgroup's chunk range
    nwg: int = 0


def _chunk_plan(panel: DevicePanel):
    cache = getattr(panel, "_chunk_cache", None)
    if cache is not None:
        return cache
    pol = panel.chunk_policy
    if pol is None and panel.chunk_rows is not None:   # a sharded caller's global months policy
        pol = ("months", panel.chunk_rows)
    split = panel.chunk_split
    if split is None:
        split = pol is None and split_policy(panel.nseg)
    if pol is None and not split:
        pol = chunk_policy(panel.nrows, panel.nseg, panel.max_seg_len)
    order = wg = None
    if split:
        seg, rows, off, order = make_chunks_split(panel.seg_off_h)
    elif pol[0] == "balanced":
        seg, rows, off, wg = make_chunks_balanced(panel.seg_off_h, pol[1], panel.row_origin)
    else:
        seg, rows, off = make_chunks(panel.seg_off_h, pol[1])
    dev = panel.device
    t = lambda a: None if a is None else torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    plan = _Plan(t(seg), t(rows), t(off), len(seg), t(order), t(wg), 0 if wg is None else len(wg) - 1)
    panel._chunk_cache = plan
    return plan


@dataclass
class _GroupPlan:
    """Device-resident description of one model group (built once per model set)."""
    nmodels: int
    npatterns: int
    nprob: int
    mm: torch.Tensor     # [nmodels] column masks
    ym: torch.Tensor     # [nmodels] y-column bit
    lut: torch.Tensor    # [1<<nmodels] validity pattern -> pattern index
    patm: torch.Tensor   # [npatterns] model set of each pattern
    pm: torch.Tensor     # [nprob] group-local model of each problem
    pl: torch.Tensor     # [nprob] universe level
    pf: torch.Tensor     # [nprob] const-check flag
    pz: torch.Tensor     # [nprob, 32] z columns (0 = intercept, 1+c = panel column c)
    pnz: torch.Tensor    # [nprob]
    idx: torch.Tensor    # [nprob] global problem index


def _group_plans(panel, models, problems, nlevels, cap, const_check, dev):
    key = (tuple((m.y, tuple(m.xs), tuple(m.levels), bool(m.const_check)) for m in models),
           nlevels, cap, bool(const_check), str(dev))
    cache = panel.__dict__.setdefault("_group_cache", {})
    if key in cache:
        return cache[key]
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    plans = []
    for g in group_models(models, nlevels, cap):
        gm = [models[i] for i in g]
        lut, pats = plan_patterns(gm)
        gp = [(k, p) for k, p in enumerate(problems) if p.model in g]
        local = {mi: j for j, mi in enumerate(g)}
        pz = np.zeros((len(gp), 32), dtype=np.int32)
        pnz = np.zeros(len(gp), dtype=np.int32)
        for j, (_, p) in enumerate(gp):
            m = models[p.model]
            z = [0] + [1 + x for x in m.xs] + [1 + m.y]
            pz[j, :len(z)] = z
            pnz[j] = len(z)
        plans.append(_GroupPlan(
            nmodels=len(gm), npatterns=len(pats), nprob=len(gp),
            mm=t(np.array([m.mask for m in gm], dtype=np.int64).astype(np.int32)),
            ym=t(np.array([1 << m.y for m in gm], dtype=np.int32)),
            lut=t(lut),
            patm=t(np.array(pats, dtype=np.int64).astype(np.uint32).view(np.int32)),
            pm=t(np.array([local[p.model] for _, p in gp], dtype=np.int32)),
            pl=t(np.array([p.level for _, p in gp], dtype=np.int32)),
            pf=t(np.array([1 if (models[p.model].const_check and const_check) else 0 for _, p in gp],
                          dtype=np.int32)),
            pz=t(pz), pnz=t(pnz),
            idx=t(np.array([k for k, _ in gp], dtype=np.int64))))
    cache[key] = plans
    return plans


def _solve_group(panel, src, gpl, partial, seg_chunk_off, zw, nlevels, T, pmax, mom_stride, lo, hi,
                 shift, inv_scale, add_back, level, const_check, keep):
    """fm_solve + the statsmodels fix-ups (inf in y, nonzero constant columns) for one
    model group; returns (rec, status, moments) [T, ng, ...]."""
    dev = src.device
    ng = gpl.nprob
    rs = pmax + 2
    grec = torch.empty((T, ng, rs), dtype=torch.float64, device=dev)
    gst = torch.empty((T, ng), dtype=torch.int32, device=dev)   # the solve writes every entry
    # centered moments are always produced: the inf-in-y fix reads them
    gmom = torch.empty((T, ng, mom_stride), dtype=torch.float64, device=dev)
    sa = L.SolveArgs(
        partial=partial.data_ptr(), seg_chunk_off=seg_chunk_off.data_ptr(), nseg=T, zw=zw,
        nlevels=nlevels, npatterns=gpl.npatterns, pattern_models=gpl.patm.data_ptr(), nprob=ng,
        prob_model=gpl.pm.data_ptr(), prob_level=gpl.pl.data_ptr(), prob_z=gpl.pz.data_ptr(),
        prob_nz=gpl.pnz.data_ptr(), prob_flags=gpl.pf.data_ptr(), add_back=_ptr(add_back),
        gram_flags=None, nmodels=gpl.nmodels, pmax=pmax, rec=grec.data_ptr(),
        status=gst.data_ptr(), moments=_ptr(gmom), mom_stride=mom_stride, ab_ncols=src.ncols)
    # statsmodels fix-ups: the exact nonzero-constant test where the solve saw a near-zero
    # variance (CONST_SUSPECT), inf in y (pinv(X) @ y gives +-inf / NaN coefficients) and the
    # QR + SVD refit of ill-conditioned / rank-deficient problems (FM_ST_REFIT).  The 16-wide
    # solve does them inside its own launch (each month's workgroup, right after its solve);
    # the 32-wide one is followed by fm_solve_fixup, which scans the status on the device
    # (npairs = -1): no host round trip either way.
    inline_fix = zw == 16 and pmax + 1 <= 16
    if not inline_fix and src.f64 is None:   # fm_solve_fixup reads FP64 columns
        src = _source(panel, panel.values())
    if inline_fix:
        # the fix-ups' rows: the FP64 columns, else the planes of a planes-only panel
        sa.fix_cols, sa.fix_stride, sa.fix_seg_off = src.ptr, src.stride, panel.seg_off.data_ptr()
        if src.f64 is None:
            sa.fix_hi_plane, sa.fix_lo_plane = src.hp, src.lp
        sa.fix_lo, sa.fix_hi, sa.fix_shift, sa.fix_inv_scale = _ptr(lo), _ptr(hi), _ptr(shift), _ptr(inv_scale)
        sa.fix_level, sa.fix_check_const = _ptr(level), int(bool(const_check))
    _kcall("fm_solve", "fm_solve", L.C.byref(sa), _stream())
    _remember("fm_solve", "fm_solve", sa, partial, seg_chunk_off, gpl, add_back, grec, gst, gmom, src.f64,
              panel.planes, lo, hi, shift, inv_scale, level, *keep)
    if inline_fix:
        return grec, gst, gmom
    _kcall("fm_solve_fixup", "fm_solve_fixup", src.ptr, src.stride, panel.seg_off.data_ptr(), T,
           _ptr(lo), _ptr(hi), _ptr(shift), _ptr(inv_scale), _ptr(add_back), _ptr(level), ng,
           gpl.pl.data_ptr(), gpl.pz.data_ptr(), gpl.pnz.data_ptr(), None, -1,
           gmom.data_ptr(), mom_stride, pmax, grec.data_ptr(), gst.data_ptr(), int(bool(const_check)),
           _stream())
    return grec, gst, gmom


def _problems(models, nlevels):
    problems = []
    for mi, m in enumerate(models):
        for u in m.levels:
            if u >= nlevels:
                raise ValueError("model level beyond the universe levels provided")
            problems.append(Problem(mi, u, len(m.xs)))
    return problems


def fm_pass(panel: DevicePanel, models: Sequence[Model], level=None, nlevels=1, cuts: Cuts = None,
            shift=None, inv_scale=None, add_back=None, moments=False, cols=None, const_check=True):
    """One batched cross-sectional pass: every (model, universe level) problem for every
    month from one read of the panel per model group.  Returns an FMResult."""
    src = _source(panel, cols)
    ncols = src.ncols
    if ncols > L.FM_MAX_COLS:
        raise ValueError(f"at most {L.FM_MAX_COLS} columns per pass")
    dev = src.device
    T = panel.nseg
    zw = 16 if ncols <= 15 else 32
    cap = 16 if zw == 16 else 8
    if shift is None:
        shift = pilot_shift(panel, cols)
    if add_back is None and inv_scale is None:
        add_back = shift
    problems = _problems(models, nlevels)
    pmax = max(2, max(p.K + 1 for p in problems))
    nprob = len(problems)
    rs = pmax + 2
    rec = torch.empty((T, nprob, rs), dtype=torch.float64, device=dev)
    status = torch.empty((T, nprob), dtype=torch.int32, device=dev)   # every problem is in one group
    mom_stride = 1 + (pmax + 1) + (pmax + 1) ** 2
    mom = torch.empty((T, nprob, mom_stride), dtype=torch.float64, device=dev) if moments else None
    plan = _chunk_plan(panel)
    lo = cuts.lo if cuts is not None else None
    hi = cuts.hi if cuts is not None else None
    groups = _group_plans(panel, models, problems, nlevels, cap, const_check, dev)
    for gpl in groups:
        nb = gpl.npatterns * nlevels
        partial = torch.empty((plan.nchunks, nb, zw * (zw + 1) // 2), dtype=torch.float64, device=dev)
        flags = torch.empty((T, gpl.nmodels), dtype=torch.int32, device=dev)   # reserved: never read
        ga = L.GramArgs(
            cols=src.ptr, col_stride=src.stride if src.f64 is not None else 0, ncols=ncols, nseg=T,
            seg_off=panel.seg_off.data_ptr(), chunk_seg=plan.chunk_seg.data_ptr(),
            chunk_row=plan.chunk_row.data_ptr(), nchunks=plan.nchunks,
            lo=_ptr(lo), hi=_ptr(hi), shift=_ptr(shift), inv_scale=_ptr(inv_scale),
            level=_ptr(level), nlevels=nlevels, model_mask=gpl.mm.data_ptr(),
            model_ymask=gpl.ym.data_ptr(), nmodels=gpl.nmodels, pattern_id=gpl.lut.data_ptr(),
            npatterns=gpl.npatterns, partial=partial.data_ptr(), flags=flags.data_ptr(),
            chunk_order=_ptr(plan.order), hi_plane=src.hp, lo_plane=src.lp, plane_stride=src.pstride,
            wg_chunk_off=_ptr(plan.wg_off), nwg=plan.nwg)
        _kcall("fm_gram", "fm_gram", L.C.byref(ga), _stream())
        _remember("fm_gram", "fm_gram", ga, src.f64, panel.planes, partial, flags, lo, hi, shift, inv_scale, level,
                  plan, gpl)
        grec, gst, gmom = _solve_group(panel, src, gpl, partial, plan.seg_chunk_off, zw, nlevels, T, pmax,
                                       mom_stride, lo, hi, shift, inv_scale, add_back, level,
                                       const_check, (src.f64, panel.planes, flags, lo, hi, shift, inv_scale,
                                                     level, plan))
        if len(groups) == 1:
            rec, status = grec, gst
            mom = gmom if moments else None
        else:
            rec.index_copy_(1, gpl.idx, grec)
            status.index_copy_(1, gpl.idx, gst)
            if moments:
                mom.index_copy_(1, gpl.idx, gmom)
    return FMResult(problems=problems, rec=rec, status=status, pmax=pmax, moments=mom,
                    mom_stride=mom_stride)


def drop_degenerate_months(res: FMResult, models: Sequence[Model], sd):
    """Standardized passes (A9): a month in which a regressor has fewer than two values or
    zero dispersion has an all-NaN z-score column, so every row drops out and the month is
    not fitted for the models using it; clear FM_ST_FITTED there.  ``sd`` [C, T]."""
    bad = ~(sd > 0)                                              # NaN sd -> True
    C = sd.shape[0]
    use = np.zeros((res.nprob, C), dtype=np.float64)
    for k, p in enumerate(res.problems):
        use[k, models[p.model].xs] = 1.0
    hit = _small_tensor(tuple(map(tuple, use)), torch.float64, sd.device) @ bad.to(torch.float64)
    res.status &= ~((hit.t() > 0).to(torch.int32) * L.FM_ST_FITTED)
    return res


# ------------------------------------------------------------------------------------------
# Time-series stage
# ------------------------------------------------------------------------------------------
@dataclass
class TSIndex:
    idx: torch.Tensor     # [nprob, T] int32: fitted months in order
    count: torch.Tensor   # [nprob] int32


def ts_compact(status, s_seg, s_prob, nseg, nprob):
    dev = status.device
    idx = torch.empty((nprob, nseg), dtype=torch.int32, device=dev)
    cnt = torch.empty(nprob, dtype=torch.int32, device=dev)
    _kcall("fm_ts_compact", "fm_ts_compact", status.data_ptr(), s_seg, s_prob, nseg, nprob, idx.data_ptr(),
           cnt.data_ptr(), _stream())
    return TSIndex(idx, cnt)


def compact_result(res: FMResult):
    T, P = res.status.shape
    return ts_compact(res.status, P, 1, T, P)


@dataclass
class Summary:
    mean: torch.Tensor   # [nprob, kmax]
    se: torch.Tensor
    tstat: torch.Tensor
    nobs: torch.Tensor


def _sum_outputs(nprob, kmax, dev, sum_range):
    """Summary output buffers; with a problem range (sharded runs) pre-filled with the -0.0 /
    0 that the SUM-combine across ranks needs for the problems this rank does not summarize."""
    if sum_range is None:
        mean = torch.empty((nprob, kmax), dtype=torch.float64, device=dev)
        se, ts = torch.empty_like(mean), torch.empty_like(mean)
        nobs = torch.empty((nprob, kmax), dtype=torch.int32, device=dev)
    else:
        mean = torch.full((nprob, kmax), -0.0, dtype=torch.float64, device=dev)
        se, ts = mean.clone(), mean.clone()
        nobs = torch.zeros((nprob, kmax), dtype=torch.int32, device=dev)
    return mean, se, ts, nobs


def ts_summary(rec, r_seg, r_prob, ix: TSIndex, nseg, nprob, kmax, nw_lags=4, sum_range=None):
    """FM means / NW standard errors of every (problem, coefficient).  ``sum_range`` = (p0, p1):
    problems [p0, p1) only (pointer offsets into the same buffers), -0.0 / 0 elsewhere."""
    dev = rec.device
    mean, se, ts, nobs = _sum_outputs(nprob, kmax, dev, sum_range)
    p0, p1 = (0, nprob) if sum_range is None else sum_range
    n = p1 - p0
    if n <= 0:
        return Summary(mean, se, ts, nobs)
    # the series [n][kmax][nseg] and the long-series chunk partials (fm_hip.h)
    work = torch.empty(n * kmax * (max(nseg, 1) + -(-nseg // 2048) * 28), dtype=torch.float64, device=dev)
    _kcall("fm_ts_summary", "fm_ts_summary", rec.data_ptr() + 8 * p0 * r_prob, r_seg, r_prob,
           ix.idx[p0].data_ptr(), ix.count[p0:].data_ptr(), nseg, n, kmax, nw_lags, mean[p0].data_ptr(),
           se[p0].data_ptr(), ts[p0].data_ptr(), nobs[p0].data_ptr(), work.data_ptr(), _stream())
    return Summary(mean, se, ts, nobs)


def summarize_result(res: FMResult, ix: TSIndex = None, nw_lags=4, sum_range=None):
    ix = ix or compact_result(res)
    T, P, rs = res.rec.shape
    return ts_summary(res.rec, P * rs, rs, ix, T, P, rs, nw_lags, sum_range), ix


def rolling_result(res: FMResult, ix: TSIndex, window=120, min_periods=60, own=None):
    """Rolling means [P, T, pmax] of the fitted-month series.  ``own`` = (seg_lo, seg_hi, lag)
    (sharded runs): only the rows a predictive stage of those months reads, the same bits
    (fm_rolling_mean_own); other rows are left unwritten."""
    T, P, rs = res.rec.shape
    out = torch.empty((P, T, res.pmax), dtype=torch.float64, device=res.rec.device)
    if own is None:
        _kcall("fm_rolling_mean", "fm_rolling_mean", res.rec.data_ptr(), P * rs, rs, ix.idx.data_ptr(),
               ix.count.data_ptr(), T, P, res.pmax, window, min_periods, out.data_ptr(), _stream())
    else:
        _kcall("fm_rolling_mean", "fm_rolling_mean_own", res.rec.data_ptr(), P * rs, rs, ix.idx.data_ptr(),
               ix.count.data_ptr(), T, P, res.pmax, window, min_periods, int(own[0]), int(own[1]), int(own[2]),
               out.data_ptr(), _stream())
    return out


_SMALL = {}


def _small_tensor(values, dtype, dev):
    """Cached device copy of a small constant list (no per-call host-to-device copy)."""
    key = (values, dtype, str(dev))
    t = _SMALL.get(key)
    if t is None:
        t = _SMALL[key] = torch.tensor(list(values), dtype=dtype, device=dev)
    return t


def predictive_result(res: FMResult, ix: TSIndex, roll, lag=1, seg_lo=0, seg_hi=None, moments=None):
    """A7/A8 per (problem, fitted-month row): slope, R2, N of y on the lagged-rolling
    forecast, from the month's centered moments.  In sharded runs ``res`` holds the
    gathered global records and ``moments`` the local months [seg_lo, seg_hi) only."""
    T, P, _ = res.rec.shape
    dev = res.rec.device
    mom = res.moments if moments is None else moments
    seg_hi = T if seg_hi is None else seg_hi
    pk = _small_tensor(tuple(p.K for p in res.problems), torch.int32, dev)
    pred = torch.empty((P, T, 4), dtype=torch.float64, device=dev)
    pst = torch.empty((P, T), dtype=torch.int32, device=dev)
    _kcall("fm_predictive", "fm_predictive", mom.data_ptr(), res.mom_stride, T, P, pk.data_ptr(),
           ix.idx.data_ptr(), ix.count.data_ptr(), roll.data_ptr(), res.pmax, lag, seg_lo, seg_hi,
           pred.data_ptr(), pst.data_ptr(), _stream())
    return pred, pst


def summarize_predictive(pred, pst, nw_lags=4, sum_range=None):
    """FM summary of the predictive records (slope, R^2, n).  ``sum_range`` (sharded runs):
    problems [p0, p1) only, -0.0 / 0 elsewhere (combined across ranks by a SUM)."""
    P, T, _ = pred.shape
    if not ts_fused_fits(T):
        p0, p1 = (0, P) if sum_range is None else sum_range
        ix = TSIndex(torch.empty((P, T), dtype=torch.int32, device=pred.device),
                     torch.zeros(P, dtype=torch.int32, device=pred.device))
        if p1 > p0:
            _kcall("fm_ts_compact", "fm_ts_compact", pst[p0].data_ptr(), 1, T, T, p1 - p0, ix.idx[p0].data_ptr(),
                   ix.count[p0:].data_ptr(), _stream())
        return ts_summary(pred, 4, T * 4, ix, T, P, 3, nw_lags, sum_range), ix
    ix, summ, _, _, _ = ts_fused(pred, 4, T * 4, pst, 1, T, T, P, 3, nw_lags, tag="fm_ts_fused[pred]",
                                 sum_range=sum_range)
    return summ, ix


def ts_fused_fits(nseg, pmax=0, window=None, lag=1, predictive=False):
    """Whether fm_ts_fused can stage this series in LDS (else the per-stage kernels run)."""
    need = L.load().fm_ts_fused_lds_bytes(nseg, pmax, window or 0, lag, int(window is not None),
                                           int(bool(predictive)))
    return need <= L.FM_TS_FUSED_MAX_LDS


def ts_fused(rec, r_seg, r_prob, status, s_seg, s_prob, nseg, nprob, kmax, nw_lags=4,
             window=None, min_periods=None, pmax=None, moments=None, mom_stride=0, prob_k=None,
             lag=1, seg_lo=0, seg_hi=None, predictive=False, tag="fm_ts_fused", sum_range=None,
             roll_own=False):
    """The whole time-series stage in one launch (fm_ts_fused): TSIndex, Summary and, when
    ``window`` is given, the rolling means [P, T, pmax]; with ``predictive`` also the
    predictive records [P, T, 4] and status [P, T].  Returns (ix, summ, roll, pred, pst).
    Sharded runs: ``sum_range`` = (p0, p1) summarizes problems [p0, p1) only (-0.0 / 0
    elsewhere), ``roll_own`` rolls only the rows the months [seg_lo, seg_hi) read."""
    dev = rec.device
    idx = torch.empty((nprob, nseg), dtype=torch.int32, device=dev)
    cnt = torch.empty(nprob, dtype=torch.int32, device=dev)
    mean = torch.empty((nprob, kmax), dtype=torch.float64, device=dev)
    se, ts = torch.empty_like(mean), torch.empty_like(mean)
    nobs = torch.empty((nprob, kmax), dtype=torch.int32, device=dev)
    roll = pred = pst = None
    if window is not None:
        roll = torch.empty((nprob, nseg, pmax), dtype=torch.float64, device=dev)
    if predictive:
        pred = torch.empty((nprob, nseg, 4), dtype=torch.float64, device=dev)
        pst = torch.empty((nprob, nseg), dtype=torch.int32, device=dev)
    # problem range of the summaries: (0, 0) = every problem; an empty range of a sharded rank
    # (more ranks than problems) = (nprob, nprob): the kernel then summarizes none
    sp_lo, sp_hi = 0, 0
    if sum_range is not None:
        sp_lo, sp_hi = int(sum_range[0]), int(sum_range[1])
        if sp_hi <= sp_lo:
            sp_lo = sp_hi = nprob
    ta = L.TsArgs(rec=rec.data_ptr(), r_seg=r_seg, r_prob=r_prob, status=status.data_ptr(), s_seg=s_seg,
                  s_prob=s_prob, nseg=nseg, nprob=nprob, kmax=kmax, nw_lags=nw_lags, idx=idx.data_ptr(),
                  count=cnt.data_ptr(), mean=mean.data_ptr(), se=se.data_ptr(), tstat=ts.data_ptr(),
                  nobs=nobs.data_ptr(), work=None, window=window or 0,
                  min_periods=min_periods or 0, pmax=pmax or 0, roll=_ptr(roll), moments=_ptr(moments),
                  mom_stride=mom_stride, prob_k=_ptr(prob_k), lag=lag, seg_lo=seg_lo,
                  seg_hi=nseg if seg_hi is None else seg_hi, pred=_ptr(pred), pred_status=_ptr(pst),
                  sum_p_lo=sp_lo, sum_p_hi=sp_hi, roll_own=int(bool(roll_own)))
    _kcall(tag, "fm_ts_fused", L.C.byref(ta), _stream())
    _remember(tag, "fm_ts_fused", ta, rec, status, idx, cnt, mean, se, ts, nobs, roll,
              moments, prob_k, pred, pst)
    return TSIndex(idx, cnt), Summary(mean, se, ts, nobs), roll, pred, pst


def time_series_result(res: FMResult, nw_lags=4, window=120, min_periods=60, lag=1, seg_lo=0,
                       seg_hi=None, moments=None, rolling=True, predictive=True, sum_range=None,
                       roll_own=False):
    """compact_result + summarize_result + rolling_result + predictive_result in one launch.
    Returns (ix, summ, roll, pred, pst).  Sharded runs (every rank on the gathered series):
    ``sum_range`` = this rank's problems for the FM summaries, ``roll_own`` = rolling means only
    where this rank's predictive records [seg_lo, seg_hi) read them."""
    T, P, rs = res.rec.shape
    mom = res.moments if moments is None else moments
    window = window if (rolling or predictive) else None
    if not ts_fused_fits(T, res.pmax, window, lag, predictive):
        ix = compact_result(res)
        summ, _ = summarize_result(res, ix, nw_lags, sum_range)
        roll = pred = pst = None
        if window is not None:
            own = None
            if roll_own:
                own = (seg_lo, T if seg_hi is None else seg_hi, lag if predictive else 0)
            roll = rolling_result(res, ix, window, min_periods, own)
        if predictive:
            pred, pst = predictive_result(res, ix, roll, lag, seg_lo, seg_hi, moments)
        return ix, summ, roll, pred, pst
    pk = _small_tensor(tuple(p.K for p in res.problems), torch.int32, res.rec.device) if predictive else None
    return ts_fused(res.rec, P * rs, rs, res.status, P, 1, T, P, rs, nw_lags,
                    window=window, min_periods=min_periods,
                    pmax=res.pmax, moments=mom if predictive else None, mom_stride=res.mom_stride,
                    prob_k=pk, lag=lag, seg_lo=seg_lo, seg_hi=seg_hi, predictive=predictive,
                    sum_range=sum_range, roll_own=roll_own)


def forecast(panel: DevicePanel, coef, cols=None):
    """A7 per-row forecasts F = c0[t] + sum_k c_k[t] x_k for coef [T, K+1] (NaN propagates)."""
    src = panel.values() if cols is None else cols
    coef = coef.contiguous()
    out = torch.empty(panel.nrows, dtype=torch.float64, device=src.device)
    _kcall("fm_forecast", "fm_forecast", src.data_ptr(), src.stride(0), src.shape[0], panel.seg_off.data_ptr(),
           panel.nseg, panel.nrows, coef.data_ptr(), coef.stride(0), out.data_ptr(), _stream())
    return out


def segment_moments(panel: DevicePanel, level=None, min_level=0, finite_only=True, cols=None):
    """Per (column, month) count, mean and ddof=1 std of the non-missing values."""
    src = panel.values() if cols is None else cols
    C, T = src.shape[0], panel.nseg
    cnt = torch.empty((C, T), dtype=torch.int32, device=src.device)
    mean = torch.empty((C, T), dtype=torch.float64, device=src.device)
    sd = torch.empty_like(mean)
    _kcall("fm_segment_moments", "fm_segment_moments", src.data_ptr(), src.stride(0), C,
           panel.seg_off.data_ptr(), T, _ptr(level), int(min_level), int(bool(finite_only)),
           cnt.data_ptr(), mean.data_ptr(), sd.data_ptr(), _stream())
    return cnt, mean, sd


def distinct_count(ids, cols, level=None, min_level=0, finite_only=True):
    """Number of distinct ids among rows where each column is present -> int32 [C]."""
    C, n = cols.shape
    dev = cols.device
    out = torch.empty(C, dtype=torch.int32, device=dev)
    if n == 0:
        out.zero_()
        return out
    lo = int(ids.min().item())
    rng = int(ids.max().item()) - lo + 1
    bitmap = torch.empty((C, (rng + 31) // 32), dtype=torch.int32, device=dev)
    _kcall("fm_distinct_count", "fm_distinct_count", ids.data_ptr(), n, cols.data_ptr(), cols.stride(0), C,
           _ptr(level), int(min_level), int(bool(finite_only)), lo, rng, bitmap.data_ptr(), out.data_ptr(),
           _stream())
    return out


# ------------------------------------------------------------------------------------------
# Firm-axis characteristics (src/calc_Lewellen_2014.py:137-466)
# ------------------------------------------------------------------------------------------
CHAR_FIELDS = ("me", "be", "retx", "accruals", "depreciation", "earnings", "assets", "dvc", "prc",
               "shrout", "total_debt", "sales")
CHAR_NAMES = ("log_size", "log_bm", "return_12_2", "accruals_final", "roa", "log_assets_growth",
              "dy", "log_return_13_36", "log_issues_12", "log_issues_36", "debt_price", "sales_price")


def _check_ids(ids):
    """Firm ids are read as raw int64 words: reject any other dtype / layout."""
    if ids.dtype != torch.int64 or ids.dim() != 1 or not ids.is_contiguous():
        raise ValueError("firm ids must be a contiguous int64 [n] tensor")


def firm_chars(ids, fields, names=CHAR_NAMES, out=None):
    """Monthly characteristics for FIRM-major rows (each firm's rows contiguous, in frame
    order).  ``ids`` int64 [n]; ``fields`` maps CHAR_FIELDS names -> float64 [n] device
    tensors (only those the requested characteristics read); returns {name: float64 [n]}.
    ``out`` (optional) is a [len(names), n] float64 tensor to write into."""
    n = int(ids.shape[0])
    dev = ids.device
    _check_ids(ids)
    if out is None:
        out = torch.empty((len(names), n), dtype=torch.float64, device=dev)
    if out.dtype != torch.float64 or out.dim() != 2 or out.shape != (len(names), n) or out.stride(1) != 1:
        raise ValueError("firm_chars: out must be float64 [len(names), n] with contiguous rows")
    a = L.CharsArgs()
    a.ids = ids.data_ptr()
    a.n = n
    keep = [ids, out]
    for f, nm in enumerate(CHAR_FIELDS):
        t = fields.get(nm)
        if t is not None:
            if t.dtype != torch.float64 or t.dim() != 1 or t.shape[0] != n or t.device != dev:
                raise ValueError(f"firm_chars: field {nm!r} must be a float64 [{n}] tensor on {dev}")
            t = t.contiguous()
            keep.append(t)
            a.field[f] = t.data_ptr()
    for j, nm in enumerate(names):
        a.out[CHAR_NAMES.index(nm)] = out[j].data_ptr()
    _remember("fm_firm_chars", "fm_firm_chars", a, *keep)
    _kcall("fm_firm_chars", "fm_firm_chars", L.C.byref(a), _stream())
    return {nm: out[j] for j, nm in enumerate(names)}


def rolling_std(ids, x, window=252, min_periods=100, scale=252 ** 0.5, out=None):
    """Per-row rolling std (ddof=1) over the last ``window`` rows of each firm group."""
    n = int(x.shape[0])
    _check_ids(ids)
    if x.dtype != torch.float64 or x.dim() != 1 or ids.shape[0] != n or x.device != ids.device:
        raise ValueError("rolling_std: x must be a float64 [n] tensor beside int64 [n] ids")
    x = x.contiguous()
    # fm_rolling_std moves row pairs with 16-byte accesses: views at odd offsets are copied
    if x.data_ptr() % 16:
        x = x.clone()
    if ids.data_ptr() % 16 or not ids.is_contiguous():
        ids = ids.clone()
    if out is None:
        out = torch.empty(n, dtype=torch.float64, device=x.device)
    if out.dtype != torch.float64 or out.shape != (n,) or not out.is_contiguous() or out.data_ptr() % 16:
        raise ValueError("rolling_std: out must be a contiguous, 16-byte aligned float64 [n] tensor")
    args = (ids.data_ptr(), x.data_ptr(), n, int(window), int(min_periods), float(scale), out.data_ptr())
    _kcall("fm_rolling_std", "fm_rolling_std", *args, _stream())
    LAST_LAUNCH["fm_rolling_std"] = ("fm_rolling_std", None, ((ids, x, out), args))
    return out


def rolling_beta(day, ri, rm, seg_off, q_seg, q_day0, q_day1, period_weeks=156):
    """fm_rolling_beta on device tensors: day int32 [n], ri / rm float64 [n] (firm-major,
    days ascending per firm), seg_off int64 [nseg+1]; queries int32 [nq]; -> float64 [nq]."""
    n = int(day.shape[0])
    for t, dt in ((day, torch.int32), (ri, torch.float64), (rm, torch.float64), (seg_off, torch.int64),
                  (q_seg, torch.int32), (q_day0, torch.int32), (q_day1, torch.int32)):
        if t.dtype != dt or t.dim() != 1 or not t.is_contiguous():
            raise ValueError(f"rolling_beta: expected contiguous {dt} vectors")
    if ri.shape[0] != n or rm.shape[0] != n:
        raise ValueError("rolling_beta: day / ri / rm lengths differ")
    nq = int(q_seg.shape[0])
    out = torch.empty(nq, dtype=torch.float64, device=day.device)
    ws = torch.empty((5, max(n, 1)), dtype=torch.float64, device=day.device)
    _kcall("fm_rolling_beta", "fm_rolling_beta", day.data_ptr(), ri.data_ptr(), rm.data_ptr(), n,
           seg_off.data_ptr(), int(seg_off.shape[0]) - 1, int(period_weeks) * 7, q_seg.data_ptr(),
           q_day0.data_ptr(), q_day1.data_ptr(), nq, ws.data_ptr(), out.data_ptr(), _stream())
    return out


def stream_probe(t):
    """fm_stream_probe: the sum of a contiguous, 16-byte aligned float64 tensor read as a
    plain HBM stream (bench.py's measured read rate; re-issued by time_launch)."""
    if t.dtype != torch.float64 or not t.is_contiguous() or t.data_ptr() % 16:
        raise ValueError("stream_probe: a contiguous, 16-byte aligned float64 tensor")
    out = torch.zeros(1, dtype=torch.float64, device=t.device)
    args = (t.data_ptr(), t.numel(), out.data_ptr())
    _kcall("fm_stream_probe", "fm_stream_probe", *args, _stream())
    LAST_LAUNCH["fm_stream_probe"] = ("fm_stream_probe", None, ((t, out), args))
    return out


def stream_copy_probe(src, dst):
    """fm_stream_copy_probe: dst <- src (contiguous, 16-byte aligned float64 tensors of one
    size) as the probe's 16-byte stream (bench.py's measured copy rate; re-issued by
    time_launch)."""
    for t in (src, dst):
        if t.dtype != torch.float64 or not t.is_contiguous() or t.data_ptr() % 16:
            raise ValueError("stream_copy_probe: contiguous, 16-byte aligned float64 tensors")
    if src.numel() != dst.numel() or src.device != dst.device:
        raise ValueError("stream_copy_probe: src and dst must match in size and device")
    args = (src.data_ptr(), dst.data_ptr(), src.numel())
    _kcall("fm_stream_copy_probe", "fm_stream_copy_probe", *args, _stream())
    LAST_LAUNCH["fm_stream_copy_probe"] = ("fm_stream_copy_probe", None, ((src, dst), args))
    return dst

"""GPU parity: the HIP path (through the C ABI) against the reference goldens and the oracle.

Bit-exact: winsorize cuts and clipped values, NYSE breakpoints and universe masks, N and
month lists, the synthetic generator.  FP64 slopes/R2/t-stats/rolling/forecast moments:
|a-b| <= 1e-9 * max(|b|, RMS of the series) (tests/fmtol.py).
"""
import hashlib

import numpy as np
import pandas as pd
import pytest

import cases
from fmtol import (RTOL, assert_series_close, frame_from, load_json, load_npz, scalar_close)
from oracle import fm_oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def E():
    from fmcore import engine
    engine.require_device()
    return engine


@pytest.fixture(scope="module")
def R():
    from fmdrop import regressions
    return regressions


@pytest.fixture(scope="module")
def CL():
    from fmdrop import calc_Lewellen_2014
    return calc_Lewellen_2014


def _same(a, b):
    """Bit-exact up to NaN payloads: same NaN positions, same values, and the same SIGN of
    every zero (np.percentile's zero cuts take it from numpy's partition order)."""
    a, b = np.asarray(a), np.asarray(b)
    if a.shape != b.shape or not np.array_equal(np.isnan(a), np.isnan(b)):
        return False
    m = ~np.isnan(a)
    return np.array_equal(a[m], b[m]) and np.array_equal(np.signbit(a[m]), np.signbit(b[m]))


# ---------------------------------------------------------------- order statistics
def test_percentile_cuts_bit_exact(E):
    g = load_npz("pct.npz")
    vals, off, qs, ref = g["values"], g["offsets"], g["qs"], g["np_percentile"]
    labels = np.repeat(np.arange(len(off) - 1), np.diff(off))
    panel = E.panel_from_arrays([vals], ["v"], labels)
    pairs = [(0, 1), (2, 3), (4, 5), (6, 6)]
    for a, b in pairs:
        cuts = E.select_cuts(panel, qs[a] / 100, qs[b] / 100, 1, E.LERP_NUMPY)
        lo, hi = cuts.lo.cpu().numpy()[0], cuts.hi.cpu().numpy()[0]
        assert _same(lo, ref[:, a]), (qs[a], np.nonzero(~((lo == ref[:, a]) | (np.isnan(lo) & np.isnan(ref[:, a])))))
        assert _same(hi, ref[:, b]), qs[b]


def test_zero_cut_sign_bit_exact(E):
    """Cuts that are exactly zero (pct.npz arrays with +-0.0 ties): value AND sign equal the
    reference's np.percentile (numpy 1.26.4), whose sign comes from its partition's swap order
    over the values in frame order -- replayed on the device by the fix-up kernel
    (fm_npsel_dev.h) for units holding both signed zeros."""
    g = load_npz("pct.npz")
    vals, off, qs, ref = g["values"], g["offsets"], g["qs"], g["np_percentile"]
    labels = np.repeat(np.arange(len(off) - 1), np.diff(off))
    panel = E.panel_from_arrays([vals], ["v"], labels)
    zero = neg = flips = 0
    for a, b in [(0, 1), (2, 3), (4, 5), (6, 6)]:
        cuts = E.select_cuts(panel, qs[a] / 100, qs[b] / 100, 1, E.LERP_NUMPY)
        for got, j in ((cuts.lo.cpu().numpy()[0], a), (cuts.hi.cpu().numpy()[0], b)):
            z = ref[:, j] == 0.0
            assert np.array_equal(got[z], ref[z, j])
            zero += int(z.sum())
            neg += int(np.signbit(ref[z, j]).sum())
            flips += int(np.sum(np.signbit(got[z]) != np.signbit(ref[z, j])))
    assert zero > 100 and 0 < neg < zero
    assert flips == 0, f"{flips} of {zero} exactly-zero cuts differ in sign"


@pytest.mark.parametrize("n", [7, 300, 5000, 6144, 6145, 9000, 20000, 30000])
def test_zero_cut_sign_vs_numpy_partition(E, n):
    """Signed-zero-heavy months on every select path (two-wave kernel <= 6,144 rows, the
    long-month kernel 6,145-20,480, streaming beyond; LDS replay <= 6,144 rows, a global
    slot beyond): every cut bit-exact against the CPU restatement of numpy's partition
    (oracle/np_select.py, itself pinned to numpy 1.26.4), incl. month-of-zeros extremes and
    a median-of-3 killer that drives the partition into its median-of-medians pivots."""
    from oracle import np_select
    rng = np.random.default_rng(n)
    segs = []
    x = rng.choice([-0.0, 0.0], n)
    segs.append(x)                                                   # all zeros, both signs
    y = rng.standard_normal(n)
    y[rng.random(n) < 0.6] = rng.choice([-0.0, 0.0], int((rng.random(n) < 0.6).sum()) or 1)[0]
    y[rng.random(n) < 0.3] = -0.0
    segs.append(y)                                                   # zero run across both cut ranks
    z = np.where(rng.random(n) < 0.5, -0.0, 0.0)
    z[: n // 50] = -1.0
    z[-(n // 50):] = 1.0
    segs.append(rng.permutation(z))
    k = n // 2
    w = np.zeros(n)
    for i in range(1, k + 1):                                        # median-of-3 killer
        if i % 2 == 1:
            w[i - 1], w[i] = i, k + i
        w[k + i - 1] = 2 * i
    w = w - n // 2
    w[w == 0] = -0.0
    w[rng.random(n) < 0.2] = 0.0
    segs.append(w)
    vals = np.concatenate(segs)
    labels = np.repeat(np.arange(len(segs)), [len(s_) for s_ in segs])
    panel = E.panel_from_arrays([vals], ["v"], labels)
    for qa, qb in ((1, 99), (0, 100), (50, 50), (2, 98)):
        cuts = E.select_cuts(panel, qa / 100, qb / 100, 1, E.LERP_NUMPY)
        lo, hi = cuts.lo.cpu().numpy()[0], cuts.hi.cpu().numpy()[0]
        for t, s_ in enumerate(segs):
            for q, got in ((qa, lo[t]), (qb, hi[t])):
                exp = O.percentile_linear(s_, q)
                assert _same([got], [exp]), (n, t, q, got, exp)
    assert np_select is not None


def _adversarial_segments(rng, lengths=(1, 2, 3, 5, 10, 50, 63, 64, 65, 255, 256, 257, 1000, 5000,
                                        12345, 24000)):
    """Month segments that stress the tail fast path and its fallbacks: row-sorted data
    (the thread minima all sit in one wave), heavy ties, constants, infinities, NaNs, and
    lengths around the 256-thread / 64-lane boundaries."""
    segs = []
    for n in lengths:
        x = rng.standard_normal(n)
        segs.append(x)
        segs.append(np.sort(x))
        segs.append(np.sort(x)[::-1].copy())
        segs.append(rng.integers(0, 3, n).astype(np.float64))
        segs.append(np.full(n, 1.5))
        y = rng.standard_t(2, n)
        y[rng.random(n) < 0.3] = np.nan
        if n > 4:
            y[:2] = [np.inf, -np.inf]
        segs.append(y)
        z = rng.standard_normal(n)
        z[rng.random(n) < 0.05] = 0.0
        z[rng.random(n) < 0.05] = -0.0
        segs.append(z)
    return segs


@pytest.mark.parametrize("wave_path", [False, True])
def test_percentile_tails_adversarial(E, wave_path):
    """wave_path: every segment <= 6144 rows, so the wave-per-unit kernel runs first and
    the workgroup kernel redoes only the units it marks; otherwise the workgroup kernel
    does everything (a 24000-row segment exceeds the wave kernel's register budget)."""
    rng = np.random.default_rng(7)
    lengths = (1, 2, 3, 5, 10, 50, 63, 64, 65, 127, 128, 129, 255, 256, 257, 1000, 4999, 5000, 5120,
               6144) if wave_path else (1, 2, 3, 5, 10, 50, 63, 64, 65, 255, 256, 257, 1000, 5000, 12345,
                                        24000)
    segs = _adversarial_segments(rng, lengths)
    vals = np.concatenate(segs)
    labels = np.repeat(np.arange(len(segs)), [len(s) for s in segs])
    panel = E.panel_from_arrays([vals], ["v"], labels)
    for qa, qb in ((1, 99), (0, 100), (0.5, 99.5), (5, 95), (25, 75), (10, 99)):
        cuts = E.select_cuts(panel, qa / 100, qb / 100, 1, E.LERP_NUMPY)
        lo, hi = cuts.lo.cpu().numpy()[0], cuts.hi.cpu().numpy()[0]
        for t, s in enumerate(segs):
            v = s[~np.isnan(s)]
            if len(v) == 0:
                assert np.isnan(lo[t]) and np.isnan(hi[t])
                continue
            with np.errstate(invalid="ignore"):
                ra, rb = np.percentile(v, qa), np.percentile(v, qb)
            assert _same([lo[t]], [ra]) and _same([hi[t]], [rb]), (qa, qb, t, len(v), lo[t], ra, hi[t], rb)


def _hard_segment(rng, n, kind):
    if kind == "t2":
        x = rng.standard_t(2, n)
        x[rng.random(n) < 0.2] = np.nan
        x[:3] = [np.inf, -np.inf, -0.0]
        return x
    if kind == "ties":
        return rng.integers(-2, 3, n).astype(np.float64) * 0.5
    if kind == "const":
        return np.full(n, 2.5)
    if kind == "cluster":     # > HCAP keys inside one level-1 bin: the refinement levels
        x = 1.0 + rng.integers(0, 4000, n) * np.finfo(np.float64).eps
        x[rng.random(n) < 0.01] = -1e300
        x[rng.random(n) < 0.01] = 1e300
        return x
    raise ValueError(kind)


@pytest.mark.parametrize("n", [30000, 100000, 1000000])
def test_long_segment_cuts_bit_exact(E, n):
    """Segments longer than the 24,576-row register budget stream from HBM (adaptive
    histogram select): bit-exact against np.percentile and the pandas group-quantile lerp,
    on heavy tails with NaN / +-inf / -0.0, heavy ties, a constant segment and clustered
    keys behind extreme outliers, next to a short segment."""
    rng = np.random.default_rng(n)
    kinds = ["t2", "ties", "const", "cluster"]
    segs = [_hard_segment(rng, n, k) for k in kinds] + [rng.standard_normal(777)]
    vals = np.concatenate(segs)
    labels = np.repeat(np.arange(len(segs)), [len(x) for x in segs])
    panel = E.panel_from_arrays([vals], ["v"], labels)
    for qa, qb in ((1, 99), (0, 100), (20, 50)):
        cuts = E.select_cuts(panel, qa / 100, qb / 100, 1, E.LERP_NUMPY)
        lo, hi = cuts.lo.cpu().numpy()[0], cuts.hi.cpu().numpy()[0]
        for t, x in enumerate(segs):
            v = x[~np.isnan(x)]
            with np.errstate(invalid="ignore"):
                ra, rb = np.percentile(v, qa), np.percentile(v, qb)
            assert _same([lo[t]], [ra]) and _same([hi[t]], [rb]), (kinds + ["short"])[t]
    cuts = E.select_cuts(panel, 0.2, 0.5, 1, E.LERP_PANDAS)
    lo, hi = cuts.lo.cpu().numpy()[0], cuts.hi.cpu().numpy()[0]
    for t, x in enumerate(segs):
        y = np.where(np.isfinite(x), x, np.nan) if t == 0 else x
        if t == 0:
            continue    # pandas' quantile of +-inf rows is not the lerp's business
        assert _same([lo[t]], [O.pandas_quantile(y, 0.2)]) and _same([hi[t]], [O.pandas_quantile(y, 0.5)])


def _thread_clustered_segment(rng, n):
    """Both tails sit in the rows of 64 of the long kernel's 512 threads (row % 512), so the
    thread-extremum bound leaves far more than 512 candidates: the unit is marked and the
    streaming fallback redoes it."""
    x = rng.standard_normal(n)
    r = np.arange(n) % 512
    x[r < 64] -= 100.0
    x[r >= 448] += 100.0
    return x


@pytest.mark.parametrize("maxlen", [8192, 12288, 16384, 20480])
def test_long_month_register_select_bit_exact(E, maxlen):
    """Months of 6,145 .. 20,480 rows (C5's 20,000-firm cross-sections) take the 512-thread
    register-resident kernel (one read per unit; VPT 16 / 24 / 32 / 40 by the longest month)
    and the streaming fallback for the units it marks: bit-exact against np.percentile on
    the adversarial kinds, the hard segments and thread-clustered tails, next to short
    segments (which ride the same launch)."""
    rng = np.random.default_rng(maxlen)
    lengths = sorted({1, 5, 257, 5000, 6145, maxlen - 1, maxlen, (6145 + maxlen) // 2})
    segs = _adversarial_segments(rng, lengths)
    segs += [_hard_segment(rng, maxlen, k) for k in ("t2", "ties", "const", "cluster")]
    segs += [_thread_clustered_segment(rng, maxlen), _thread_clustered_segment(rng, 6200)]
    vals = np.concatenate(segs)
    labels = np.repeat(np.arange(len(segs)), [len(s) for s in segs])
    panel = E.panel_from_arrays([vals], ["v"], labels)
    assert panel.max_seg_len == maxlen
    for qa, qb in ((1, 99), (0, 100), (5, 95), (25, 75)):
        cuts = E.select_cuts(panel, qa / 100, qb / 100, 1, E.LERP_NUMPY)
        lo, hi = cuts.lo.cpu().numpy()[0], cuts.hi.cpu().numpy()[0]
        nv = cuts.nvalid.cpu().numpy()[0]
        assert (nv >= 0).all()    # every marked unit was redone
        for t, s in enumerate(segs):
            v = s[~np.isnan(s)]
            assert nv[t] == len(v)
            if len(v) == 0:
                assert np.isnan(lo[t]) and np.isnan(hi[t])
                continue
            with np.errstate(invalid="ignore"):
                ra, rb = np.percentile(v, qa), np.percentile(v, qb)
            assert _same([lo[t]], [ra]) and _same([hi[t]], [rb]), (qa, qb, t, len(v), lo[t], ra, hi[t], rb)


def _high_word_tie_segments(rng, n):
    """Months whose cut ranks sit in runs of equal HIGH 32-bit words (values differing only
    in the low word), exact duplicates at the ranks, and the high-word plane's ambiguous keys."""
    segs = []
    x = rng.standard_normal(n)
    k = max(1, n // 100)
    lo_ix = np.argsort(x)[: 3 * k]
    base = np.float64(-2.5).view(np.uint64)
    x[lo_ix] = (base + rng.integers(0, 2 ** 16, lo_ix.size).astype(np.uint64)).view(np.float64)
    segs.append(x)                                   # ~3k values share one high word at the low cut
    y = rng.standard_normal(n)
    y[np.argsort(y)[-2 * k:]] = 4.0                  # exact duplicates across the upper cut
    segs.append(y)
    z = rng.standard_normal(n)
    z[rng.choice(n, 4, replace=False)] = [np.inf, -np.inf, np.inf, -np.inf]
    segs.append(z)                                   # +-inf: ambiguous high words -> fix-up
    w = rng.standard_normal(n)
    w[rng.choice(n, 6, replace=False)] = _payload_nan(1, 6)
    segs.append(w)
    v = np.round(rng.standard_normal(n), 2)          # heavy exact ties everywhere
    segs.append(v)
    return segs


@pytest.mark.parametrize("maxlen", [128, 5000, 6144, 9000, 20000])
def test_hi_plane_select_bit_exact(E, maxlen):
    """The split panel: the two-wave kernel (<= 6,144-row months) and the long-month kernel
    order values by their HIGH words (fm_split_planes) and gather full values only at the
    target ranks.  Cuts, counts and pivots bit-identical to the FP64-column path and to
    np.percentile, over the adversarial kinds, high-word ties at the cut ranks, duplicates,
    +-inf and low-payload NaNs."""
    rng = np.random.default_rng(maxlen + 11)
    lengths = sorted(x for x in {1, 2, 5, 63, 64, 65, 127, 128, 129, maxlen // 2 + 1, maxlen - 1, maxlen} if x <= maxlen)
    segs = _adversarial_segments(rng, lengths) + _high_word_tie_segments(rng, maxlen)
    vals = np.concatenate(segs)
    labels = np.repeat(np.arange(len(segs)), [len(s_) for s_ in segs])
    panel = E.panel_from_arrays([vals, vals[::-1].copy()], ["v", "r"], labels)
    rv = [np.concatenate(segs)[::-1]]
    assert panel.max_seg_len == maxlen
    qs = ((1, 99), (0, 100), (5, 95))
    ref = [E.select_cuts(panel, a / 100, b / 100, 1, E.LERP_NUMPY, center=True) for a, b in qs]
    E.split_planes(panel)
    for (qa, qb), r in zip(qs, ref):
        got = E.select_cuts(panel, qa / 100, qb / 100, 1, E.LERP_NUMPY, center=True)
        for f in ("lo", "hi", "center"):
            assert _same(getattr(got, f).cpu().numpy(), getattr(r, f).cpu().numpy()), (qa, qb, f)
        assert np.array_equal(got.nvalid.cpu().numpy(), r.nvalid.cpu().numpy())
        lo, hi = got.lo.cpu().numpy()[0], got.hi.cpu().numpy()[0]
        for t, s_ in enumerate(segs):
            v = s_[~np.isnan(s_)]
            if len(v) == 0:
                continue
            assert _same([lo[t]], [O.percentile_linear(v, qa)]) and _same([hi[t]], [O.percentile_linear(v, qb)]), \
                (qa, qb, t, len(v))
    assert rv is not None


def _payload_nan(sign, n):
    """n NaNs whose payload sits entirely in the LOW 32 bits (high word 0x7FF00000 /
    0xFFF00000, the same high word as +-inf)."""
    bits = np.full(n, (0xFFF00000 if sign < 0 else 0x7FF00000) << 32, dtype=np.uint64)
    bits |= np.arange(1, n + 1, dtype=np.uint64)
    return bits.view(np.float64)


@pytest.mark.parametrize("maxlen", [9000, 20000])
def test_long_month_high_key_edge_cases(E, maxlen):
    """The long-month kernel orders values by the high 32 bits of their keys until the final
    candidate sort.  Units whose high words cannot tell +-inf from a NaN (payload only in the
    low word) are redone by the streaming kernel: bit-exact against np.percentile over the
    non-NaN values with such NaNs, with +-inf in the tails, with both, with values that share
    high words across the cut ranks (differing only in the low word), and with the cut ranks
    inside a long run of equal high words."""
    rng = np.random.default_rng(maxlen + 7)
    n = maxlen
    segs = []
    x = rng.standard_normal(n)
    x[rng.choice(n, 40, replace=False)] = _payload_nan(1, 40)
    x[rng.choice(n, 40, replace=False)] = _payload_nan(-1, 40)
    segs.append(x)                                   # low-payload NaNs, no infinities
    x = rng.standard_normal(n)
    x[rng.choice(n, 30, replace=False)] = np.inf
    x[rng.choice(n, 30, replace=False)] = -np.inf
    segs.append(x)                                   # +-inf inside both tails
    x = rng.standard_normal(n)
    x[rng.choice(n, 5, replace=False)] = np.inf
    x[rng.choice(n, 25, replace=False)] = _payload_nan(1, 25)
    segs.append(x)                                   # both
    base = 1.0 + rng.integers(0, 2 ** 20, n).astype(np.uint64)   # low-word-only differences
    segs.append((np.float64(3.0).view(np.uint64) + base).view(np.float64) * np.where(rng.random(n) < 0.5, 1, -1))
    x = rng.standard_normal(n)
    k = n // 20                                      # 5% of rows: one high word at each end
    x[:k] = (np.float64(-7.0).view(np.uint64) + np.arange(k, dtype=np.uint64)).view(np.float64)
    x[-k:] = (np.float64(7.0).view(np.uint64) + np.arange(k, dtype=np.uint64)).view(np.float64)
    segs.append(rng.permutation(x))
    segs.append(rng.standard_normal(6500))
    vals = np.concatenate(segs)
    labels = np.repeat(np.arange(len(segs)), [len(s) for s in segs])
    panel = E.panel_from_arrays([vals], ["v"], labels)
    assert panel.max_seg_len == maxlen
    for qa, qb in ((1, 99), (0, 100), (2, 98)):
        cuts = E.select_cuts(panel, qa / 100, qb / 100, 1, E.LERP_NUMPY, center=True)
        lo, hi = cuts.lo.cpu().numpy()[0], cuts.hi.cpu().numpy()[0]
        nv = cuts.nvalid.cpu().numpy()[0]
        for t, s in enumerate(segs):
            v = s[~np.isnan(s)]
            assert nv[t] == len(v), t
            with np.errstate(invalid="ignore"):
                ra, rb = np.percentile(v, qa), np.percentile(v, qb)
            assert _same([lo[t]], [ra]) and _same([hi[t]], [rb]), (qa, qb, t, lo[t], ra, hi[t], rb)


def test_masked_middle_quantiles_hist_select(E):
    """NYSE-style row-masked middle quantiles (pandas lerp) through the workgroup path's
    adaptive histogram select, incl. clustered keys that need the refinement levels."""
    rng = np.random.default_rng(5)
    segs, masks = [], []
    for n in (1, 2, 7, 300, 5000, 20000):
        for kind in ("lognormal", "cluster", "ties"):
            x = np.exp(rng.normal(5, 2, n)) if kind == "lognormal" else _hard_segment(rng, n, kind)
            segs.append(x)
            masks.append(rng.random(n) < 0.4)
    vals = np.concatenate(segs)
    mask = np.concatenate(masks).astype(np.uint8)
    labels = np.repeat(np.arange(len(segs)), [len(x) for x in segs])
    panel = E.panel_from_arrays([vals], ["me"], labels, me=vals, nyse=mask)
    a, b = E.nyse_breakpoints(panel)
    a, b = a.cpu().numpy(), b.cpu().numpy()
    for t, (x, m) in enumerate(zip(segs, masks)):
        assert _same([a[t]], [O.pandas_quantile(x[m], 0.2)]), t
        assert _same([b[t]], [O.pandas_quantile(x[m], 0.5)]), t


@pytest.mark.parametrize("maxlen", [6000, 20000, 30000])
def test_select_level_output(E, maxlen):
    """fm_select's level output (get_subsets' nested masks from the NYSE cuts, reference
    src/calc_Lewellen_2014.py:95-105) after every select path: <= 6,144-row months (the
    workgroup kernel), 6,145..20,480 (the register kernel), longer (streaming); NaN me on
    NYSE and other rows, a month without NYSE rows (NaN cuts: level 0)."""
    import torch
    rng = np.random.default_rng(maxlen)
    segs, masks = [], []
    for n in (1, 7, 300, maxlen // 2, maxlen):
        x = np.exp(rng.normal(5, 2, n))
        x[rng.random(n) < 0.05] = np.nan
        segs.append(x)
        masks.append(rng.random(n) < 0.4)
    segs.append(np.exp(rng.normal(5, 2, 500)))
    masks.append(np.zeros(500, dtype=bool))
    vals = np.concatenate(segs)
    mask = np.concatenate(masks).astype(np.uint8)
    labels = np.repeat(np.arange(len(segs)), [len(x) for x in segs])
    panel = E.panel_from_arrays([vals], ["me"], labels, me=vals, nyse=mask)
    level = torch.full((panel.nrows,), 7, dtype=torch.uint8, device=panel.cols.device)
    a, b = E.nyse_breakpoints(panel, level=level)
    a, b, level = a.cpu().numpy(), b.cpu().numpy(), level.cpu().numpy()
    off = panel.seg_off_h
    for t, (x, m) in enumerate(zip(segs, masks)):
        v = x[m & ~np.isnan(x)]
        ea = O.pandas_quantile(v, 0.2) if v.size else np.nan
        eb = O.pandas_quantile(v, 0.5) if v.size else np.nan
        assert _same([a[t]], [ea]) and _same([b[t]], [eb]), t
        with np.errstate(invalid="ignore"):
            exp = (x >= ea).astype(np.uint8) + (x >= eb).astype(np.uint8)
        assert np.array_equal(level[off[t]:off[t + 1]], exp), t


def test_universe_kernel_vs_oracle(E):
    """fm_universe (NYSE me_20 / me_50 + the nested level byte, one launch) against the
    pandas lerp restatement and the reference's masks (me >= cut, NaN False): months of
    1 .. 16,384 rows (the register budget's edge), lognormal / clustered / tied keys, NaN me
    on NYSE and non-NYSE rows, a month without NYSE rows and one whose NYSE me are all NaN."""
    rng = np.random.default_rng(55)
    segs, masks = [], []
    for n in (1, 2, 7, 300, 5000, 16384):
        for kind in ("lognormal", "cluster", "ties"):
            x = np.exp(rng.normal(5, 2, n)) if kind == "lognormal" else _hard_segment(rng, n, kind)
            x[rng.random(n) < 0.05] = np.nan
            segs.append(x)
            masks.append(rng.random(n) < 0.4)
    segs.append(np.exp(rng.normal(5, 2, 900)))
    masks.append(np.zeros(900, dtype=bool))                       # no NYSE row
    x = np.exp(rng.normal(5, 2, 900))
    m = rng.random(900) < 0.4
    x[m] = np.nan
    segs.append(x)
    masks.append(m)                                               # every NYSE me NaN
    vals = np.concatenate(segs)
    mask = np.concatenate(masks).astype(np.uint8)
    labels = np.repeat(np.arange(len(segs)), [len(x) for x in segs])
    panel = E.panel_from_arrays([vals], ["me"], labels, me=vals, nyse=mask)
    assert panel.max_seg_len <= E.UNIVERSE_MAX_ROWS
    a, b, level = E.universe(panel)
    assert "fm_universe" in E.LAST_LAUNCH
    a, b, level = a.cpu().numpy(), b.cpu().numpy(), level.cpu().numpy()
    off = panel.seg_off_h
    for t, (x, m) in enumerate(zip(segs, masks)):
        v = x[m & ~np.isnan(x)]
        ea = O.pandas_quantile(v, 0.2) if v.size else np.nan
        eb = O.pandas_quantile(v, 0.5) if v.size else np.nan
        assert _same([a[t]], [ea]) and _same([b[t]], [eb]), t
        with np.errstate(invalid="ignore"):
            exp = (x >= ea).astype(np.uint8) + (x >= eb).astype(np.uint8)
        assert np.array_equal(level[off[t]:off[t + 1]], exp), t


@pytest.mark.parametrize("maxlen", [2500, 5120, 6144, 9000, 20000, 24000])
def test_select_universe_fused(E, maxlen):
    """fm_select_universe: the winsorize cuts and get_subsets' NYSE breakpoints + level bytes
    from one call.  Months of <= 5,120 rows (the two-wave kernel) run the universe in the
    select fix-up's launch; 6,145-20,480 rows ride the long-month high-key kernel's launch
    (one more grid column); 5,121-6,144 (the workgroup kernel) and longer ones (the streaming
    select) launch the universe on its own first (fm_universe / the row-masked NYSE select).  Cuts must equal fm_select's alone bit for bit, breakpoints the
    pandas lerp restatement and levels the reference's masks, over adversarial me months
    (clusters, ties, NaN me, no NYSE row, every NYSE me NaN, 1-row months)."""
    rng = np.random.default_rng(77)
    segs, masks = [], []
    for n in (1, 2, 7, 300, 2500, maxlen):
        for kind in ("lognormal", "cluster", "ties"):
            x = np.exp(rng.normal(5, 2, n)) if kind == "lognormal" else _hard_segment(rng, n, kind)
            x[rng.random(n) < 0.05] = np.nan
            segs.append(x)
            masks.append(rng.random(n) < 0.4)
    segs.append(np.exp(rng.normal(5, 2, 900)))
    masks.append(np.zeros(900, dtype=bool))
    x = np.exp(rng.normal(5, 2, 900))
    m = rng.random(900) < 0.4
    x[m] = np.nan
    segs.append(x)
    masks.append(m)
    me = np.concatenate(segs)
    ny = np.concatenate(masks).astype(np.uint8)
    labels = np.repeat(np.arange(len(segs)), [len(x) for x in segs])
    cols = [rng.standard_t(2, me.size) for _ in range(4)]
    for c in cols:
        c[rng.random(me.size) < 0.03] = np.nan
    panel = E.panel_from_arrays(cols, ["a", "b", "c", "d"], labels, me=me, nyse=ny)
    ref = E.select_cuts(panel, 0.01, 0.99, 5, E.LERP_NUMPY, center=True)
    cuts, (a, b, level) = E.select_cuts(panel, 0.01, 0.99, 5, E.LERP_NUMPY, center=True, universe=(0.2, 0.5))
    for x_, y_ in ((cuts.lo, ref.lo), (cuts.hi, ref.hi), (cuts.nvalid, ref.nvalid), (cuts.center, ref.center)):
        assert _same(x_.cpu().numpy(), y_.cpu().numpy())
    ua, ub, ul = E.universe(panel)
    assert _same(a.cpu().numpy(), ua.cpu().numpy()) and _same(b.cpu().numpy(), ub.cpu().numpy())
    assert np.array_equal(level.cpu().numpy(), ul.cpu().numpy())
    a, b, level = a.cpu().numpy(), b.cpu().numpy(), level.cpu().numpy()
    off = panel.seg_off_h
    order = panel.order
    for t in range(len(segs)):
        xs = me[order][off[t]:off[t + 1]]
        ms = ny[order][off[t]:off[t + 1]].astype(bool)
        v = xs[ms & ~np.isnan(xs)]
        ea = O.pandas_quantile(v, 0.2) if v.size else np.nan
        eb = O.pandas_quantile(v, 0.5) if v.size else np.nan
        assert _same([a[t]], [ea]) and _same([b[t]], [eb]), t
        with np.errstate(invalid="ignore"):
            exp = (xs >= ea).astype(np.uint8) + (xs >= eb).astype(np.uint8)
        assert np.array_equal(level[off[t]:off[t + 1]], exp), t


def test_select_universe_fused_bench_panel(E):
    """The bench panel (600 x 5,000, generated in HBM): fused cuts / breakpoints / levels equal
    the separate fm_select + fm_universe launches bit for bit."""
    panel = E.panel_synthetic(600, 5000, 1)
    ref = E.select_cuts(panel, 0.01, 0.99, 5, E.LERP_NUMPY, center=True)
    ua, ub, ul = E.universe(panel)
    cuts, (a, b, level) = E.select_cuts(panel, 0.01, 0.99, 5, E.LERP_NUMPY, center=True, universe=(0.2, 0.5))
    for x_, y_ in ((cuts.lo, ref.lo), (cuts.hi, ref.hi), (cuts.nvalid, ref.nvalid), (cuts.center, ref.center),
                   (a, ua), (b, ub)):
        assert _same(x_.cpu().numpy(), y_.cpu().numpy())
    assert np.array_equal(level.cpu().numpy(), ul.cpu().numpy())


def test_pandas_quantile_bit_exact(E):
    g = load_npz("pct.npz")
    vals, off, ref = g["values"], g["offsets"], g["pd_quantile"]
    labels = np.repeat(np.arange(len(off) - 1), np.diff(off))
    v = np.where(np.isfinite(vals), vals, np.nan)   # the golden used finite values only
    panel = E.panel_from_arrays([v], ["v"], labels)
    cuts = E.select_cuts(panel, 0.2, 0.5, 1, E.LERP_PANDAS)
    # values bit-exact; the sign of an exactly-zero pandas quantile is not compared: pandas'
    # group_quantile orders equal values by an unstable argsort that numpy dispatches to its
    # AVX-512 sort on the host that made the golden (get_subsets' NYSE me is positive anyway)
    for got, exp in ((cuts.lo.cpu().numpy()[0], ref[:, 0]), (cuts.hi.cpu().numpy()[0], ref[:, 1])):
        assert _same(np.where(got == 0.0, 0.0, got), np.where(exp == 0.0, 0.0, exp))


def test_winsorize_cuts_and_frame_bit_exact(E, CL):
    g = load_npz("wins.npz")
    df = frame_from(g, "in_")
    srt = df.sort_values(["mthcaldt", "permno"])
    panel = E.panel_from_arrays([srt[v].values for v in cases.WINSOR_VARS], cases.WINSOR_VARS,
                                srt["mthcaldt"].values)
    cuts = E.select_cuts(panel, 0.01, 0.99, 5, E.LERP_NUMPY)
    assert _same(cuts.lo.cpu().numpy(), g["cut_lo"])
    assert _same(cuts.hi.cpu().numpy(), g["cut_hi"])
    assert np.array_equal(cuts.nvalid.cpu().numpy(), g["cut_n"])
    got = CL.winsorize(df, cases.WINSOR_VARS, 1, 99)
    exp = frame_from(g, "out_")
    assert list(got.index) == list(exp.index)
    for v in cases.WINSOR_VARS:
        assert _same(got[v].values, exp[v].values), v


def test_gen_panel_matches_numpy_generator(E):
    from fmcore import synth
    T, N, seed = 7, 333, 20150101
    panel = E.panel_synthetic(T, N, seed, month0=5, nan_rate=0.02)
    a = synth.synth_arrays(T, N, seed, nan_rate=0.02, month0=5)
    cols = panel.cols.cpu().numpy()
    for i, v in enumerate(synth.WINSOR_VARS):
        assert _same(cols[i], a[v]), v
    assert _same(panel.me.cpu().numpy(), a["me"])
    assert np.array_equal(panel.nyse.cpu().numpy().astype(bool), a["nyse"])


# ---------------------------------------------------------------- universes
def test_get_subsets_bit_exact(CL):
    g = load_npz("fm.npz")
    df = frame_from(g, "in_")
    w = CL.winsorize(df, cases.WINSOR_VARS, 1, 99)
    subs = CL.get_subsets(w)
    exp = frame_from(g, "sub_")
    a = subs["All stocks"]
    for c in ("me_20", "me_50"):
        assert _same(a[c].values, exp[c].values), c
    for c in ("is_all_but_tiny", "is_large"):
        assert np.array_equal(a[c].values, exp[c].values), c
    for s in cases.SUBSETS:
        assert len(subs[s]) == int(g["len|" + s][0])


# ---------------------------------------------------------------- regressions
def _check_cs(got, g, key, xs):
    n = g[key + "|N"]
    if len(n) == 0:
        assert len(got) == 0
        return
    assert list(got.columns) == ["mthcaldt", "N", "R2"] + ["slope_" + x for x in xs]
    assert np.array_equal(got["N"].values, n), key
    assert np.array_equal(got["mthcaldt"].values.astype("datetime64[ns]").astype(np.int64), g[key + "|date"])
    assert_series_close(got["R2"].values, g[key + "|R2"], key + " R2")
    for x in xs:
        assert_series_close(got["slope_" + x].values, g[key + "|slope_" + x], key + " " + x)


def test_fm_regressions_and_summaries_golden(R, CL):
    g = load_npz("fm.npz")
    meta = load_json("fm.json")
    df = frame_from(g, "in_")
    subs = CL.get_subsets(CL.winsorize(df, cases.WINSOR_VARS, 1, 99))
    for mname, xs in cases.MODELS.items():
        for s in cases.SUBSETS:
            key = f"{mname}|{s}"
            got = R.run_monthly_cs_regressions(subs[s], "retx", xs, "mthcaldt")
            _check_cs(got, g, key, xs)
            summ = R.fama_macbeth_summary(got, xs, "mthcaldt", 4)
            assert list(summ.index) == list(meta[key].keys())
            for k, v in meta[key].items():
                assert scalar_close(summ[k], v), (key, k, summ[k], v)


def test_build_table_2_strings_golden(CL):
    g = load_npz("fm.npz")
    meta = load_json("fm.json")["table2"]
    df = frame_from(g, "in_")
    subs = CL.get_subsets(CL.winsorize(df, cases.WINSOR_VARS, 1, 99))
    t2 = CL.build_table_2(subs, cases.VARIABLES_DICT)
    assert [list(i) for i in t2.index] == meta["index"]
    assert [list(c) for c in t2.columns] == meta["columns"]
    assert [[str(x) for x in r] for r in t2.values.tolist()] == meta["values"]


def _edge_inputs(g):
    """The edge cases with the INPUT frames stored in edge.npz (the exact inputs the
    reference saw), not regenerated: a regeneration can differ in the last ulp."""
    for name, _, xs in cases.edge_cases():
        yield name, frame_from(g, name + "|in_"), xs


def test_edge_cases_golden(R):
    g = load_npz("edge.npz")
    meta = load_json("edge.json")
    for name, df, xs in _edge_inputs(g):
        m = meta[name]
        if m["error"]:
            exc = {"MissingDataError": R.MissingDataError, "IndexError": IndexError}[m["error"]]
            with pytest.raises(exc):
                R.run_monthly_cs_regressions(df, "retx", xs, "mthcaldt")
            continue
        got = R.run_monthly_cs_regressions(df, "retx", xs, "mthcaldt")
        assert list(got.columns) == m["columns"], name
        exp = frame_from(g, name + "|out_")
        assert np.array_equal(got["N"].values, exp["N"].values), name
        for c in got.columns[2:]:
            assert_series_close(got[c].values, exp[c].values, f"{name} {c}")
        summ = R.fama_macbeth_summary(got, xs, "mthcaldt", 4)
        assert list(summ.index) == m["summary_keys"]
        for k, v in m["summary"].items():
            assert scalar_close(summ[k], v), (name, k, summ[k], v)


def test_affine_collinear_pinned(R):
    """x2 = 2 x1 + 0.5 in every month: statsmodels' pinv null space involves the intercept;
    the Jacobi fallback's uncentered min-norm correction (fm_solve.hip jacobi_pinv) matches
    the reference's slopes, R2 and summaries at 1e-9 (diverge.npz, reference-generated)."""
    g = load_npz("diverge.npz")
    meta = load_json("diverge.json")
    name, _, xs = cases.divergence_cases()[0]
    df = frame_from(g, name + "|in_")
    got = R.run_monthly_cs_regressions(df, "retx", xs, "mthcaldt")
    exp = frame_from(g, name + "|out_")
    assert np.array_equal(got["N"].values, exp["N"].values)
    for c in got.columns[2:]:
        assert_series_close(got[c].values, exp[c].values, f"{name} {c}")
    summ = R.fama_macbeth_summary(got, xs, "mthcaldt", 4)
    for k, v in meta[name]["summary"].items():
        assert scalar_close(summ[k], v), (name, k, summ[k], v)


def _assert_conditioned(got, exp, xs, pair, cond_tol):
    """N exact; every other column within max(1e-9, cond_tol).  cond_tol is the rounding
    floor eps * cond([1, X]) of any backward-stable solve — statsmodels' own SVD and its
    resid = y - X @ params included — so below it neither side is more right."""
    assert np.array_equal(got["N"].values, exp["N"].values)
    tol = max(RTOL, cond_tol)
    assert_series_close(got["R2"].values, exp["R2"].values, "R2", rtol=tol)
    for c in xs:
        assert_series_close(got[f"slope_{c}"].values, exp[f"slope_{c}"].values, c, rtol=tol)
    a, b = (f"slope_{c}" for c in pair)
    assert_series_close(got[a].values + got[b].values, exp[a].values + exp[b].values, "pair sum", rtol=tol)


def test_near_collinear_refit(R):
    """x2 = x1 + 1e-7 noise (sigma_min / sigma_max of [1, X] ~ 1e-7), reference-generated
    golden: cond(Sxx) ~ 1e14 is beyond the normal equations, so fm_solve flags the months
    FM_ST_REFIT and fm_solve_fixup re-solves them from the rows (Householder QR + one-sided
    Jacobi SVD, statsmodels' pinv semantics).  Within eps * cond ~ 1e-7 of the reference
    (measured on MI355X: R2 2.3e-9 relative)."""
    g = load_npz("diverge.npz")
    name, _, xs = cases.divergence_cases()[1]
    df = frame_from(g, name + "|in_")
    got = R.run_monthly_cs_regressions(df, "retx", xs, "mthcaldt")
    exp = frame_from(g, name + "|out_")
    _assert_conditioned(got, exp, xs, ("x1", "x2"), 1e-7)


@pytest.mark.parametrize("noise", [1e-2, 1e-4, 1e-6, 1e-8, 1e-10])
def test_conditioning_sweep_vs_pinv(R, noise):
    """x2 = x1 + noise * N(0,1) with noise 1e-2 .. 1e-10 (cond([1, X]) ~ 1e2 / noise), plus a
    large-mean regressor (x3 = 100 + x): months whose Sxx pivots fall below 1e-6 take the
    QR + SVD refit, the rest the Cholesky.  Against the oracle's SVD pinv (= statsmodels'
    pinv_extended) within max(1e-9, 2e-13 / noise)."""
    df = cases._edge_base(8, 300, 4, 77)
    rng = np.random.default_rng(78)
    df["x2"] = df["x1"] + noise * rng.standard_normal(len(df))
    df["x3"] = 100.0 + df["x3"]
    xs = ["x0", "x1", "x2", "x3"]
    got = R.run_monthly_cs_regressions(df, "retx", xs, "mthcaldt")
    exp = O.run_monthly_cs_regressions(df, "retx", xs, "mthcaldt")
    _assert_conditioned(got, exp, xs, ("x1", "x2"), 2e-13 / noise)


def test_inf_in_y_matches_pinv_semantics(R):
    g = load_npz("edge.npz")
    name, df, xs = [c for c in _edge_inputs(g) if c[0] == "inf_y"][0]
    got = R.run_monthly_cs_regressions(df, "retx", xs, "mthcaldt")
    exp = frame_from(g, name + "|out_")
    for c in got.columns[2:]:
        assert_series_close(got[c].values, exp[c].values, c)


def test_newey_west_golden(R):
    for case in load_json("nw.json"):
        got = R.newey_west_mean_se(np.array(case["x"]), case["lags"])
        assert scalar_close(got, case["se"], 1e-12), case["lags"]


@pytest.mark.parametrize("T", [4095, 4096, 10000, 100000])
def test_long_series_summary_vs_oracle(E, T):
    """fm_ts_summary on long series (>= 4,096 months: the chunked one-pass kernels -- shifted
    sums and lagged cross sums per 2,048-row chunk, combined in chunk order) against the
    oracle's two-pass mean / Newey-West s.e. on the dropna'd series, lags 0..8: NaN runs
    across chunk boundaries (longer than the lag), a NaN-led series, a series with a large
    mean relative to its spread, an all-NaN column and a column with one value."""
    import torch
    from fmcore import api
    rng = np.random.default_rng(T)
    cols = []
    x = rng.standard_normal(T) * 0.05 + 0.01
    x[rng.random(T) < 0.1] = np.nan
    x[2040:2060] = np.nan                      # straddles the first chunk boundary
    cols.append(x)
    y = rng.standard_t(3, T)
    y[:7] = np.nan                             # K0 is the 8th value
    cols.append(y)
    cols.append(1e3 + rng.standard_normal(T) * 1e-3)   # mean >> spread
    cols.append(np.full(T, np.nan))
    z = np.full(T, np.nan)
    z[T // 2] = 2.5
    cols.append(z)
    vals = torch.from_numpy(np.stack(cols, axis=1)).to(E.require_device())
    for lags in (0, 1, 4, 8):
        mean, se, t, nobs = api.records_summary_device(vals, lags)
        for j, c in enumerate(cols):
            v = c[~np.isnan(c)]
            assert nobs[j] == v.size, (lags, j)
            if v.size == 0:
                assert np.isnan(mean[j]) and np.isnan(se[j])
                continue
            assert scalar_close(mean[j], v.mean(), RTOL, 1e-12), (lags, j)
            exp = O.newey_west_mean_se(v, lags)
            if np.isnan(exp):
                assert np.isnan(se[j]), (lags, j)
            else:
                assert scalar_close(se[j], exp, 1e-9, 1e-15), (lags, j, se[j], exp)


@pytest.mark.parametrize("fixture,panel", [("fig1.npz", cases.fig1_panel), ("fig1c.npz", cases.fig1_const_panel)])
def test_figure1_golden(CL, fixture, panel):
    """fig1c: Figure-1 regressors constant within a month (has_constant='add'), the
    intercept split over [1, c] by the uncentered min-norm (reference :913-921)."""
    g = load_npz(fixture)
    df = panel()
    h = hashlib.sha256()
    for c in cases.WINSOR_VARS + ["me"]:
        h.update(np.ascontiguousarray(df[c].values).tobytes())
    assert h.hexdigest().encode() == g["in_sha"].tobytes()
    subs = CL.get_subsets(CL.winsorize(df, cases.WINSOR_VARS, 1, 99))
    res = CL.figure_1_coefficients(subs)
    for tag, name in (("all", "All stocks"), ("large", "Large stocks")):
        monthly, roll = res[name]
        assert np.array_equal(monthly.index.values.astype("datetime64[ns]").astype(np.int64), g[tag + "|date"])
        for k in range(6):
            assert_series_close(monthly.values[:, k], g[tag + "|params"][:, k], f"{tag} param {k}")
        for k, v in enumerate(cases.FIG1_VARS):
            assert_series_close(roll[v].values, g[tag + "|rolling_plotted"][:, k], f"{tag} roll {v}")
    fig, axes = CL.create_figure_1(subs)
    assert len(axes) == 2 and len(axes[0].lines) == 5


def test_mid_panel_golden(R):
    g = load_npz("mid.npz")
    meta = load_json("mid.json")
    df = cases.mid_panel()
    for mname in ("M2", "M3"):
        xs = cases.MODELS[mname]
        got = R.run_monthly_cs_regressions(df, "retx", xs)
        assert np.array_equal(got["N"].values, g[mname + "|N"])
        assert_series_close(got["R2"].values, g[mname + "|R2"], mname)
        for k, x in enumerate(xs):
            assert_series_close(got["slope_" + x].values, g[mname + "|slopes"][:, k], mname + x)
        summ = R.fama_macbeth_summary(got, xs)
        for k, v in meta[mname].items():
            assert scalar_close(summ[k], v), (mname, k)


# ---------------------------------------------------------------- full pipeline vs oracle
def _compare_with_oracle(res, model_names, model_cols, ref, summary, rolling, pred_t, pst_t, pred_summary):
    """Every problem of a device pass against oracle.pipeline_arrays on the same month-sorted
    arrays: fitted-month lists and N exact; params, R2, rolling means, predictive slopes/R2
    and every FM / predictive summary within the series-RMS tolerance."""
    rec = res.rec.cpu().numpy()
    st = res.status.cpu().numpy()
    mean = summary.mean.cpu().numpy()
    tstat = summary.tstat.cpu().numpy()
    roll = rolling.cpu().numpy()
    pred = pred_t.cpu().numpy()
    pst = pst_t.cpu().numpy()
    pmean = pred_summary.mean.cpu().numpy()
    ptst = pred_summary.tstat.cpu().numpy()
    assert len(res.problems) == len(ref)
    for k, p in enumerate(res.problems):
        name = model_names[p.model]
        r = ref[(name, p.level)]
        fitted = np.nonzero(st[:, k] & 1)[0]
        assert np.array_equal(fitted, r["month"]), (name, p.level)
        assert np.array_equal(rec[fitted, k, res.pmax + 1].astype(np.int64), r["N"])
        assert_series_close(rec[fitted, k, res.pmax], r["R2"], f"{name} R2")
        for j in range(p.K + 1):
            assert_series_close(rec[fitted, k, j], r["params"][:, j], f"{name}/{p.level} param {j}")
            assert_series_close(roll[k, :len(fitted), j], r["rolling"][:, j], f"{name} roll {j}")
        # rows past the fitted-month count are written (NaN / status 0), never left stale
        assert np.isnan(roll[k, len(fitted):]).all() and (pst[k, len(fitted):] == 0).all(), name
        for j, x in enumerate(model_cols[name]):
            assert scalar_close(mean[k, 1 + j], r["summary"][x][0], RTOL, 1e-12), (name, x)
            assert scalar_close(tstat[k, 1 + j], r["summary"][x][1], RTOL, 1e-12), (name, x)
        pf = np.nonzero(pst[k] & 1)[0]
        assert np.array_equal(fitted[pf], r["pred_month"]), name
        assert_series_close(pred[k, pf, 0], r["pred_slope"], f"{name} pred slope")
        assert_series_close(pred[k, pf, 1], r["pred_R2"], f"{name} pred R2")
        assert scalar_close(pmean[k, 0], r["pred_summary"][0], RTOL, 1e-12)
        assert scalar_close(ptst[k, 0], r["pred_summary"][1], RTOL, 1e-12)


def _pipeline_vs_oracle(E, T, N, seed, model_cols=None, fig1=True, standardize=False, tweak=None):
    from fmcore import lewellen as LW, synth
    model_cols = model_cols or LW.table2_models()
    a = synth.synth_arrays(T, N, seed, nan_rate=0.03, present_rate=0.9)
    if tweak is not None:
        tweak(a)
    cols = list(dict.fromkeys(["retx"] + [c for xs in model_cols.values() for c in xs] +
                              (LW.FIG1_VARS if fig1 else [])))
    panel = E.panel_from_arrays([a[c] for c in cols], cols, a["month"], me=a["me"], nyse=a["nyse"])
    out = LW.run_pipeline(panel, LW.PipelineConfig(fig1=fig1, standardize=standardize), model_cols=model_cols)
    seg_off = panel.seg_off_h
    srt = {c: a[c][panel.order] for c in cols}
    models = {name: ("retx", xs, (0, 1, 2)) for name, xs in model_cols.items()}
    if fig1:
        models["Figure 1"] = ("retx", LW.FIG1_VARS, (0, 2))
    ref = O.pipeline_arrays(srt, seg_off, a["me"][panel.order], a["nyse"][panel.order].astype(bool), models,
                            None, standardize=standardize)
    _compare_with_oracle(out.res, out.model_names, out.model_cols, ref, out.summary, out.rolling, out.pred,
                         out.pred_status, out.pred_summary)
    return out


@pytest.mark.parametrize("fused", [True, False], ids=["ts_fused", "ts_per_stage"])
def test_pipeline_vs_oracle(E, fused, monkeypatch):
    """C3/C4 shape (all Table-2 models x 3 universes + Figure 1), 150 months x 400 firms."""
    if not fused:   # the per-stage kernels that serve series too long for LDS staging
        monkeypatch.setattr(E, "ts_fused_fits", lambda *a, **k: False)
    _pipeline_vs_oracle(E, 150, 400, 99)


def _unfitted_early_months(a):
    """Real Lewellen data has months where a Model-3-only characteristic is missing for
    every firm (log_return_13_36 needs 36 months of history), so those problems fit fewer
    months than the panel has (count < T)."""
    early = a["month"] < a["month"].min() + 17
    a["log_return_13_36"][early] = np.nan
    a["beta"][a["month"] == a["month"].min() + 40] = np.nan


@pytest.mark.parametrize("fused", [True, False], ids=["ts_fused", "ts_per_stage"])
def test_pipeline_unfitted_months(E, fused, monkeypatch):
    """problems with count < T.  The fused and per-stage time-series
    paths must both match the oracle (incl. the predictive NW summary) and write NaN /
    status 0 to every row past the fitted count."""
    if not fused:
        monkeypatch.setattr(E, "ts_fused_fits", lambda *a, **k: False)
    out = _pipeline_vs_oracle(E, 120, 300, 41, tweak=_unfitted_early_months)
    cnt = out.ix.count.cpu().numpy()
    assert (cnt < out.res.status.shape[0]).any()


def test_pipeline_unfitted_months_fused_equals_per_stage(E, monkeypatch):
    from fmcore import lewellen as LW, synth
    a = synth.synth_arrays(100, 250, 43, nan_rate=0.03, present_rate=0.9)
    _unfitted_early_months(a)
    cols = list(dict.fromkeys(["retx"] + [c for xs in LW.table2_models().values() for c in xs] + LW.FIG1_VARS))
    panel = E.panel_from_arrays([a[c] for c in cols], cols, a["month"], me=a["me"], nyse=a["nyse"])
    f = LW.run_pipeline(panel)
    monkeypatch.setattr(E, "ts_fused_fits", lambda *a, **k: False)
    s = LW.run_pipeline(panel)
    # statuses and NaN patterns exact; values to the FP tolerance (the fused kernel slides its
    # window sums, the per-stage one sums every window directly)
    assert np.array_equal(f.pred_status.cpu().numpy(), s.pred_status.cpu().numpy())
    for x, y in ((f.rolling, s.rolling), (f.pred[..., :3], s.pred[..., :3]), (f.summary.mean, s.summary.mean),
                 (f.pred_summary.mean, s.pred_summary.mean), (f.pred_summary.tstat, s.pred_summary.tstat)):
        x, y = x.cpu().numpy(), y.cpu().numpy()
        for k in range(x.shape[0]):
            assert_series_close(x[k].ravel(), y[k].ravel(), f"problem {k}")


def _degenerate_std_months(a):
    """A9 edge months: a predictor constant (exactly representable, so its std is exactly
    0) in one month and present in a single row of another: z is all-NaN there."""
    m0 = a["month"].min()
    a["roa"][a["month"] == m0 + 3] = 0.5
    one = np.nonzero(a["month"] == m0 + 5)[0]
    a["log_bm"][one[1:]] = np.nan


def test_pipeline_standardized_vs_oracle(E):
    """A9 through the whole pass: winsorize -> per-month z-scores of every predictor (the
    Gram's shift / inv_scale path, nothing added back) -> regressions, rolling,
    forecasts; against the oracle's standardize-then-pinv (parity unpinned vs the
    reference, which has no standardization)."""
    _pipeline_vs_oracle(E, 90, 300, 17, standardize=True, tweak=_degenerate_std_months)


def test_standardize_frame_vs_oracle(CL):
    """A9 drop-in: calc_Lewellen_2014.standardize against the oracle's pandas transform."""
    from fmcore import synth
    df = synth.synth_frame(30, 200, 23, nan_rate=0.05, present_rate=0.9)
    df = df.sample(frac=1.0, random_state=1)                # scrambled row order
    months = np.sort(df["mthcaldt"].unique())
    df.loc[df["mthcaldt"] == months[2], "roa"] = 0.25          # zero dispersion -> NaN z
    df.loc[(df["mthcaldt"] == months[4]) & (df["permno"] != df["permno"].min()), "dy"] = np.nan
    vs = ["log_size", "log_bm", "roa", "dy", "retx"]
    got = CL.standardize(df, vs)
    exp = O.standardize(df, vs)
    assert list(got.index) == list(exp.index) and list(got.columns) == list(exp.columns)
    for v in vs:
        assert_series_close(got[v].values, exp[v].values, v)


def test_forecast_api_vs_oracle(CL):
    """A7/A8 per-row API: monthly_coefficients -> rolling_coefficients (host .shift(lag))
    -> expected_return_forecasts (fm_forecast) -> predictive_slope_regressions, against
    the oracle's monthly_params / rolling_coefficients / expected_return_forecasts /
    predictive_slope_regressions (tolerance 1e-9 series RMS, NaN patterns exact)."""
    from fmcore import synth
    df = synth.synth_frame(200, 150, 29, nan_rate=0.03, present_rate=0.9)
    xs = ["log_size", "log_bm", "return_12_2", "roa"]
    pg = CL.monthly_coefficients(df, "retx", xs)
    pe = O.monthly_params(df, "retx", xs)
    assert list(pg.index) == list(pe.index) and list(pg.columns) == list(pe.columns)
    for c in pe.columns:
        assert_series_close(pg[c].values, pe[c].values, "params " + c)
    for lag in (1, 3):
        rg = CL.rolling_coefficients(pe, 120, 60, lag)
        re_ = O.rolling_coefficients(pe, 120, 60, lag)
        assert list(rg.index) == list(re_.index)
        for c in re_.columns:
            assert_series_close(rg[c].values, re_[c].values, f"rolling {c} lag {lag}")
    roll = O.rolling_coefficients(pe, 120, 60, 1)
    fg = CL.expected_return_forecasts(df, roll, xs)
    fe = O.expected_return_forecasts(df, roll, xs)
    assert list(fg.index) == list(fe.index)
    assert_series_close(fg.values, fe.values, "forecast")
    assert np.isfinite(fe.values).sum() > 1000
    csg, sg = CL.predictive_slope_regressions(df, fe)
    cse, se = O.predictive_slope_regressions(df, fe)
    assert np.array_equal(csg["N"].values, cse["N"].values)
    for c in ("R2", "slope_forecast"):
        assert_series_close(csg[c].values, cse[c].values, c)
    for k in se.index:
        assert scalar_close(sg[k], se[k], RTOL, 1e-12), k


def test_rolling_skips_infinite_coefficients(CL):
    """pandas rolling().mean() turns +-inf into NaN (Window._prep_values): an inf-in-y month
    (statsmodels' +-inf params) must not spread through the 120-row window."""
    idx = pd.date_range("1970-01-31", periods=150, freq="ME")
    rng = np.random.default_rng(3)
    p = pd.DataFrame({"const": rng.normal(size=150), "x": rng.normal(size=150)}, index=idx)
    p.iloc[70, 1] = np.inf
    p.iloc[90, 0] = -np.inf
    p.iloc[100, 1] = np.nan
    got = CL.rolling_coefficients(p, 120, 60, 0)
    exp = p.rolling(120, min_periods=60).mean()
    for c in p.columns:
        assert_series_close(got[c].values, exp[c].values, c)
    assert np.isfinite(got.values[75:]).all()


@pytest.mark.parametrize("policy", ["default", "balanced"])
def test_sharded_pipeline_bit_identical(E, policy):
    """SURVEY §8(e) on one GPU: split a ragged panel into 3 month ranges with
    dist.shard_bounds, run local_stage per range with the GLOBAL chunk policy (whole-month
    chunks, or the balanced plan cut in global row space: chunks crossing workgroups
    mid-month), concatenate the records, run time_series_stage per shard (global records,
    local moments, its seg_lo/seg_hi) and SUM the predictive records -- every output must
    equal the unsharded run_pipeline bit for bit (NaN patterns included)."""
    import torch
    from fmcore import dist as D, lewellen as LW, synth
    a = synth.synth_arrays(96, 400, 13, nan_rate=0.03, present_rate=0.6)   # ragged months
    _unfitted_early_months(a)
    cols = list(dict.fromkeys(["retx"] + [c for xs in LW.table2_models().values() for c in xs] + LW.FIG1_VARS))
    panel = E.panel_from_arrays([a[c] for c in cols], cols, a["month"], me=a["me"], nyse=a["nyse"])
    pol = {"default": E.chunk_policy(panel.nrows, panel.nseg, panel.max_seg_len), "balanced": ("balanced", 997)}[policy]
    panel.chunk_policy = pol
    cfg = LW.PipelineConfig()
    mc = LW.table2_models()
    full = LW.run_pipeline(panel, cfg, model_cols=mc)
    off = panel.seg_off_h
    bounds = D.shard_bounds(np.diff(off), 3)
    assert len({e - s for s, e in bounds}) > 1
    locs = []
    for s0, s1 in bounds:
        r0, r1 = int(off[s0]), int(off[s1])
        so = off[s0:s1 + 1] - off[s0]
        sub = E.DevicePanel(cols=panel.cols[:, r0:r1].contiguous(), names=panel.names,
                            seg_off=torch.from_numpy(so).to(panel.cols.device), seg_off_h=so,
                            me=panel.me[r0:r1].contiguous(), nyse=panel.nyse[r0:r1].contiguous(),
                            chunk_policy=pol, row_origin=r0)
        locs.append(LW.local_stage(sub, cfg, mc)[0])
    rec = torch.cat([r.rec for r in locs])
    st = torch.cat([r.status for r in locs])
    assert _same(rec.cpu().numpy(), full.res.rec.cpu().numpy())
    assert np.array_equal(st.cpu().numpy(), full.res.status.cpu().numpy())
    mom = torch.cat([r.moments for r in locs]).cpu().numpy()
    fm_ = full.res.moments.cpu().numpy()
    stf = full.res.status.cpu().numpy()
    for k, p in enumerate(full.res.problems):   # fitted months: the solve writes 1 + K1 + K1^2
        w = 1 + (p.K + 1) + (p.K + 1) ** 2
        fit = (stf[:, k] & 1) != 0
        assert _same(mom[fit, k, :w], fm_[fit, k, :w])
    pred = pst = None
    for (s0, s1), loc in zip(bounds, locs):
        g = E.FMResult(problems=loc.problems, rec=rec, status=st, pmax=loc.pmax, moments=loc.moments,
                       mom_stride=loc.mom_stride)
        ix, summ, roll, p, ps = LW.time_series_stage(g, cfg, moments=loc.moments, seg_lo=s0, seg_hi=s1)
        for x, y in ((summ.mean, full.summary.mean), (summ.tstat, full.summary.tstat), (roll, full.rolling),
                     (ix.count, full.ix.count)):
            assert _same(x.cpu().numpy(), y.cpu().numpy())
        pred = p.clone() if pred is None else pred + p
        pst = ps.clone() if pst is None else pst + ps
    assert np.array_equal(pst.cpu().numpy(), full.pred_status.cpu().numpy())
    keep = (full.pred_status.cpu().numpy() & 1) != 0
    assert _same(pred.cpu().numpy()[keep], full.pred.cpu().numpy()[keep])
    psumm, _ = E.summarize_predictive(pred, pst, cfg.nw_lags)
    assert _same(psumm.mean.cpu().numpy(), full.pred_summary.mean.cpu().numpy())
    assert _same(psumm.tstat.cpu().numpy(), full.pred_summary.tstat.cpu().numpy())


def test_pipeline_c5_month_width(E):
    """C5 month width: 20,000 firms per month (> the wave select's 6,144-row register
    budget, so the cuts take the workgroup select path), 12 months."""
    _pipeline_vs_oracle(E, 12, 20000, 7)


def test_pipeline_c5_rank_shard_full_size(E):
    """C5 at full per-rank size: one of 8 ranks' shards of the 100,000-month x 20,000-firm
    panel (12,500 months x 20,000 firms = 250M rows, 30 GB of FP64 columns in HBM, seed
    20150101, months 50,000..62,499 as rank 4 would generate them) through run_pipeline.
    The 12,500-month series exceeds the fused time-series kernel's LDS staging, so the
    per-stage kernels run.  Checked: (1) four sampled months' monthly records against the
    oracle run on exactly those months (host regeneration of the same counter-hash rows);
    (2) the FM summaries (mean, NW t) and the 120/60 rolling means against the oracle's
    restatement applied to the device's own monthly records (12,500-long series)."""
    import torch
    from fmcore import lewellen as LW
    T, N, seed, m0 = 12500, 20000, 20150101, 50000
    # the layout bench.py's C5 shard uses: the split planes only (no FP64 columns), 30 GB of
    # values for the 250M x 15 panel, 32.25 GB with me / NYSE (round 5 held 60 GB)
    panel = E.panel_synthetic(T, N, seed, month0=m0, layout="planes")
    assert panel.cols is None
    held = sum(t.numel() * t.element_size() for t in (panel.planes, panel.me, panel.nyse, panel.seg_off))
    assert held <= 32.3e9, held
    cfg = LW.PipelineConfig()
    assert not E.ts_fused_fits(T, 16, cfg.window, cfg.lag, predictive=True)
    out = LW.run_pipeline(panel, cfg)
    torch.cuda.synchronize()
    _check_records_vs_oracle(out.res, out.model_names, (0, 1, T // 2, T - 1), N, seed, m0)
    assert ((out.res.status.cpu().numpy() & 1) != 0).all()
    _check_series_vs_restatement(out.res, out.summary, out.rolling, cols=2)
    assert "_merged" not in panel.__dict__   # the pass never materialized FP64 columns


def _check_records_vs_oracle(res, names, months, N, seed, m0=0):
    """Sampled months' monthly records (every problem) against the oracle run on exactly
    those months (host regeneration of the same counter-hash rows)."""
    from fmcore import lewellen as LW, synth
    rec = res.rec.cpu().numpy()
    st = res.status.cpu().numpy()
    models = {name: ("retx", xs, (0, 1, 2)) for name, xs in LW.table2_models().items()}
    models["Figure 1"] = ("retx", LW.FIG1_VARS, (0, 2))
    for t in months:
        a = synth.synth_arrays(1, N, seed, month0=m0 + t)
        cols = {c: a[c] for c in synth.WINSOR_VARS}
        ref = O.pipeline_arrays(cols, np.array([0, N], dtype=np.int64), a["me"], a["nyse"].astype(bool),
                                models, None)
        for k, p in enumerate(res.problems):
            r = ref[(names[p.model], p.level)]
            assert (st[t, k] & 1) != 0 and list(r["month"]) == [0], (t, k)
            assert int(rec[t, k, res.pmax + 1]) == int(r["N"][0])
            b = r["params"][0]
            a_ = rec[t, k, :p.K + 1]
            assert np.all(np.abs(a_ - b) <= RTOL * np.maximum(np.abs(b), np.sqrt(np.mean(b ** 2)))), (t, k)
            assert abs(rec[t, k, res.pmax] - r["R2"][0]) <= RTOL * abs(r["R2"][0])


def _rolling_rows(x, rows, window=120, min_periods=60):
    """oracle.rolling_mean's definition evaluated at the given rows only (long series)."""
    out = np.full(len(rows), np.nan)
    for i, r in enumerate(rows):
        w = x[max(0, r - window + 1):r + 1]
        w = w[np.isfinite(w)]
        if w.size >= min_periods:
            out[i] = w.sum() / w.size
    return out


def _check_series_vs_restatement(res, summ, roll, cols=2, pred=None, pst=None, psumm=None):
    """FM means, NW(4) t-stats and 120/60 rolling means of the device's own monthly records
    against the oracle's restatement (oracle.newey_west_mean_se / rolling_mean); the
    predictive-slope FM summary likewise from the device's predictive records."""
    rec = res.rec.cpu().numpy()
    st = res.status.cpu().numpy()
    mean, tstat, rl = summ.mean.cpu().numpy(), summ.tstat.cpu().numpy(), roll.cpu().numpy()
    for k, p in enumerate(res.problems):
        fit = np.nonzero(st[:, k] & 1)[0]
        for j in range(1, p.K + 1):
            x = rec[fit, k, j]
            m = x.mean()
            assert scalar_close(mean[k, j], m, RTOL, 1e-12), (k, j)
            assert scalar_close(tstat[k, j], m / O.newey_west_mean_se(x, 4), RTOL, 1e-12), (k, j)
        rows = np.unique(np.concatenate([np.arange(min(fit.size, 300)),
                                         np.linspace(0, fit.size - 1, 700).astype(np.int64)]))
        for j in range(cols):
            assert_series_close(rl[k, rows, j], _rolling_rows(rec[fit, k, j], rows), f"roll {k}/{j}")
    if pred is not None:
        pr, ps = pred.cpu().numpy(), pst.cpu().numpy()
        pm, pt = psumm.mean.cpu().numpy(), psumm.tstat.cpu().numpy()
        for k in range(len(res.problems)):
            x = pr[k, (ps[k] & 1) != 0, 0]
            assert x.size > 0
            assert scalar_close(pm[k, 0], x.mean(), RTOL, 1e-12), k
            assert scalar_close(pt[k, 0], x.mean() / O.newey_west_mean_se(x, 4), RTOL, 1e-12), k


def test_pipeline_headline_panel_full_size(E):
    """The bench's own panel (600 months x 5,000 firms x 15 characteristics, seed 1, generated
    in HBM by fm_gen_panel) through the bench's step (ShardedStep, world size 1, eager and
    HIP-graph replay) against oracle.pipeline_arrays on the SAME panel: all 600 months x 11
    problems -- fitted months and N exact; params, R2, rolling means, predictive slopes and
    every FM / predictive summary from the oracle's own records within the tolerance."""
    import torch
    from fmcore import lewellen as LW
    from fmcore.step import ShardedStep
    T, N, seed = 600, 5000, 1
    panel = E.panel_synthetic(T, N, seed)
    cfg = LW.PipelineConfig()
    # the FP64-column pass first, then the bench's split panel (fm_split_planes: the selects on
    # the high-word plane, the Gram on both planes): bit-identical records
    flat, _, _ = ShardedStep(panel, cfg, LW.table2_models()).eager()
    flat_rec = flat.rec.cpu().numpy()
    E.split_planes(panel)
    step = ShardedStep(panel, cfg, LW.table2_models())
    gres, summ, psumm = step.eager()
    assert _same(gres.rec.cpu().numpy(), flat_rec)
    # the panel exactly as bench.py generates it: the planes only (fm_gen_panel_planes)
    pp = E.panel_synthetic(T, N, seed, layout="planes")
    pres, _, ppsumm = ShardedStep(pp, cfg, LW.table2_models()).eager()
    assert _same(pres.rec.cpu().numpy(), flat_rec)
    del pp, pres
    step.capture()
    ggres, gsumm, gpsumm = step.replay()
    torch.cuda.synchronize()
    assert _same(ggres.rec.cpu().numpy(), gres.rec.cpu().numpy())
    assert _same(gpsumm.tstat.cpu().numpy(), psumm.tstat.cpu().numpy())
    names = list(LW.table2_models()) + ["Figure 1"]
    model_cols = dict(LW.table2_models(), **{"Figure 1": LW.FIG1_VARS})
    ix, summ2, roll, pred, pst = LW.time_series_stage(gres, cfg)
    assert _same(summ2.mean.cpu().numpy(), summ.mean.cpu().numpy())
    cols = {name: panel.cols[i].cpu().numpy() for i, name in enumerate(panel.names)}
    models = {name: ("retx", xs, (0, 1, 2)) for name, xs in LW.table2_models().items()}
    models["Figure 1"] = ("retx", LW.FIG1_VARS, (0, 2))
    ref = O.pipeline_arrays(cols, panel.seg_off_h, panel.me.cpu().numpy(),
                            panel.nyse.cpu().numpy().astype(bool), models, None)
    _compare_with_oracle(gres, names, model_cols, ref, summ, roll, pred, pst, psumm)


def test_time_series_stage_gathered_c5_length(E):
    """C5's time-series stage at gathered length: every rank runs it on the full 100,000-month
    series of 11 problems (reference src/regressions.py:78-131, calc_Lewellen_2014.py:926).
    The series = a 12,500-month local pass's records tiled 8 times (what the all-gather of 8
    ranks' records assembles); the predictive slopes for the rank-4 month range use that
    pass's own moments.  Checked: summaries, NW t-stats, rolling means (intercept + first
    slope) and the predictive-slope summary against the oracle's restatement."""
    import torch
    from fmcore import lewellen as LW
    Tl, world, rank = 12500, 8, 4
    panel = E.panel_synthetic(Tl, 200, 77, month0=rank * Tl)
    cfg = LW.PipelineConfig()
    res, _, _, _, _ = LW.local_stage(panel, cfg, LW.table2_models())
    rec = res.rec.repeat(world, 1, 1).contiguous()
    st = res.status.repeat(world, 1).contiguous()
    st[3, :] = 0                       # a few unfitted months in the gathered series
    rec[3, :, :] = float("nan")
    g = E.FMResult(problems=res.problems, rec=rec, status=st, pmax=res.pmax, moments=res.moments,
                   mom_stride=res.mom_stride)
    assert not E.ts_fused_fits(rec.shape[0], res.pmax, cfg.window, cfg.lag, predictive=True)
    ix, summ, roll, pred, pst = LW.time_series_stage(g, cfg, moments=res.moments, seg_lo=rank * Tl,
                                                     seg_hi=(rank + 1) * Tl)
    psumm, _ = E.summarize_predictive(pred, pst, cfg.nw_lags)
    torch.cuda.synchronize()
    assert np.array_equal(ix.count.cpu().numpy(), (st.cpu().numpy() & 1).sum(axis=0))
    _check_series_vs_restatement(g, summ, roll, cols=2, pred=pred, pst=pst, psumm=psumm)
    # predictive rows exist only for the rank's own months (index = fitted-month position)
    ps = pst.cpu().numpy()
    for k in range(len(res.problems)):
        rows = np.nonzero(ps[k] & 1)[0]
        assert rows.min() >= rank * Tl - 1 and rows.max() < (rank + 1) * Tl, k


@pytest.mark.parametrize("path", ["fused", "per_stage"])
def test_sharded_time_series_stage_bit_identical(E, path):
    """The time-series stage split over W month-sharded ranks (ShardedStep, round 6): each rank
    summarizes its problem block (dist.problem_block; -0.0 / 0 for the others), rolls only the
    rows its own months' predictive records read, writes -0.0 records for other ranks' months;
    the SUM of the ranks' outputs (what the RCCL all-reduces return) equals the unsharded stage
    bit for bit, signed zeros included: summaries, predictive records and status, and the
    predictive summaries computed per problem block on the combined records.  Both the fused
    launch (a short gathered series) and the per-stage kernels (a 100,000-month series, C5's
    gathered length) are covered; W = 3 uneven month ranges."""
    import torch
    from fmcore import dist as D
    from fmcore import lewellen as LW
    Tl, tile, W = (200, 4, 3) if path == "fused" else (12500, 8, 3)
    panel = E.panel_synthetic(Tl, 120 if path == "fused" else 200, 31, month0=0)
    cfg = LW.PipelineConfig()
    res, _, _, _, _ = LW.local_stage(panel, cfg, LW.table2_models())
    rec = res.rec.repeat(tile, 1, 1).contiguous()
    st = res.status.repeat(tile, 1).contiguous()
    st[5, :] = 0
    rec[5, :, :] = float("nan")
    T, P = st.shape
    mom = res.moments.repeat(tile, 1, 1).contiguous()
    g = E.FMResult(problems=res.problems, rec=rec, status=st, pmax=res.pmax, moments=mom,
                   mom_stride=res.mom_stride)
    assert E.ts_fused_fits(T, res.pmax, cfg.window, cfg.lag, predictive=True) == (path == "fused")
    ix, summ, roll, pred, pst = LW.time_series_stage(g, cfg, moments=mom, seg_lo=0, seg_hi=T)
    psumm, _ = E.summarize_predictive(pred, pst, cfg.nw_lags)
    bounds = D.shard_bounds(np.full(T, 1), W)
    acc = None
    outs = []
    for r, (s0, s1) in enumerate(bounds):
        blk = D.problem_block(P, W, r)
        _, sm, _, pr, ps = LW.time_series_stage(g, cfg, moments=mom[s0:s1], seg_lo=s0, seg_hi=s1,
                                                sum_range=blk, roll_own=True)
        parts = [pr, ps, sm.mean, sm.se, sm.tstat, sm.nobs]
        acc = [t.clone() for t in parts] if acc is None else [a + t for a, t in zip(acc, parts)]
        outs.append(blk)
    cpred, cpst = acc[0], acc[1]
    pacc = None
    for r in range(W):
        ps_r, _ = E.summarize_predictive(cpred, cpst, cfg.nw_lags, sum_range=outs[r])
        parts = [ps_r.mean, ps_r.se, ps_r.tstat, ps_r.nobs]
        pacc = [t.clone() for t in parts] if pacc is None else [a + t for a, t in zip(pacc, parts)]
    torch.cuda.synchronize()
    full = [pred, pst, summ.mean, summ.se, summ.tstat, summ.nobs]
    names = ["pred", "pst", "mean", "se", "tstat", "nobs"]
    for nm, a, b in zip(names, acc, full):
        assert _same(a.cpu().numpy(), b.cpu().numpy()), nm
    for nm, a, b in zip(["pmean", "pse", "ptstat", "pnobs"], pacc, [psumm.mean, psumm.se, psumm.tstat, psumm.nobs]):
        assert _same(a.cpu().numpy(), b.cpu().numpy()), nm


@pytest.mark.parametrize("cfg", ["C1", "C2"])
def test_pipeline_single_model_configs(E, cfg):
    """C1 (Model 1, K=3) and C2 (Model 2, K=7) alone, 3 universes, no Figure 1."""
    from fmcore import lewellen as LW
    name = {"C1": "Model 1: Three Predictors", "C2": "Model 2: Seven Predictors"}[cfg]
    _pipeline_vs_oracle(E, 80, 600, 11, model_cols={name: LW.table2_models()[name]}, fig1=False)


def test_table1_golden(CL):
    g = load_json("table1.json")
    df = frame_from(load_npz("wins.npz"), "in_")
    subs = CL.get_subsets(CL.winsorize(df, cases.WINSOR_VARS, 1, 99))
    vd = dict(cases.VARIABLES_DICT)
    vd["Missing column"] = "not_a_column"
    t1 = CL.build_table_1(subs, vd)
    assert list(t1.index) == g["index"]
    assert [list(c) for c in t1.columns] == g["columns"]
    assert [str(t) for t in t1.dtypes] == g["dtypes"]
    for r, row in enumerate(g["values"]):
        for c, v in enumerate(row):
            assert scalar_close(t1.values[r, c], v, 1e-12), (g["index"][r], g["columns"][c])


# ---------------------------------------------------------------- firm-axis characteristics
from oracle import chars_oracle as CO  # noqa: E402
from fmtol import beta_inputs, chars_inputs  # noqa: E402

_CHAR_FUNCS = ["calc_log_size", "calc_log_bm", "calc_return_12_2", "calc_accruals", "calc_roa",
               "calc_log_assets_growth", "calc_dy", "calc_log_return_13_36", "calc_log_issues_12",
               "calc_log_issues_36", "calc_debt_price", "calc_sales_price"]


def test_chars_single_golden(CL):
    """Each calc_* on a scrambled frame (groupby order = frame order) vs the reference."""
    g = load_npz("chars.npz")
    m, _ = chars_inputs(g)
    for fn, col in zip(_CHAR_FUNCS, CO.CHARS):
        out = getattr(CL, fn)(m.copy())
        assert np.array_equal(out.index.values, g[f"single_{col}_index"]), fn
        assert list(out.columns) == list(g[f"single_{col}_columns"]), fn
        assert_series_close(out[col].values, g[f"single_{col}"], fn)


def test_chars_chain_golden(CL):
    """get_factors' order (sorted, twelve characteristics, calc_std_12) vs the reference;
    calc_characteristics (one launch) must equal the per-function chain."""
    g = load_npz("chars.npz")
    m, d = chars_inputs(g)
    ms = m.sort_values(["permno", "mthcaldt"])
    ds = d.sort_values(["permno", "dlycaldt"])
    one = CL.calc_characteristics(ms.copy())
    cc = ms.copy()
    for fn in _CHAR_FUNCS:
        cc = getattr(CL, fn)(cc)
    for col in CO.CHARS:
        assert _same(one[col].values, cc[col].values), col
    cc = CL.calc_std_12(ds, cc)
    assert list(cc.columns) == list(g["chain_columns"])
    assert np.array_equal(cc.index.values, g["chain_index"])
    for col in CO.CHARS + ["rolling_std_252"]:
        assert_series_close(cc[col].values, g["chain_" + col], col)


def test_std_12_scrambled_golden(CL):
    g = load_npz("chars.npz")
    m, d = chars_inputs(g)
    out = CL.calc_std_12(d.copy(), m.copy())
    assert np.array_equal(out["permno"].values, g["std_permno"])
    assert_series_close(out["rolling_std_252"].values, g["std_rolling_std_252"], "std_12")


def _ragged_firm_panel(rng, nfirms, maxlen):
    lens = rng.integers(1, maxlen + 1, nfirms)
    lens[::5] = maxlen
    ids = np.repeat(np.arange(nfirms, dtype=np.int64) * 3 + 10, lens)
    n = len(ids)
    f = {k: rng.standard_t(4, n) * 0.1 + (1.0 if k not in ("retx", "accruals", "earnings") else 0.0)
         for k in CO.FIELDS}
    for k in ("me", "be", "assets", "shrout", "prc", "total_debt", "sales"):
        f[k] = np.exp(rng.normal(3, 1, n))
    for k in CO.FIELDS:
        f[k][rng.random(n) < 0.02] = np.nan
    return ids, f


def test_firm_chars_vs_oracle_many_tiles(E):
    """Ragged firms across many 256-row tiles (halo reads across tile and firm edges)."""
    import torch
    rng = np.random.default_rng(31)
    ids, f = _ragged_firm_panel(rng, 900, 130)
    exp = CO.firm_chars(ids, f)
    got = E.firm_chars(torch.from_numpy(ids).cuda(), {k: torch.from_numpy(v).cuda() for k, v in f.items()})
    for col in CO.CHARS:
        assert_series_close(got[col].cpu().numpy(), exp[col], col)
    # a subset of characteristics reads only its fields
    sub = E.firm_chars(torch.from_numpy(ids).cuda(), {"me": torch.from_numpy(f["me"]).cuda()},
                       names=("log_size",))
    assert _same(sub["log_size"].cpu().numpy(), got["log_size"].cpu().numpy())
    with pytest.raises(Exception):
        E.firm_chars(torch.from_numpy(ids).cuda(), {"me": torch.from_numpy(f["me"]).cuda()},
                     names=("log_bm",))


@pytest.mark.parametrize("window,minp", [(252, 100), (5, 3), (1, 1), (3000, 2), (4096, 50), (17, 17)])
def test_rolling_std_vs_oracle(E, window, minp):
    """Ragged firms (1..3999 rows) crossing the kernel's 2,048-row tiles; firm ids differ only
    above bit 32 (the firm-start test compares full int64 ids); window sizes from 1 to the
    4,096 maximum."""
    import torch
    rng = np.random.default_rng(window)
    lens = rng.integers(1, 4000, 40)
    ids = np.repeat(np.arange(40, dtype=np.int64) << 33, lens)
    x = rng.normal(0, 0.02, len(ids))
    x[rng.random(len(ids)) < 0.05] = np.nan
    x[rng.random(len(ids)) < 0.002] = np.inf
    x[1000:1300] = 0.01                       # a run of equal values -> exact 0
    exp = CO.rolling_std(ids, x, window, minp, 1.0)
    got = E.rolling_std(torch.from_numpy(ids).cuda(), torch.from_numpy(x).cuda(), window, minp, 1.0)
    assert_series_close(got.cpu().numpy(), exp, f"rolling_std w={window}")


def test_chars_empty_and_single_row(E):
    import torch
    for n in (0, 1):
        ids = torch.arange(n, dtype=torch.int64, device="cuda")
        flds = {k: torch.ones(n, dtype=torch.float64, device="cuda") for k in CO.FIELDS}
        out = E.firm_chars(ids, flds)
        assert all(v.shape == (n,) for v in out.values())
        sd = E.rolling_std(ids, flds["retx"], 252, 100)
        assert sd.shape == (n,) and (n == 0 or torch.isnan(sd).all())


def test_firm_chars_full_size_firm_locality(E):
    """Bench-size firm-major panel (5,000 firms x 600 months): a firm's characteristics depend
    on its own rows only, so the device result on the whole panel must equal the oracle run on
    a sample of firms alone."""
    import torch
    from fmcore import synth_chars
    ids_d, flds_d = synth_chars.device_raw_panel(5000, 600, seed=5)
    got = E.firm_chars(ids_d, flds_d)
    ids = ids_d.cpu().numpy()
    pick = np.isin(ids, ids[np.random.default_rng(0).choice(len(ids), 40)])
    exp = CO.firm_chars(ids[pick], {k: v.cpu().numpy()[pick] for k, v in flds_d.items()})
    for col in CO.CHARS:
        assert_series_close(got[col].cpu().numpy()[pick], exp[col], col)


def test_panel_from_arrow_matches_frame_path(E):
    """§8(f) row 3: the Arrow ingest (pinned single copy, device month-major gather) builds a
    DevicePanel bit-identical to panel_from_arrays on the same DataFrame columns."""
    import pyarrow as pa
    from fmcore import ingest
    rng = np.random.default_rng(8)
    n = 20000
    months = pd.date_range("1964-01-31", periods=40, freq="ME")
    df = pd.DataFrame({"mthcaldt": rng.choice(months, n), "retx": rng.normal(1, 10, n),
                       "x1": rng.normal(0, 1, n), "me": np.exp(rng.normal(5, 2, n)),
                       "primaryexch": rng.choice(["N", "Q"], n)})
    df.loc[rng.random(n) < 0.05, "x1"] = np.nan
    tab = pa.Table.from_pandas(df, preserve_index=False)
    got = ingest.panel_from_arrow(tab, ["retx", "x1"], me_col="me", exch_col="primaryexch")
    exp = E.panel_from_arrays([df["retx"].to_numpy(), df["x1"].to_numpy()], ["retx", "x1"],
                              df["mthcaldt"].values, me=df["me"].to_numpy(),
                              nyse=(df["primaryexch"] == "N").to_numpy().astype(np.uint8))
    assert _same(got.cols.cpu().numpy(), exp.cols.cpu().numpy())
    assert np.array_equal(got.seg_off_h, exp.seg_off_h)
    assert _same(got.me.cpu().numpy(), exp.me.cpu().numpy())
    assert np.array_equal(got.nyse.cpu().numpy(), exp.nyse.cpu().numpy())
    a1, b1 = E.nyse_breakpoints(got)
    a2, b2 = E.nyse_breakpoints(exp)
    assert _same(a1.cpu().numpy(), a2.cpu().numpy()) and _same(b1.cpu().numpy(), b2.cpu().numpy())


def test_rolling_beta_vs_oracle(CL):
    """§8(f) row 2's 156-week rolling beta (calculate_rolling_beta, reference :344-434) on
    device against the oracle's restatement of polars group_by_dynamic (parity UNPINNED vs
    the reference: polars is not installed).  Ragged firms, a > 3-year gap (empty windows),
    NaN and -100% returns, missing market days, a permno without daily data."""
    crsp_d, idx, comp = beta_inputs()
    got = CL.calculate_rolling_beta(crsp_d, idx, comp)
    exp = CO.calculate_rolling_beta(crsp_d, idx, comp)
    assert list(got.columns) == list(exp.columns) and len(got) == len(exp)
    assert np.array_equal(got["permno"].values, exp["permno"].values)
    assert np.isfinite(exp["beta"].values).sum() > 500
    assert_series_close(got["beta"].values, exp["beta"].values, "beta")


# ---------------------------------------------------------------- §8(f) row 3: panel ETL
def _etl_frame_equal(got, g):
    assert list(got.columns) == [str(c) for c in g["out_columns"]]
    for c in got.columns:
        a = got[c].to_numpy()
        if c == "gvkey":
            a = a.astype(np.int64)
        elif np.issubdtype(got[c].dtype, np.datetime64):
            a = got[c].to_numpy(dtype="datetime64[ns]").astype(np.int64)
        b = g["out_" + c] if isinstance(g, dict) or hasattr(g, "files") else g[c]
        assert np.array_equal(a, b, equal_nan=a.dtype.kind == "f"), c


def test_expand_compustat_golden():
    """Drop-in expand_compustat_annual_to_monthly (fm_ffill_expand) against the reference's
    own output (tests/golden/etl.npz): 40 gvkeys, 1..12 annual records with multi-year gaps,
    the 12-month extension clipped at the table's last report date, one group with
    mid-month report dates, NaN values, an int column -- every column exact."""
    import etl_cases
    from fmdrop import transform_compustat as TC
    got = TC.expand_compustat_annual_to_monthly(etl_cases.comp_annual())
    _etl_frame_equal(got, load_npz("etl.npz"))


def test_expand_compustat_vs_oracle_large():
    """3,000 gvkeys x up to 30 annual records (shuffled), device vs the oracle restatement,
    exact; duplicated (gvkey, report_date) labels raise like the reference's reindex."""
    from fmdrop import transform_compustat as TC
    from oracle import etl_oracle as X
    rng = np.random.default_rng(17)
    rows = []
    for k in range(3000):
        n = int(rng.integers(1, 31))
        yrs = np.sort(rng.choice(np.arange(1950, 2020), size=n, replace=False))
        fye = int(rng.integers(1, 13))
        dd = pd.to_datetime({"year": yrs, "month": np.full(n, fye), "day": np.ones(n, int)}) + pd.offsets.MonthEnd(0)
        rows.append(pd.DataFrame({"gvkey": f"{k:06d}", "datadate": dd, "fyear": yrs,
                                  "report_date": dd + pd.offsets.MonthEnd(4),
                                  "be": rng.standard_normal(n), "at": rng.standard_normal(n)}))
    df = pd.concat(rows, ignore_index=True)
    df = df.iloc[rng.permutation(len(df))].reset_index(drop=True)
    got = TC.expand_compustat_annual_to_monthly(df)
    exp = X.expand_compustat_annual_to_monthly(df)
    assert list(got.columns) == list(exp.columns) and len(got) == len(exp)
    for c in got.columns:
        assert np.array_equal(got[c].to_numpy(), exp[c].to_numpy()), c
    with pytest.raises(ValueError):
        TC.expand_compustat_annual_to_monthly(pd.concat([df, df.iloc[:1]], ignore_index=True))


def test_merge_crsp_compustat_golden():
    """Drop-in merge_CRSP_and_Compustat (device joins, fm_sorted_join) against the
    reference's own output (tests/golden/etl_merge.npz): one- and two-link gvkeys, open-ended
    links, an unlinked gvkey, a permno linked to two gvkeys, _x / _y suffixes -- columns,
    dtypes and every value in order; the caller's ccm gets its NaT linkenddt filled, as the
    reference does."""
    import etl_cases
    from fmdrop import transform_compustat as TC
    g = load_npz("etl_merge.npz")
    comp = TC.expand_compustat_annual_to_monthly(etl_cases.comp_annual())
    crsp = etl_cases.frame_from_golden(g, "crsp_", {"jdate", "datadate"})
    ccm = etl_cases.frame_from_golden(g, "ccm_", {"linkdt", "linkenddt"})
    out = TC.merge_CRSP_and_Compustat(crsp, comp, ccm)
    assert not ccm["linkenddt"].isna().any()
    assert list(out.columns) == [str(c) for c in g["out_columns"]]
    assert [str(t) for t in out.dtypes] == [str(t) for t in g["out_dtypes"]]
    for c in out.columns:
        a = out[c].to_numpy()
        if c == "gvkey":
            a = a.astype(np.int64)
        elif np.issubdtype(out[c].dtype, np.datetime64):
            a = out[c].to_numpy(dtype="datetime64[ns]").astype(np.int64)
        assert np.array_equal(a, g["out_" + c], equal_nan=a.dtype.kind == "f"), c


def test_expand_compustat_units_and_missing_ids():
    """[us] / [s] report dates and missing gvkeys against the reference's own output
    (etl_units.npz): the 12-month clip is computed in one unit, fund_date is
    datetime64[ns] as the reference's date_range gives, missing ids are dropped as groupby
    does; a NaT report date raises ValueError like the reference's reindex."""
    import etl_cases
    from fmdrop import transform_compustat as TC
    g = load_npz("etl_units.npz")
    base = etl_cases.comp_annual()
    for name, frame in etl_cases.unit_variants(base).items():
        etl_cases.assert_frame_matches(TC.expand_compustat_annual_to_monthly(frame), g, name + "_")
    bad = base.copy()
    bad.loc[3, "report_date"] = pd.NaT
    with pytest.raises(ValueError):
        TC.expand_compustat_annual_to_monthly(bad)


@pytest.mark.parametrize("fused", [True, False], ids=["ts_fused", "ts_per_stage"])
def test_rolling_mean_outlier_months(E, fused):
    """the rolling means slide (per-stage kernel) or difference prefix sums
    (fused kernel).  A coefficient series with huge outliers (a near-singular month's slope)
    must leave nothing behind once they leave the 120-row window: every window against its
    exactly rounded mean (math.fsum), tolerance 1e-9 of the ordinary windows' scale."""
    import math

    import torch
    T, K1, W, MP = 600, 3, 120, 60
    rng = np.random.default_rng(5)
    x = rng.standard_normal((T, K1))
    x[200, 1] = 1e12
    x[333, 2] = -3e11
    x[334, 2] = 7e10
    x[400, 0] = np.inf        # pandas rolling skips +-inf (Window._prep_values)
    rs = K1 + 2
    rec = np.zeros((T, 1, rs))
    rec[:, 0, :K1] = x
    dev = torch.device("cuda", 0)
    rec_t = torch.from_numpy(rec).to(dev)
    st_t = torch.ones((T, 1), dtype=torch.int32, device=dev)
    res = E.FMResult(problems=[E.Problem(0, 0, K1 - 1)], rec=rec_t, status=st_t, pmax=K1)
    if fused:
        assert E.ts_fused_fits(T, K1, W)
        _, _, roll, _, _ = E.ts_fused(rec_t, rs, rs, st_t, 1, 1, T, 1, rs, 4, window=W, min_periods=MP, pmax=K1)
    else:
        roll = E.rolling_result(res, E.compact_result(res), W, MP)
    got = roll.cpu().numpy()[0]
    for k in range(K1):
        exp = np.full(T, np.nan)
        big = np.zeros(T, dtype=bool)
        for i in range(T):
            w = x[max(0, i - W + 1):i + 1, k]
            w = w[np.isfinite(w)]
            if w.size >= MP:
                exp[i] = math.fsum(w) / w.size
                big[i] = np.abs(w).max() > 1e6
        assert np.array_equal(np.isnan(got[:, k]), np.isnan(exp)), k
        ok = ~np.isnan(exp)
        scale = np.sqrt(np.mean(exp[ok & ~big] ** 2))
        tol = RTOL * np.maximum(np.abs(exp), scale)
        bad = np.flatnonzero(ok & ~(np.abs(got[:, k] - exp) <= tol))
        assert bad.size == 0, (k, bad[:5], got[bad[:5], k], exp[bad[:5]])


def test_split_month_gram_plan_matches_whole(E):
    """The split-month Gram plan (each month as a 3/4 + 1/4 chunk pair, big chunks launched
    first) and the balanced plan (workgroups of equal row counts cut at month boundaries,
    workgroups spanning two months) against whole-month chunks on the same 600-month panel:
    identical month lists, N and status; params and R2 within 1e-12 of the series scale (only
    the summation order differs)."""
    from fmcore import lewellen as LW
    panel = E.panel_synthetic(600, 1200, 5)
    out = {}
    for plan in ("months", "split", "balanced"):
        panel.chunk_split = plan == "split"
        panel.chunk_policy = {"months": ("months", 1200), "split": None, "balanced": ("balanced", 937)}[plan]
        panel.__dict__.pop("_chunk_cache", None)
        res = LW.local_stage(panel, LW.PipelineConfig(), LW.table2_models())[0]
        out[plan] = (res.rec.cpu().numpy(), res.status.cpu().numpy())
        if plan == "balanced":
            pl = E._chunk_plan(panel)
            assert pl.nwg == -(-600 * 1200 // 937) and pl.nchunks > pl.nwg
    ra, sa = out["months"]
    for plan in ("split", "balanced"):
        rb, sb = out[plan]
        assert np.array_equal(sa, sb)
        assert _same(ra[..., -1], rb[..., -1])   # N
        for k in range(ra.shape[1]):
            for j in range(ra.shape[2] - 1):
                assert_series_close(rb[:, k, j], ra[:, k, j], f"{plan} problem {k} col {j}", rtol=1e-12)


# ---------------------------------------------------------------- planes-only panels (round 6)
def _pipe_host(out):
    d = {"rec": out.res.rec, "status": out.res.status, "mean": out.summary.mean, "se": out.summary.se,
         "t": out.summary.tstat, "nobs": out.summary.nobs, "lo": out.cuts.lo, "hi": out.cuts.hi,
         "nvalid": out.cuts.nvalid, "center": out.cuts.center, "level": out.level,
         "bp_a": out.breakpoints[0], "bp_b": out.breakpoints[1], "pred": out.pred, "pst": out.pred_status,
         "pmean": out.pred_summary.mean, "ptstat": out.pred_summary.tstat}
    return {k: v.cpu().numpy() for k, v in d.items()}


@pytest.mark.parametrize("shape", [(60, 5000), (12, 20000)])
def test_planes_only_panel_pipeline_bit_identical(E, shape):
    """A panel generated straight into the split layout (fm_gen_panel_planes: high / low
    32-bit planes, NO FP64 columns) gives the Table-2 / Figure-1 pass of the FP64 panel bit
    for bit: cuts (signs of the dy column's exactly-zero 1% cuts included: their replay reads
    the planes), universes, records, status, summaries, predictive records.  Short months (the
    two-wave select) and C5-length 20,000-row months (the long-month high-key kernel, whose
    candidate gathers read the planes)."""
    from fmcore import lewellen as LW
    T, N = shape
    pa = E.panel_synthetic(T, N, 9, layout="f64")
    pb = E.panel_synthetic(T, N, 9, layout="planes")
    assert pb.cols is None and pb.planes is not None
    cfg = LW.PipelineConfig()
    a = _pipe_host(LW.run_pipeline(pa, cfg))
    b = _pipe_host(LW.run_pipeline(pb, cfg))
    assert pb.cols is None and "_merged" not in pb.__dict__   # the pass never asked for FP64 columns
    for k in a:
        if a[k].dtype.kind == "f":
            assert _same(b[k], a[k]), k
        else:
            assert np.array_equal(b[k], a[k]), k
    # the generator's planes are the FP64 values' words
    ha = pa.cols.cpu().numpy().view(np.uint64)
    hb = (pb.planes[0].cpu().numpy().astype(np.uint32).astype(np.uint64) << np.uint64(32)) | \
        pb.planes[1].cpu().numpy().astype(np.uint32).astype(np.uint64)
    assert np.array_equal(ha, hb)


def test_planes_only_panel_fixup_paths(E):
    """The rare select / solve paths on a planes-only panel read values through the planes:
    pct.npz (+-inf, NaN runs, ties, signed zeros: units marked for the workgroup fix-up and
    zero-cut sign replays) from panel_from_arrays(layout="planes") gives the FP64 panel's cuts
    bit for bit; a near-collinear model (x2 = x1 + 1e-8 noise: FM_ST_REFIT months re-solved
    from the rows by the solve's inline QR + SVD refit) the same records and status."""
    g = load_npz("pct.npz")
    vals, off, qs = g["values"], g["offsets"], g["qs"]
    labels = np.repeat(np.arange(len(off) - 1), np.diff(off))
    pf = E.panel_from_arrays([vals], ["v"], labels)
    pp = E.panel_from_arrays([vals], ["v"], labels, layout="planes")
    assert pp.cols is None
    for a, b in [(0, 1), (2, 3), (4, 5), (6, 6)]:
        cf = E.select_cuts(pf, qs[a] / 100, qs[b] / 100, 1, E.LERP_NUMPY, center=True)
        cp = E.select_cuts(pp, qs[a] / 100, qs[b] / 100, 1, E.LERP_NUMPY, center=True)
        for f in ("lo", "hi", "center"):
            assert _same(getattr(cp, f).cpu().numpy(), getattr(cf, f).cpu().numpy()), (qs[a], f)
        assert np.array_equal(cp.nvalid.cpu().numpy(), cf.nvalid.cpu().numpy())
    df = cases._edge_base(8, 300, 4, 77)
    rng = np.random.default_rng(78)
    df["x2"] = df["x1"] + 1e-8 * rng.standard_normal(len(df))
    names = ["retx", "x0", "x1", "x2", "x3"]
    labels = df["mthcaldt"].values
    out = {}
    for layout in ("f64", "planes"):
        p = E.panel_from_arrays([df[c].values for c in names], names, labels, layout=layout)
        m = E.Model("m", y=0, xs=[1, 2, 3, 4])
        cuts = E.select_cuts(p, 0.01, 0.99, 5, E.LERP_NUMPY, center=True)
        res = E.fm_pass(p, [m], cuts=cuts, shift=cuts.center, moments=True)
        out[layout] = (res.rec.cpu().numpy(), res.status.cpu().numpy())
    st = out["f64"][1]
    assert ((st & E.L.FM_ST_REFIT) != 0).any(), "the case must take the refit path"
    assert _same(out["planes"][0], out["f64"][0]) and np.array_equal(out["planes"][1], st)


def test_planes_stale_after_in_place_write_refused(E):
    """A panel holding both layouts refuses to run once its FP64 columns were written in
    place after the planes were made (the planes would be stale); split_planes re-arms it."""
    p = E.panel_synthetic(4, 300, 2, layout="both")
    E.select_cuts(p, 0.01, 0.99, 5, E.LERP_NUMPY)
    p.cols[0, 0] = 1.0
    with pytest.raises(RuntimeError, match="modified in place"):
        E.select_cuts(p, 0.01, 0.99, 5, E.LERP_NUMPY)
    E.split_planes(p)
    E.select_cuts(p, 0.01, 0.99, 5, E.LERP_NUMPY)


def test_stream_probes_read_and_copy(E):
    """bench.py's measured read / copy peaks come from fm_stream_probe / fm_stream_copy_probe:
    the read probe sums every element (odd tail included), the copy probe copies them."""
    import torch
    for n in (1, 7, 4096 * 1024 + 3):
        src = torch.arange(n, dtype=torch.float64, device="cuda") * 0.5 - 3.0
        s = E.stream_probe(src)
        assert abs(float(s.item()) - float(src.sum().item())) <= 1e-9 * max(1.0, float(src.abs().sum().item()))
        dst = torch.full_like(src, float("nan"))
        E.stream_copy_probe(src, dst)
        assert torch.equal(dst, src)


@pytest.mark.parametrize("layout", ["f64", "planes"])
def test_long_month_tails_crowded_into_one_wave(E, layout):
    """The long-month kernel writes each wave's tail candidates into a 64-entry list of its
    own; a wave holding more than that sends the unit to the counted compaction.  Rows
    r with (r mod 2,048) < 256 are one wave's (16-byte slots: four rows per lane, 512 lanes);
    here every tail value of a month sits in them (and in another month in the last wave's
    rows), so the fallback runs -- bit-exact against np.percentile either way."""
    rng = np.random.default_rng(11)
    n = 20000
    rows = np.arange(n)
    segs = []
    for lo_w, hi_w in ((0, 0), (7, 7), (0, 7), (3, 3)):
        x = rng.standard_normal(n)
        order = np.argsort(x)
        k = 400                                      # > 64 per tail, 1 % ranks at ~200
        low_rows = rows[(rows % 2048) // 256 == lo_w]
        high_rows = rows[(rows % 2048) // 256 == hi_w]
        xs = x[order]
        y = np.empty(n)
        taken = np.zeros(n, dtype=bool)
        sel_lo = rng.choice(low_rows, k, replace=False)
        y[sel_lo] = xs[:k]
        taken[sel_lo] = True
        free_hi = high_rows[~taken[high_rows]]
        sel_hi = rng.choice(free_hi, k, replace=False)
        y[sel_hi] = xs[-k:]
        taken[sel_hi] = True
        rest = rows[~taken]
        y[rest] = rng.permutation(xs[k:n - k])
        segs.append(y)
    segs.append(rng.standard_normal(n))               # an ordinary month beside them
    vals = np.concatenate(segs)
    labels = np.repeat(np.arange(len(segs)), [len(s) for s in segs])
    panel = E.panel_from_arrays([vals], ["v"], labels, layout=layout)
    assert panel.max_seg_len == n
    for qa, qb in ((1, 99), (2, 98)):
        cuts = E.select_cuts(panel, qa / 100, qb / 100, 1, E.LERP_NUMPY, center=True)
        lo, hi = cuts.lo.cpu().numpy()[0], cuts.hi.cpu().numpy()[0]
        for t, s in enumerate(segs):
            ra, rb = np.percentile(s, qa), np.percentile(s, qb)
            assert _same([lo[t]], [ra]) and _same([hi[t]], [rb]), (layout, qa, t, lo[t], ra, hi[t], rb)

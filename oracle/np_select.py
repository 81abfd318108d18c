"""CPU ORACLE — test infrastructure only, never the product path.

numpy 1.26.4's `ndarray.partition` restated, to pin the SIGN of an exactly-zero winsorize
cut.  `np.percentile(vals, q)` (reference src/calc_Lewellen_2014.py:522-523, numpy
function_base._quantile) partitions a copy of `vals` (frame order: the month's non-NaN rows
after `sort_values(["mthcaldt","permno"])`, :514/:519) at kth = unique([0, -1, i, i+1]),
then reads arr[i], arr[i+1].  -0.0 and +0.0 compare equal, so WHICH signed zero lands at
position i is decided by the partition's swap order alone -- and it decides the sign of a
zero cut (and of every value clipped to it).

numpy (npysort/selection.cpp, item_selection.c `partition_prep_kth_array` /
`_new_sortlike`): the kth list is made non-negative (+n) and sorted, then introselect runs
once per kth IN ORDER over the whole array with one shared stack of pivots (<= 50):

* pop pivots <= kth to raise `low`; a pivot > kth caps `high`; a pivot == kth -> done;
* kth - low < 3: selection sort of positions low..kth over [low, high] (strict <, first
  minimum wins), push kth;
* else median-of-3 quickselect (median3_swap: mid = low + (high-low)/2; pivot to low, the
  smallest of the three to low+1) with an unguarded Hoare partition
  (`do ++ll while v[ll] < p; do --hh while p < v[hh]; swap unless crossed`), the pivot
  swapped into hh, hh pushed when != kth; depth limit 2*msb(n) then median-of-medians-of-5.

`tests/test_oracle_golden.py::test_np_partition_restatement_matches_numpy` pins this against
numpy 1.26.4 itself (the reference's pin) on adversarial tie-heavy arrays, and pct.npz's
zero cuts' signs against the reference's np.percentile.
"""
from __future__ import annotations

import numpy as np

MAX_PIVOT_STACK = 50


def _less(a, b):
    # npy::double_tag::less: a < b || (b != b && a == a)  (NaN last; no NaN reaches here)
    return a < b or (b != b and a == a)


def _msb(n):
    d = 0
    n >>= 1
    while n:
        d += 1
        n >>= 1
    return d


def _store_pivot(pivot, kth, piv):
    if pivot == kth and len(piv) == MAX_PIVOT_STACK:
        piv[-1] = pivot
    elif pivot >= kth and len(piv) < MAX_PIVOT_STACK:
        piv.append(pivot)


def _dumb_select(v, o, num, kth):
    """selection sort of v[o : o+kth+1] over v[o : o+num]"""
    for i in range(kth + 1):
        mi, mv = i, v[o + i]
        for k in range(i + 1, num):
            if _less(v[o + k], mv):
                mi, mv = k, v[o + k]
        v[o + i], v[o + mi] = v[o + mi], v[o + i]


def _median5(v, o):
    def sw(i, j):
        v[o + i], v[o + j] = v[o + j], v[o + i]
    if _less(v[o + 1], v[o + 0]):
        sw(1, 0)
    if _less(v[o + 4], v[o + 3]):
        sw(4, 3)
    if _less(v[o + 3], v[o + 0]):
        sw(3, 0)
    if _less(v[o + 4], v[o + 1]):
        sw(4, 1)
    if _less(v[o + 2], v[o + 1]):
        sw(2, 1)
    if _less(v[o + 3], v[o + 2]):
        return 1 if _less(v[o + 3], v[o + 1]) else 3
    return 2


def _median_of_median5(v, o, num):
    right = num - 1
    nmed = (right + 1) // 5
    subleft = 0
    for i in range(nmed):
        m = _median5(v, o + subleft)
        v[o + subleft + m], v[o + i] = v[o + i], v[o + subleft + m]
        subleft += 5
    if nmed > 2:
        _introselect(v, o, nmed, nmed // 2, None)
    return nmed // 2


def _introselect(v, o, num, kth, piv):
    """numpy introselect_<double_tag, false> on v[o : o+num] (piv None = no pivot stack)."""
    low, high = 0, num - 1
    while piv is not None and piv:
        if piv[-1] > kth:
            high = piv[-1] - 1
            break
        if piv[-1] == kth:
            return
        low = piv[-1] + 1
        piv.pop()
    if kth - low < 3:
        _dumb_select(v, o + low, high - low + 1, kth - low)
        if piv is not None:
            _store_pivot(kth, kth, piv)
        return
    if kth == num - 1:
        # inexact types: one max scan (>=: the LAST maximum wins), swapped to kth; no pivot
        mi, mv = low, v[o + low]
        for k in range(low + 1, num):
            if not _less(v[o + k], mv):
                mi, mv = k, v[o + k]
        v[o + kth], v[o + mi] = v[o + mi], v[o + kth]
        return
    depth = _msb(num) * 2
    while low + 1 < high:
        ll, hh = low + 1, high
        if depth > 0 or hh - ll < 5:
            mid = low + (high - low) // 2
            # median3_swap
            if _less(v[o + high], v[o + mid]):
                v[o + high], v[o + mid] = v[o + mid], v[o + high]
            if _less(v[o + high], v[o + low]):
                v[o + high], v[o + low] = v[o + low], v[o + high]
            if _less(v[o + low], v[o + mid]):
                v[o + low], v[o + mid] = v[o + mid], v[o + low]
            v[o + mid], v[o + low + 1] = v[o + low + 1], v[o + mid]
        else:
            mid = ll + _median_of_median5(v, o + ll, hh - ll)
            v[o + mid], v[o + low] = v[o + low], v[o + mid]
            ll -= 1
            hh += 1
        depth -= 1
        p = v[o + low]
        while True:       # unguarded_partition
            ll += 1
            while _less(v[o + ll], p):
                ll += 1
            hh -= 1
            while _less(p, v[o + hh]):
                hh -= 1
            if hh < ll:
                break
            v[o + ll], v[o + hh] = v[o + hh], v[o + ll]
        v[o + low], v[o + hh] = v[o + hh], v[o + low]
        if hh != kth and piv is not None:
            _store_pivot(hh, kth, piv)
        if hh >= kth:
            high = hh - 1
        if hh <= kth:
            low = ll
    if high == low + 1 and _less(v[o + high], v[o + low]):
        v[o + high], v[o + low] = v[o + low], v[o + high]
    if piv is not None:
        _store_pivot(kth, kth, piv)


def partition(vals, kth):
    """`np.asarray(vals).copy().partition(kth)` for a 1-d float64 array, restated."""
    v = [float(x) for x in np.asarray(vals, dtype=np.float64)]
    n = len(v)
    ks = sorted(int(k) + n if int(k) < 0 else int(k) for k in np.atleast_1d(kth))
    piv = []
    for k in ks:
        _introselect(v, 0, n, k, piv)
    return np.array(v, dtype=np.float64)


def percentile_pair(vals, i):
    """arr[i], arr[i+1] (or arr[-1] twice) after np.percentile's partition of `vals`."""
    n = len(vals)
    if i < 0:
        arr = partition(vals, [0, -1])
        return arr[n - 1], arr[n - 1]
    arr = partition(vals, np.unique([0, -1, i, i + 1]))
    return arr[i], arr[i + 1]

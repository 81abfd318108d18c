"""CPU check of the device replay's batched Hoare partition (fm_npsel_dev.h np_hoare).

The device replays numpy's unguarded Hoare partition 64 positions at a time: the stoppers of
a 64-position window on each side are paired in order and every pair with L < R is swapped
at once; the first pair with L >= R ends the batch and the next round rescans from the last
swapped pair.  This test restates that batched loop in Python (lane for lane) and checks it
against the sequential partition of oracle/np_select.py (itself pinned to numpy 1.26.4) on
tie-heavy and adversarial arrays: same final array bit for bit and the same (ll, hh)."""
import numpy as np

from oracle import np_select as S

WAVE = 64


def _less(a, b):
    return S._less(a, b)


def hoare_sequential(v, low, high, pv, mom5=False):
    ll, hh = (low, high + 1) if mom5 else (low + 1, high)
    while True:
        ll += 1
        while _less(v[ll], pv):
            ll += 1
        hh -= 1
        while _less(pv, v[hh]):
            hh -= 1
        if hh < ll:
            break
        v[ll], v[hh] = v[hh], v[ll]
    return ll, hh


def hoare_batched(v, n, pv, ll, hh):
    """np_hoare, lane for lane (the ballots as lists)."""
    it = 0
    while True:
        it += 1
        assert it < 10 * n + 100, "no progress"
        ml = [ll + 1 + l < n and not _less(v[min(ll + 1 + l, n - 1)], pv) for l in range(WAVE)]
        mr = [hh - 1 - l >= 0 and not _less(pv, v[max(hh - 1 - l, 0)]) for l in range(WAVE)]
        Ls = [ll + 1 + l for l in range(WAVE) if ml[l]]
        Rs = [hh - 1 - l for l in range(WAVE) if mr[l]]
        if not Ls or not Rs:
            if not Ls:
                ll += WAVE
            if not Rs:
                hh -= WAVE
            continue
        m = min(len(Ls), len(Rs))
        P = 0
        while P < m and Ls[P] < Rs[P]:
            P += 1
        if P == 0:
            ll, hh = Ls[0], Rs[0]
            if ll > hh:
                return ll, hh
            continue
        old = [(v[Ls[j]], v[Rs[j]]) for j in range(P)]   # every lane loads, then stores
        for j in range(P):
            v[Ls[j]], v[Rs[j]] = old[j][1], old[j][0]
        ll, hh = Ls[P - 1], Rs[P - 1]


def _cases(rng):
    for trial in range(600):
        n = int(rng.choice([8, 16, 33, 64, 65, 100, 257, 1000, 3000]))
        kind = trial % 5
        if kind == 0:
            x = rng.choice([-0.0, 0.0], n)
        elif kind == 1:
            x = rng.choice([-1.0, -0.0, 0.0, 1.0, 2.0], n)
        elif kind == 2:
            x = rng.standard_normal(n)
            x[rng.random(n) < 0.4] = 0.0
        elif kind == 3:
            x = np.sort(rng.integers(-3, 4, n).astype(float))
        else:
            x = rng.integers(0, 5, n).astype(float)[::-1].copy()
        yield x


def test_batched_hoare_equals_sequential():
    rng = np.random.default_rng(5)
    checked = 0
    for x in _cases(rng):
        n = len(x)
        for low, high in ((0, n - 1), (n // 3, n - 1), (0, max(2, n // 2)), (1, n - 2)):
            if high - low < 2:
                continue
            for mom5 in (False, True):
                a = list(x)
                b = list(x)
                if not mom5:
                    mid = low + (high - low) // 2
                    for arr in (a, b):   # median3_swap_
                        if _less(arr[high], arr[mid]):
                            arr[high], arr[mid] = arr[mid], arr[high]
                        if _less(arr[high], arr[low]):
                            arr[high], arr[low] = arr[low], arr[high]
                        if _less(arr[low], arr[mid]):
                            arr[low], arr[mid] = arr[mid], arr[low]
                        arr[mid], arr[low + 1] = arr[low + 1], arr[mid]
                else:
                    # the median of medians swapped to low (it has elements >= it to its right)
                    for arr in (a, b):
                        seg = np.array(arr[low:high + 1])
                        k = low + int(np.argsort(seg, kind="stable")[len(seg) // 2])
                        arr[k], arr[low] = arr[low], arr[k]
                pv = a[low]
                r1 = hoare_sequential(a, low, high, pv, mom5)
                ll0, hh0 = (low, high + 1) if mom5 else (low + 1, high)
                r2 = hoare_batched(b, n, pv, ll0, hh0)
                assert r1 == r2, (n, low, high, mom5)
                assert np.array_equal(np.array(a).view(np.uint64), np.array(b).view(np.uint64))
                checked += 1
    assert checked > 2000

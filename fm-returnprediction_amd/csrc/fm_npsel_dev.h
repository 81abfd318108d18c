// numpy 1.26.4's ndarray.partition replayed by ONE wave, to pin the SIGN of an exactly-zero
// winsorize cut.
//
// np.percentile(vals, q) (reference src/calc_Lewellen_2014.py:522-523; numpy
// function_base._quantile) partitions a copy of `vals` -- the month's non-NaN values in frame
// order -- at kth = unique([0, -1, i, i+1]) and lerps arr[i], arr[i+1].  -0.0 == +0.0, so which
// signed zero lands at i / i+1 is decided by the partition's swap order alone.  This file
// replays that order exactly (npysort/selection.cpp introselect_ + item_selection.c
// _new_sortlike: kth made non-negative and sorted, one introselect per kth over the whole
// array with a shared stack of <= 50 pivots; dumb selection when kth - low < 3; a max scan
// when kth == n - 1; median-of-3 quickselect with an unguarded Hoare partition; median of
// medians of 5 past the depth limit 2 msb(n)).  oracle/np_select.py is the CPU restatement,
// pinned bit for bit against numpy 1.26.4 (tools/check_np_select.py).
//
// The wave replays the SEQUENTIAL algorithm with the sequential scans done 64 positions at a
// time: the Hoare loop's stoppers (left: !(v < p), right: !(p < v)) of a 64-position window
// on each side are found by ballots and paired in order; every pair with L < R is swapped at
// once (positions strictly between the last swapped pair are untouched, so the stoppers
// computed before the batch are the ones the sequential scans would find); the first pair
// with L >= R ends the batch, and the next round rescans the current values from the last
// swapped pair, which reproduces the sequential scans' stops exactly (a swapped position
// holds a stopper for the opposite scan).  Only reached for units whose cut is exactly zero
// and whose values hold both signed zeros, so speed is secondary.
#pragma once

#include "fm_common.h"

namespace fm {

// the unit's values, in LDS (one wave's LDS operations complete in order)
struct NpLds {
    double* p;
    __device__ __forceinline__ double ld(int i) const { return p[i]; }
    __device__ __forceinline__ void st(int i, double v) const { p[i] = v; }
    __device__ __forceinline__ void sync() const { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); }
    __device__ __forceinline__ NpLds off(int o) const { return NpLds{p + o}; }
};

// ... or in a global scratch slot (L2-coherent loads / stores; a fence orders each batch)
struct NpGlobal {
    double* p;
    __device__ __forceinline__ double ld(int i) const {
        return __longlong_as_double((long long)__hip_atomic_load((unsigned long long*)(p + i), __ATOMIC_RELAXED,
                                                                 __HIP_MEMORY_SCOPE_AGENT));
    }
    __device__ __forceinline__ void st(int i, double v) const {
        __hip_atomic_store((unsigned long long*)(p + i), (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
    __device__ __forceinline__ void sync() const { __threadfence(); }
    __device__ __forceinline__ NpGlobal off(int o) const { return NpGlobal{p + o}; }
};

constexpr int NP_MAX_PIVOT_STACK = 50;

// npy::double_tag::less (NaN sorts last)
__device__ __forceinline__ bool np_less(double a, double b) { return a < b || (b != b && a == a); }

__device__ __forceinline__ int np_msb(int n) {
    int d = 0;
    for (n >>= 1; n; n >>= 1) ++d;
    return d;
}

// position of the j-th set bit of m (j < popcount(m))
__device__ __forceinline__ int np_nth_bit(uint64_t m, int j) {
    int pos = 0;
#pragma unroll
    for (int w = 32; w >= 1; w >>= 1) {
        const uint64_t low = m & ((w == 64 ? 0ull : (1ull << w)) - 1ull);
        const int c = __popcll(low);
        if (j >= c) {
            j -= c;
            m >>= w;
            pos += w;
        } else {
            m = low;
        }
    }
    return pos;
}

// the pivot stack lives in one VGPR (lane i = pivots[i]); npiv is wave-uniform
__device__ __forceinline__ void np_store_pivot(int pivot, int kth, int& piv, int& npiv) {
    const int lane = lane_id();
    if (pivot == kth && npiv == NP_MAX_PIVOT_STACK) {
        if (lane == npiv - 1) piv = pivot;
    } else if (pivot >= kth && npiv < NP_MAX_PIVOT_STACK) {
        if (lane == npiv) piv = pivot;
        ++npiv;
    }
}

template <class A>
__device__ __forceinline__ void np_swap1(A arr, int i, int j) {   // lane 0
    if (lane_id() == 0 && i != j) {
        const double x = arr.ld(i), y = arr.ld(j);
        arr.st(i, y);
        arr.st(j, x);
    }
    arr.sync();
}

// dumb_select_: selection sort of positions [b, b + kth] over [b, b + num) (first minimum wins)
template <class A>
__device__ __forceinline__ void np_dumb_select(A arr, int b, int num, int kth) {
    const int lane = lane_id();
    for (int i = 0; i <= kth; ++i) {
        double mv = 0.0;
        int mi = 0x7FFFFFFF;
        for (int p = b + i + lane; p < b + num; p += WAVE) {
            const double x = arr.ld(p);
            if (mi == 0x7FFFFFFF || np_less(x, mv)) mv = x, mi = p;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const double ov = __shfl_xor(mv, o, WAVE);
            const int oi = __shfl_xor(mi, o, WAVE);
            const bool take = oi != 0x7FFFFFFF &&
                              (mi == 0x7FFFFFFF || np_less(ov, mv) || (!np_less(mv, ov) && oi < mi));
            if (take) mv = ov, mi = oi;
        }
        np_swap1(arr, b + i, __builtin_amdgcn_readfirstlane(mi));
    }
}

// unguarded_partition_: stoppers found 64 positions at a time (see the header comment).
// In: ll / hh the scans' starting cursors (exclusive); out: where they stopped.
template <class A>
__device__ __forceinline__ void np_hoare(A arr, int n, double pv, int& ll, int& hh) {
    const int lane = lane_id();
    // every round swaps >= 1 pair, steps a window past stopper-free positions or ends: the
    // bound only guards against a hang (tests/test_npsel_batch.py checks the loop on the CPU)
    for (int it = 0; it < 2 * n + 256; ++it) {
        const int pl = ll + 1 + lane, pr = hh - 1 - lane;
        const double xl = arr.ld(pl < n ? pl : n - 1);
        const double xr = arr.ld(pr >= 0 ? pr : 0);
        const uint64_t ml = __ballot(pl < n && !np_less(xl, pv));
        const uint64_t mr = __ballot(pr >= 0 && !np_less(pv, xr));
        const int cl = __popcll(ml), cr = __popcll(mr);
        if (cl == 0 || cr == 0) {   // a window without a stopper: step past it
            if (cl == 0) ll += WAVE;
            if (cr == 0) hh -= WAVE;
            continue;
        }
        const int m = cl < cr ? cl : cr;
        const int Lj = lane < m ? ll + 1 + np_nth_bit(ml, lane) : 0x7FFFFFFF;
        const int Rj = lane < m ? hh - 1 - np_nth_bit(mr, lane) : -1;
        const uint64_t vm = __ballot(lane < m && Lj < Rj);   // a prefix: L rises, R falls
        const int P = vm == ~0ull ? WAVE : __builtin_ctzll(~vm);
        if (P == 0) {
            const int L0 = __builtin_amdgcn_readfirstlane(Lj), R0 = __builtin_amdgcn_readfirstlane(Rj);
            ll = L0;
            hh = R0;
            if (L0 > R0) return;
            continue;   // L0 == R0: an element equal to the pivot, swapped with itself
        }
        if (lane < P) {
            const double x = arr.ld(Lj), y = arr.ld(Rj);
            arr.st(Lj, y);
            arr.st(Rj, x);
        }
        arr.sync();
        ll = __builtin_amdgcn_readlane(Lj, P - 1);
        hh = __builtin_amdgcn_readlane(Rj, P - 1);
    }
}

// D: levels of median-of-medians recursion replayed exactly; past them the inner selection
// uses median-of-3 pivots (differs from numpy only if the selection over the medians ALSO
// exhausts its depth limit -- adversarial data at two levels at once).  Everything is inlined:
// no call stack, no scratch.
#ifndef FM_NP_MOM_DEPTH
#define FM_NP_MOM_DEPTH 1
#endif
template <int D, class A>
__device__ __forceinline__ void np_introselect(A arr, int num, int kth, int& piv, int& npiv, bool stack);

// median5_: index (0..4) of the median of arr[0..5), with numpy's swaps (lane 0)
template <class A>
__device__ __forceinline__ int np_median5(A v) {
    auto cs = [&](int i, int j) {   // if v[i] < v[j]: swap
        const double x = v.ld(i), y = v.ld(j);
        if (np_less(x, y)) {
            v.st(i, y);
            v.st(j, x);
        }
    };
    cs(1, 0);
    cs(4, 3);
    cs(3, 0);
    cs(4, 1);
    cs(2, 1);
    if (np_less(v.ld(3), v.ld(2))) return np_less(v.ld(3), v.ld(1)) ? 1 : 3;
    return 2;
}

// median_of_median5_ on arr[0..num): the groups' medians moved to the front, then the median
// of those by a stack-less introselect (depth-bounded here: D levels)
template <int D, class A>
__device__ __forceinline__ int np_mom5(A arr, int num) {
    const int nmed = num / 5;
    if (lane_id() == 0) {
        for (int i = 0, sl = 0; i < nmed; ++i, sl += 5) {
            const int m = np_median5(arr.off(sl));
            const double x = arr.ld(sl + m), y = arr.ld(i);
            arr.st(sl + m, y);
            arr.st(i, x);
        }
    }
    arr.sync();
    if (nmed > 2) {
        if constexpr (D > 0) {
            int p0 = 0, n0 = 0;
            np_introselect<D - 1>(arr, nmed, nmed / 2, p0, n0, false);
        }
    }
    return nmed / 2;
}

// introselect_<double_tag, false>: kth of arr[0..num) (stack == false: no pivot stack)
template <int D, class A>
__device__ __forceinline__ void np_introselect(A arr, int num, int kth, int& piv, int& npiv, bool stack) {
    const int lane = lane_id();
    int low = 0, high = num - 1;
    if (stack) {
        while (npiv > 0) {
            const int top = __builtin_amdgcn_readlane(piv, npiv - 1);
            if (top > kth) {
                high = top - 1;
                break;
            }
            if (top == kth) return;
            low = top + 1;
            --npiv;
        }
    }
    if (kth - low < 3) {
        np_dumb_select(arr, low, high - low + 1, kth - low);
        if (stack) np_store_pivot(kth, kth, piv, npiv);
        return;
    }
    if (kth == num - 1) {   // inexact types: a max scan, the LAST maximum wins; no pivot stored
        double mv = 0.0;
        int mi = -1;
        for (int p = low + lane; p < num; p += WAVE) {
            const double x = arr.ld(p);
            if (mi < 0 || !np_less(x, mv)) mv = x, mi = p;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const double ov = __shfl_xor(mv, o, WAVE);
            const int oi = __shfl_xor(mi, o, WAVE);
            const bool take = oi >= 0 && (mi < 0 || np_less(mv, ov) || (!np_less(ov, mv) && oi > mi));
            if (take) mv = ov, mi = oi;
        }
        np_swap1(arr, kth, __builtin_amdgcn_readfirstlane(mi));
        return;
    }
    int depth = np_msb(num) * 2;
    while (low + 1 < high) {
        int ll = low + 1, hh = high;
        if (depth > 0 || hh - ll < 5 || D == 0) {
            const int mid = low + (high - low) / 2;
            if (lane == 0) {   // median3_swap_
                double vl = arr.ld(low), vm = arr.ld(mid), vh = arr.ld(high), t;
                if (np_less(vh, vm)) t = vh, vh = vm, vm = t;
                if (np_less(vh, vl)) t = vh, vh = vl, vl = t;
                if (np_less(vl, vm)) t = vl, vl = vm, vm = t;
                arr.st(low, vl);
                arr.st(mid, vm);
                arr.st(high, vh);
            }
            arr.sync();
            np_swap1(arr, mid, low + 1);
        } else {
            const int mid = ll + np_mom5<D>(arr.off(ll), hh - ll);
            np_swap1(arr, mid, low);
            --ll;
            ++hh;
        }
        --depth;
        const double pv = arr.ld(low);
        np_hoare(arr, num, pv, ll, hh);
        np_swap1(arr, low, hh);
        if (hh != kth && stack) np_store_pivot(hh, kth, piv, npiv);
        if (hh >= kth) high = hh - 1;
        if (hh <= kth) low = ll;
    }
    if (high == low + 1) {
        const double x = arr.ld(low), y = arr.ld(high);
        if (np_less(y, x)) np_swap1(arr, low, high);
    }
    if (stack) np_store_pivot(kth, kth, piv, npiv);
}

// arr[i], arr[i+1] after np.percentile's partition of arr[0..n) (i < 0: the rank is past
// n - 2, numpy's index -1 for both; kth = [0, n-1]).  Wave-uniform results.
template <class A>
__device__ __forceinline__ void np_percentile_pair(A arr, int n, int i, double& va, double& vb) {
    // kth = np.unique([0, -1, i, i+1]) made non-negative and sorted: [0, i (i > 0), i+1, n-1]
    // (i+1 == n-1 stays a duplicate: its second introselect finds the pivot and returns);
    // the rank past n - 2 (i < 0): [0, n-1].  One loop (one inlined copy), no private arrays.
    int piv = 0, npiv = 0;
#pragma unroll 1
    for (int q = 0; q < 4; ++q) {
        if (i < 0 && (q == 1 || q == 2)) continue;
        if (q == 1 && i == 0) continue;
        const int kth = q == 0 ? 0 : (q == 1 ? i : (q == 2 ? i + 1 : n - 1));
        np_introselect<FM_NP_MOM_DEPTH>(arr, n, kth, piv, npiv, true);
    }
    arr.sync();
    const int ia = i < 0 ? n - 1 : i, ib = i < 0 ? n - 1 : i + 1;
    va = arr.ld(ia);
    vb = arr.ld(ib);
}

}  // namespace fm

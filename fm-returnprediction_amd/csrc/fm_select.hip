// fm_select_cuts: exact per-(month, column) order statistics on gfx950.
//
// Replaces np.percentile(vals, 1/99) in winsorize (reference src/calc_Lewellen_2014.py:
// 519-523) and pandas groupby(...).quantile([.2,.5]) of NYSE `me` in get_subsets (:74-82).
//
// One 256-thread workgroup per (segment, column).  The segment's values live in registers
// as FP64 (VPT per thread, one coalesced HBM read; NaN = missing or masked out).  Both
// winsorize tails (ranks ~n/100 from either end) are found in one pass (select_tails):
//   * tau = the exact rj-th smallest of the 256 per-thread minima (per-wave bitonic sort
//     + merge ranks by binary search): rj+1 threads own a value <= tau, so s[rj] <= tau;
//   * only the values < tau can precede s[rj]; there are about rj of them, compacted
//     to LDS with one packed scan (both tails at once) and sorted by one wave per tail.
// Middle ranks (pandas 0.2/0.5) and any overflow use an exact MSB-first 8-bit radix
// select over order-preserving uint64 keys formed on the fly.  Results are the exact order
// statistics, so the interpolated cut is bit-identical to numpy/pandas given the same
// no-FMA lerp (this file is compiled with -ffp-contract=off).
#include <math.h>
#include <stdlib.h>

#include "fm_common.h"

FM_PROBE_BUFFER(sel)
#define FM_HS_PROBE_ON 1
#include "fm_select_dev.h"
#include "fm_npsel_dev.h"

#ifndef FM_SELECT_STREAM_VPT
#define FM_SELECT_STREAM_VPT 24   // values per thread above which fm_select streams the units
#endif
#ifndef FM_AB_LONG
#define FM_AB_LONG 0              // timing builds only: 1 loads + count, 2 no candidate select
#endif
#ifndef FM_AB_SELECT_STREAM
#define FM_AB_SELECT_STREAM 0     // timing builds only: the streaming kernel for every long unit
#endif
#ifndef FM_SELECT_STREAM_SB
#define FM_SELECT_STREAM_SB 8     // loads per thread in flight in each streaming pass
#endif

namespace fm {
namespace {

template <int VPT>
__global__ __launch_bounds__(ST) void select_kernel(SelArgs a) {
    __shared__ SelSmem sm;
    select_unit_wg<VPT>(a, blockIdx.x, blockIdx.y, sm);
}

// Segments past the register budget (> 20,480 rows: a daily-frequency panel, a huge
// cross-section; > 6,144 rows with moments; the units the long-segment kernel marked): one workgroup per (segment, column) STREAMS the segment from HBM for every pass instead of holding it in registers -- count / key range, the adaptive
// histogram (hist_select: one histogram pass per level, one compaction pass), then the
// moments if asked.  Exact order statistics, same lerps, same pivot as the register paths.
__device__ __forceinline__ void stream_unit(const SelArgs& a, int s, int c, SelSmem& sm) {
    const int64_t r0 = a.seg_off[s];
    const int64_t L = a.seg_off[s + 1] - r0;
    const PCols src = sel_col(a, c, r0);
    const uint8_t* msk = a.mask ? a.mask + r0 : nullptr;
    // every pass streams the unit with SB loads per thread in flight (clamped, unconditional:
    // a load per loop iteration would wait out one memory round trip per value)
    constexpr int SB = FM_SELECT_STREAM_SB;
    auto for_each = [&](auto&& f) {
        for (int64_t i0 = threadIdx.x; i0 < L; i0 += (int64_t)SB * ST) {
            double xs[SB];
            uint8_t ms[SB];
#pragma unroll
            for (int k = 0; k < SB; ++k) {
                const int64_t i = i0 + (int64_t)k * ST;
                const int64_t ic = i < L ? i : L - 1;
                xs[k] = src[ic];
                ms[k] = msk ? msk[ic] : (uint8_t)1;
            }
#pragma unroll
            for (int k = 0; k < SB; ++k)
                if (i0 + (int64_t)k * ST < L) f(ms[k] != 0 ? xs[k] : NAN);
        }
    };
    int cnt = 0;
    uint64_t kmn = SENT, kmx = 0;
    double fmn = NAN, fmx = NAN;   // finite range (pivot fallback)
    for_each([&](double x) {
        if (!isnan(x)) {
            ++cnt;
            const uint64_t k = dkey(x);
            kmn = k < kmn ? k : kmn;
            kmx = k > kmx ? k : kmx;
            if (isfinite(x)) {
                fmn = hw_min(fmn, x);
                fmx = hw_max(fmx, x);
            }
        }
    });
    const int n = block_sum<SNW>(cnt, sm.ints);
    kmn = block_min_u64<SNW>(kmn, sm.u64s);
    kmx = block_max_u64<SNW>(kmx, sm.u64s + SNW);
    double lo = NAN, hi = NAN;
    if (n >= a.min_count && n > 0) {
        int rk[4];
        double g0, g1;
        qranks(n, a.q_lo, a.lerp_mode, rk[0], rk[1], g0);
        qranks(n, a.q_hi, a.lerp_mode, rk[2], rk[3], g1);
        uint64_t ko[4];
        hist_select(for_each, 4, rk, kmn, kmx, ko, sm);
        lo = qlerp(kval(ko[0]), kval(ko[1]), g0, a.lerp_mode);
        hi = qlerp(kval(ko[2]), kval(ko[3]), g1, a.lerp_mode);
    }
    const int64_t o = (int64_t)c * a.nseg + s;
    if (a.center != nullptr) {
        double cen = 0.5 * (lo + hi);
        if (!isfinite(cen)) {
            const double m1 = block_min_f64<SNW>(isfinite(fmn) ? fmn : NAN, sm.dbl);
            const double m2 = -block_min_f64<SNW>(isfinite(fmx) ? -fmx : NAN, sm.dbl);
            cen = 0.5 * (m1 + m2);
            if (!isfinite(cen)) cen = 0.0;
        }
        if (threadIdx.x == 0) a.center[o] = cen;
    }
    if (a.mean != nullptr) {
        // moments of the clipped values about a pivot inside the data (select_unit_wg)
        double p = isfinite(lo) ? lo : (isfinite(hi) ? hi : 0.0);
        if (!isfinite(lo) && !isfinite(hi)) {
            p = block_min_f64<SNW>(isfinite(fmn) ? fmn : NAN, sm.dbl);
            if (!isfinite(p)) p = 0.0;
        }
        double s1 = 0.0, s2 = 0.0;
        for_each([&](double x) {
            if (x < lo) x = lo;
            if (x > hi) x = hi;
            const double d = isnan(x) ? 0.0 : x - p;
            s1 += d;
            s2 = fma(d, d, s2);
        });
        double2 r = block_sum2<SNW>(s1, s2, sm.dbl);
        if (threadIdx.x == 0) {
            a.mean[o] = n > 0 ? p + r.x / (double)n : NAN;
            if (a.sd) {
                double var = n > 1 ? (r.y - r.x * (r.x / (double)n)) / (double)(n - 1) : NAN;
                if (var < 0.0) var = 0.0;
                a.sd[o] = n > 1 ? sqrt(var) : NAN;
            }
        }
    }
    if (threadIdx.x == 0) {
        a.lo[o] = lo;
        a.hi[o] = hi;
        if (a.nvalid) a.nvalid[o] = n;
        if (zero_cut(a, lo, hi)) sel_push(a, o);
    }
}


// ---- The fix-up pass: one launch after every fm_select path.  The fast kernels put on
// fm_select_args.ws's worklist the units they could not finish (marked nvalid = -1: ranks
// past their tail windows, candidate overflow, ambiguous high keys) and the units whose numpy
// cut came out exactly +-0; each workgroup here redoes its share of the list exactly (the
// register workgroup path up to VPT values per thread, else streaming) and, for a zero cut
// of a unit whose values hold both -0.0 and +0.0, replays numpy's partition to get the
// reference's sign (fm_npsel_dev.h).  An empty list costs one load per workgroup; the last
// workgroup to finish leaves the list empty for the next call.
constexpr int ZS_LDS = 6144;               // units of up to this many rows replay in LDS
constexpr int FIX_GRID = 256;
constexpr int64_t ZS_GLOBAL_BYTES = 64ll << 20;   // longer units: one global slot per workgroup

union FixSmem {
    SelSmem sel;
    double arr[ZS_LDS];
};

// wave 0: the exactly-zero numpy cuts of unit (s, c), written by this workgroup just before
template <class A>
__device__ __forceinline__ void zero_sign_unit(const SelArgs& a, int s, int c, A arr) {
    const int lane = lane_id();
    const int64_t o = (int64_t)c * a.nseg + s;
    auto ld = [](const double* p) {
        return __longlong_as_double(
            (long long)__hip_atomic_load((const unsigned long long*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    };
    const double lo = ld(a.lo + o), hi = ld(a.hi + o);
    const bool zl = lo == 0.0, zh = hi == 0.0;
    if (!zl && !zh) return;
    const int64_t r0 = a.seg_off[s];
    const int L = (int)(a.seg_off[s + 1] - r0);
    const PCols src = sel_col(a, c, r0);
    const uint8_t* msk = a.mask ? a.mask + r0 : nullptr;
    // the values np.percentile sees: the unit's non-NaN (row-mask selected) rows, frame order
    auto fill = [&](bool& both) -> int {
        int cnt = 0;
        bool ng = false, ps = false;
        for (int b = 0; b < L; b += WAVE) {
            const int r = b + lane;
            double x = r < L ? src[r] : (double)NAN;
            if (msk != nullptr && r < L && msk[r] == 0) x = NAN;
            const bool v = !isnan(x);
            const uint64_t bal = __ballot(v);
            if (v) arr.st(cnt + mask_rank(bal), x);
            cnt += (int)__popcll(bal);
            const bool z = x == 0.0;
            ng = ng || (z && __double_as_longlong(x) < 0);
            ps = ps || (z && __double_as_longlong(x) >= 0);
        }
        arr.sync();
        both = __ballot(ng) != 0ull && __ballot(ps) != 0ull;
        return cnt;
    };
    bool both = false;
    int n = fill(both);
    if (!both) return;   // one kind of zero: the key order already gave the reference's bits
    for (int t = 0; t < 2; ++t) {
        if (t == 0 ? !zl : !zh) continue;
        const double q = t == 0 ? a.q_lo : a.q_hi;
        int i, j;
        double g;
        qranks(n, q, 0, i, j, g);
        if (t == 1 && zl) n = fill(both);   // each np.percentile call partitions its own copy
        const bool top = (double)(n - 1) * q >= (double)(n - 1);
        double va, vb;
        np_percentile_pair(arr, n, top ? -1 : i, va, vb);
        const double r = qlerp(va, vb, g, 0);
        if (lane == 0) (t == 0 ? a.lo : a.hi)[o] = r;
    }
}

// The fix-up work of workgroup `bid` of `nblk` (the fix-up launch, or the fix-up part of
// the launch it shares with the universe)
template <int VPT>   // VPT == 0: the streaming exact path
__device__ __forceinline__ void fixup_body(const SelArgs& a, double* zs, int zs_len, uint32_t bid, uint32_t nblk,
                                           FixSmem& sm) {
    SelCtl* ctl = a.ctl;
    SelArgs b = a;
    b.ctl = nullptr;
    FM_PROBE_AT(sel, 4);
    const uint32_t nw0 = __hip_atomic_load(&ctl->nwork, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // an empty list (every workgroup reads the same count: nothing appends during this launch)
    // needs no reset: exit without touching the done counter (256 same-address atomics cost
    // more than the whole no-op launch)
    FM_PROBE_AT(sel, 5);
    if (nw0 == 0) return;
    // a list left over by a call whose fix-up never ran (an error between the launches) may
    // hold more entries than this call's units, or ids of a larger shape: both are bounded
    // here (a stale in-range id only redoes that unit exactly: same result)
    const uint32_t nunits = (uint32_t)((int64_t)b.nseg * b.ncols);
    const uint32_t nw = nw0 < nunits ? nw0 : nunits;
    for (uint32_t i = bid; i < nw; i += nblk) {
        const uint32_t u = ctl->work[i];
        if (u >= nunits) continue;   // workgroup-uniform
        const int s = (int)(u % (uint32_t)b.nseg), c = (int)(u / (uint32_t)b.nseg);
        if constexpr (VPT > 0) select_unit_wg<VPT>(b, s, c, sm.sel);
        else stream_unit(b, s, c, sm.sel);
        __threadfence();
        __syncthreads();
        if (b.lerp_mode == 0 && threadIdx.x < WAVE) {
            const int64_t L = b.seg_off[s + 1] - b.seg_off[s];
            if (L <= ZS_LDS) zero_sign_unit(b, s, c, NpLds{sm.arr});
            else zero_sign_unit(b, s, c, NpGlobal{zs + (int64_t)bid * zs_len});
        }
        __threadfence();
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        __threadfence();
        const uint32_t t = atomicAdd(&ctl->done, 1u);
        if (t == nblk - 1) {
            __hip_atomic_store(&ctl->nwork, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&ctl->done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

template <int VPT>
__global__ __launch_bounds__(ST) void select_fixup_kernel(SelArgs a, double* zs, int zs_len) {
    __shared__ FixSmem sm;
    fixup_body<VPT>(a, zs, zs_len, blockIdx.x, gridDim.x, sm);
}

template <int VPT>
__device__ __forceinline__ void universe_month(const double* __restrict__ me, const uint8_t* __restrict__ nyse,
                                               const int64_t* __restrict__ seg_off, double qa, double qb,
                                               double* __restrict__ cut_a, double* __restrict__ cut_b,
                                               uint8_t* __restrict__ level, int s, SelSmem& sm);

// The select fix-up and get_subsets' NYSE breakpoints + level bytes in ONE launch (the two
// are independent; the universe no longer needs a launch of its own before the select):
// workgroups [0, nseg) are universe_kernel's months, the rest the fix-up's workgroups (which
// return at once when no unit is marked).  Held to universe_kernel's 3 waves per SIMD.
template <int VPT>
__global__ __launch_bounds__(ST, 3) void select_fixup_universe_kernel(SelArgs a, double* zs, int zs_len) {
    __shared__ FixSmem sm;
    const int nuni = a.nseg;
    if ((int)blockIdx.x < nuni) {   // block-uniform
        universe_month<VPT>(a.ume, a.unyse, a.seg_off, a.uq_a, a.uq_b, a.ucut_a, a.ucut_b, a.ulevel, (int)blockIdx.x,
                            sm.sel);
        return;
    }
    fixup_body<VPT>(a, zs, zs_len, blockIdx.x - nuni, gridDim.x - nuni, sm);
}

int64_t ws_list_bytes(int64_t nunits) { return ((int64_t)offsetof(SelCtl, work) + 4 * nunits + 255) / 256 * 256; }
int fix_grid(int max_seg_len) {
    if (max_seg_len <= ZS_LDS) return FIX_GRID;
    const int64_t g = ZS_GLOBAL_BYTES / ((int64_t)max_seg_len * 8);
    return (int)(g < 1 ? 1 : (g < FIX_GRID ? g : FIX_GRID));
}
int64_t ws_bytes(int32_t nseg, int32_t ncols, int32_t max_seg_len) {
    const int64_t list = ws_list_bytes((int64_t)nseg * ncols);
    return max_seg_len <= ZS_LDS ? list : list + (int64_t)fix_grid(max_seg_len) * max_seg_len * 8;
}

void launch_fixup(const SelArgs& a, int max_seg_len, hipStream_t st) {
    const int vpt = (max_seg_len + ST - 1) / ST;
    const int g = fix_grid(max_seg_len);
    double* zs = (double*)((char*)a.ctl + ws_list_bytes((int64_t)a.nseg * a.ncols));
    const int zl = max_seg_len;
    if (vpt <= 2) hipLaunchKernelGGL(select_fixup_kernel<2>, dim3(g), dim3(ST), 0, st, a, zs, zl);
    else if (vpt <= 4) hipLaunchKernelGGL(select_fixup_kernel<4>, dim3(g), dim3(ST), 0, st, a, zs, zl);
    else if (vpt <= 8) hipLaunchKernelGGL(select_fixup_kernel<8>, dim3(g), dim3(ST), 0, st, a, zs, zl);
    else if (vpt <= 16) hipLaunchKernelGGL(select_fixup_kernel<16>, dim3(g), dim3(ST), 0, st, a, zs, zl);
    else if (vpt <= 20) hipLaunchKernelGGL(select_fixup_kernel<20>, dim3(g), dim3(ST), 0, st, a, zs, zl);
    else if (vpt <= FM_SELECT_STREAM_VPT) hipLaunchKernelGGL(select_fixup_kernel<FM_SELECT_STREAM_VPT>, dim3(g), dim3(ST), 0, st, a, zs, zl);
    else hipLaunchKernelGGL(select_fixup_kernel<0>, dim3(g), dim3(ST), 0, st, a, zs, zl);
}

// fix-up + universe in one launch (months of <= 20 x 256 rows): the fix-up workgroups are
// the slots the universe's months leave in one resident round (3 per CU), at least 32
int launch_fixup_universe(const SelArgs& a, int max_seg_len, hipStream_t st) {
    static int ncu = [] {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
            n = 256;
        return n;
    }();
    const int vpt = (max_seg_len + ST - 1) / ST;
    int nfix = 3 * ncu - a.nseg;
    nfix = nfix < 32 ? 32 : (nfix > fix_grid(max_seg_len) ? fix_grid(max_seg_len) : nfix);
    double* zs = (double*)((char*)a.ctl + ws_list_bytes((int64_t)a.nseg * a.ncols));
    const dim3 g((unsigned)(a.nseg + nfix));
    if (vpt <= 8) hipLaunchKernelGGL(select_fixup_universe_kernel<8>, g, dim3(ST), 0, st, a, zs, max_seg_len);
    else hipLaunchKernelGGL(select_fixup_universe_kernel<20>, g, dim3(ST), 0, st, a, zs, max_seg_len);
    return FM_OK;
}

// One unit per workgroup (grid nseg x ncols).
__global__ __launch_bounds__(ST) void select_stream_kernel(SelArgs a) {
    __shared__ SelSmem sm;
    stream_unit(a, blockIdx.x, blockIdx.y, sm);
}

// Long segments (6,145 .. 20,480 rows: C5's 20,000-firm months, a daily panel's short
// windows): one 512-thread workgroup per (segment, column) holds the unit in registers
// (VPT <= 40 values per thread, ONE coalesced HBM read of the unit).  Both winsorize tails:
//   * thresholds on the 32-bit HIGH words of the order-preserving keys: per wave the 64
//     thread minima's high words sorted, T_w = the wave's q-th smallest, q = ceil((k+1)/8)
//     for the largest needed rank k; c(T) = the valid thread minima with high word <= T
//     (ballots, summed over the waves by LDS atomics); tau = the smallest T_w with
//     c(tau) >= k+1.  The candidates -- every value whose high word is <= tau -- are then a
//     PREFIX of the sorted values holding at least k+1 of them, so the order statistics are
//     ranks inside the candidates (the upper tail the same on complemented keys);
//   * both tails' candidates (a little more than 2k values) are compacted to LDS (ballot
//     counts per wave, one barrier for the wave offsets); each wave sorts one 64-key run of each tail and every candidate finds its
//     merged rank by binary searches in the other runs, so the whole workgroup works on the
//     order statistics (no single-wave sort of hundreds of keys).
// Units it cannot finish (ranks >= 512, > 512 candidates per tail, too few valid thread
// minima) are marked (nvalid = -1) and redone by the streaming kernel's fallback pass.  At
// <= 128 VGPRs (4 waves per SIMD) two workgroups share a CU, so one unit's loads fly while
// the other selects.
#ifndef FM_AB_PAIR_MASKALL
#define FM_AB_PAIR_MASKALL 0   // timing builds only: test every value slot against the end
#endif
#ifndef FM_AB_LONG_MASKALL
#define FM_AB_LONG_MASKALL 0   // timing builds only: mask every value slot
#endif
// One month of get_subsets (reference src/calc_Lewellen_2014.py:69-105) by an NW-wave
// workgroup of the long-month kernel (one more grid column of fm_select_universe): the
// pandas-lerp q_a / q_b quantiles of the month's NYSE rows' `me` (NaN skipped) by the
// adaptive histogram select, then every row's level
// (me >= cut_a) + (me >= cut_b) -- universe_kernel's computation (same exact order
// statistics, same lerp), so the breakpoints and level bytes are identical.  The month's
// `me` / NYSE bytes are STREAMED (L2-resident after the first pass: 45 KB) in UB-row batches
// per pass instead of held in registers: the histogram select's own state already takes the
// host kernel's register budget, and it must stay at four waves per SIMD.
constexpr int UB = 8;
template <int NW, int HBN, int CAP, typename Sm>
__device__ __forceinline__ void universe_month_wg(const SelArgs& a, int s, Sm& sm) {
    constexpr int NT = NW * WAVE;
    const int tid = (int)threadIdx.x;
    const int64_t r0 = a.seg_off[s];
    const int L = (int)(a.seg_off[s + 1] - r0);
    const int last = L > 0 ? L - 1 : 0;
    const double* me = a.ume + r0;
    const uint8_t* ny = a.unyse + r0;
    const int nb = (L + NT * UB - 1) / (NT * UB);   // batches of UB rows per thread
    // f(x) for this thread's rows v * NT + tid: x = me of a NYSE row, NaN otherwise
    auto for_each = [&](auto&& f) {
#pragma unroll 1
        for (int b = 0; b < nb; ++b) {
            double xb[UB];
            uint8_t mb[UB];
#pragma unroll
            for (int q = 0; q < UB; ++q) {   // unconditional (clamped) loads, masked after
                const int idx = (b * UB + q) * NT + tid;
                const int ci = idx < L ? idx : last;
                xb[q] = me[ci];
                mb[q] = ny[ci];
            }
#pragma unroll
            for (int q = 0; q < UB; ++q) {
                const int idx = (b * UB + q) * NT + tid;
                f(idx < L && mb[q] != 0 ? xb[q] : NAN);
            }
        }
    };
    int cnt = 0;
    uint64_t kmn = SENT, kmx = 0;
    for_each([&](double x) {
        if (!isnan(x)) {
            ++cnt;
            const uint64_t k = dkey(x);
            kmn = k < kmn ? k : kmn;
            kmx = k > kmx ? k : kmx;
        }
    });
    const int n = block_sum<NW>(cnt, sm.ints);
    kmn = block_min_u64<NW>(kmn, sm.u64s);
    kmx = block_max_u64<NW>(kmx, sm.u64s + NW);
    double ca = NAN, cb = NAN;
    if (n > 0) {   // block-uniform
        int rk[4];
        double g0, g1;
        qranks(n, a.uq_a, 1, rk[0], rk[1], g0);
        qranks(n, a.uq_b, 1, rk[2], rk[3], g1);
        uint64_t ko[4] = {kmn, kmn, kmx, kmx};
        hist_select_t<NW, HBN, CAP>(for_each, 4, rk, kmn, kmx, ko, sm);
        ca = qlerp(kval(ko[0]), kval(ko[1]), g0, 1);
        cb = qlerp(kval(ko[2]), kval(ko[3]), g1, 1);
    }
    if (threadIdx.x == 0) {
        a.ucut_a[s] = ca;
        a.ucut_b[s] = cb;
    }
    // level bytes of every row (NYSE or not; NaN me compares False)
#pragma unroll 1
    for (int b = 0; b < nb; ++b) {
        double xb[UB];
#pragma unroll
        for (int q = 0; q < UB; ++q) {
            const int idx = (b * UB + q) * NT + tid;
            xb[q] = me[idx < L ? idx : last];
        }
#pragma unroll
        for (int q = 0; q < UB; ++q) {
            const int idx = (b * UB + q) * NT + tid;
            if (idx < L) a.ulevel[r0 + idx] = (uint8_t)((xb[q] >= ca ? 1 : 0) + (xb[q] >= cb ? 1 : 0));
        }
    }
    __syncthreads();   // the LDS is reused by the next unit
}

constexpr int LT = 512;
constexpr int LNW = LT / WAVE;
constexpr int LONG_VPT = 40;
constexpr int LCAP = 8 * WAVE;   // candidates per tail

struct LongSmem {
    double cand[2 * LCAP];       // lower-tail candidates, then upper-tail ones at LCAP
    SelSmemT<LNW> hs;            // hist_select scratch (and the block reductions)
    uint32_t tw[2][LNW];         // per-wave thresholds T_w (high words)
    int tot[2][LNW];             // c(T_w), summed over the waves
    int wc[2][LNW];              // per-wave candidate counts
    uint64_t res[4];             // keys of the four order statistics
};

// MID: any ranks (pandas' 20% / 50% NYSE breakpoints, row masks): the adaptive histogram
// select runs over the register-held values directly (no tail thresholds).
template <int VPT, bool MID>
__global__ __launch_bounds__(LT, MID ? 3 : 4) void select_long_kernel(SelArgs a) {
    __shared__ LongSmem sm;
    const int tid = (int)threadIdx.x, lane = lane_id();
    const int w = __builtin_amdgcn_readfirstlane(tid / WAVE);
    const int s = blockIdx.x, c = blockIdx.y;
    if (!MID && c == a.ncols) {   // fm_select_universe: the month's NYSE breakpoints + levels
        universe_month_wg<LNW, HB, HCAP>(a, s, sm.hs);
        return;
    }
    const int64_t o = (int64_t)c * a.nseg + s;
    const int64_t r0 = a.seg_off[s];
    const int L = (int)(a.seg_off[s + 1] - r0);
    typedef const __attribute__((address_space(1))) char* gptr;
    const gptr src = (gptr)(a.cols + (int64_t)c * a.col_stride + r0);
    const uint32_t lastb = (uint32_t)(L > 0 ? L - 1 : 0) * 8u;
    uint32_t lb = (uint32_t)tid * 8u;
    asm volatile("" : "+v"(lb));
    double xv[VPT];
    if (!MID || a.mask == nullptr) {   // block-uniform
#pragma unroll
        for (int v = 0; v < VPT; ++v) {   // unconditional (clamped) loads
            const uint32_t off = lb + (uint32_t)(v * LT * 8);
            xv[v] = *(const __attribute__((address_space(1))) double*)(src + (off < lastb ? off : lastb));
        }
        // masked after, and only the slots past the block's full rows of values (a scalar
        // branch per slot; the volatile asm keeps it a branch, not three selects per value)
        const int vf = FM_AB_LONG_MASKALL ? 0 : L / LT;
#pragma unroll
        for (int v = 0; v < VPT; ++v)
            if (v >= vf) {
                const uint32_t off = lb + (uint32_t)(v * LT * 8);
                double x = xv[v];
                asm volatile("" : "+v"(x));
                xv[v] = off <= lastb && L > 0 ? x : NAN;
            }
    } else {
        const gptr mb = (gptr)(a.mask + r0);
#pragma unroll
        for (int v = 0; v < VPT; ++v) {
            const uint32_t off = lb + (uint32_t)(v * LT * 8);
            const uint32_t oc = off < lastb ? off : lastb;
            const double x = *(const __attribute__((address_space(1))) double*)(src + oc);
            const uint8_t m = *(mb + (oc >> 3));
            xv[v] = off <= lastb && L > 0 && m != 0 ? x : NAN;
        }
    }
    int cnt = 0;
    double mn = NAN, mx = NAN;
#pragma unroll
    for (int v = 0; v < VPT; ++v) {
        cnt += isnan(xv[v]) ? 0 : 1;
        mn = hw_min(mn, xv[v]);
        mx = hw_max(mx, xv[v]);
    }
    if (tid < 2 * LNW) sm.tot[tid / LNW][tid % LNW] = 0;
    const int n = block_sum<LNW>(cnt, sm.hs.ints);
    double lo = NAN, hi = NAN;
    if (FM_AB_LONG == 1) {   // timing builds only: the load + count floor
        if (tid == 0) a.nvalid[o] = n, a.lo[o] = mn, a.hi[o] = mx;
        return;
    }
    bool ok = true;
    if (MID && n >= a.min_count && n > 0) {   // block-uniform
        int rk[4];
        double g0, g1;
        qranks(n, a.q_lo, a.lerp_mode, rk[0], rk[1], g0);
        qranks(n, a.q_hi, a.lerp_mode, rk[2], rk[3], g1);
        uint64_t kmn = SENT, kmx = 0;
#pragma unroll
        for (int v = 0; v < VPT; ++v)
            if (!isnan(xv[v])) {
                const uint64_t k = dkey(xv[v]);
                kmn = k < kmn ? k : kmn;
                kmx = k > kmx ? k : kmx;
            }
        kmn = block_min_u64<LNW>(kmn, sm.hs.u64s);
        kmx = block_max_u64<LNW>(kmx, sm.hs.u64s + LNW);
        uint64_t ko[4];
        hist_select_t<LNW, HB, HCAP>([&](auto&& f) {
#pragma unroll
            for (int v = 0; v < VPT; ++v) f(xv[v]);
        }, 4, rk, kmn, kmx, ko, sm.hs);
        lo = qlerp(kval(ko[0]), kval(ko[1]), g0, a.lerp_mode);
        hi = qlerp(kval(ko[2]), kval(ko[3]), g1, a.lerp_mode);
    } else if (!MID && n >= a.min_count && n > 0) {   // block-uniform
        int i0, j0, i1, j1;
        double g0, g1;
        qranks(n, a.q_lo, a.lerp_mode, i0, j0, g0);
        qranks(n, a.q_hi, a.lerp_mode, i1, j1, g1);
        const int kl = j0, ku = n - 1 - i1;        // largest ranks needed from either end
        const int ql = kl / LNW + 1, qu = ku / LNW + 1;
        ok = ql <= WAVE && qu <= WAVE;
        uint32_t tl = 0xFFFFFFFFu, tu = 0xFFFFFFFFu;
        if (ok) {
            // high words of the thread extrema's keys (NaN thread: 0xFFFFFFFF, above every
            // valid key's high word)
            uint32_t ha[1] = {isnan(mn) ? 0xFFFFFFFFu : (uint32_t)(dkey(mn) >> 32)};
            uint32_t hb[1] = {isnan(mx) ? 0xFFFFFFFFu : (uint32_t)(~dkey(mx) >> 32)};
            const uint32_t ua = ha[0], ub = hb[0];
            wave_sort32<1>(ha);
            wave_sort32<1>(hb);
            if (lane == 0) {
                sm.tw[0][w] = (uint32_t)__builtin_amdgcn_readlane((int)ha[0], ql - 1);
                sm.tw[1][w] = (uint32_t)__builtin_amdgcn_readlane((int)hb[0], qu - 1);
            }
            __syncthreads();
#pragma unroll
            for (int q = 0; q < LNW; ++q) {
                const uint32_t Ta = sm.tw[0][q], Tb = sm.tw[1][q];
                const int ca = (int)__popcll(__ballot(ua != 0xFFFFFFFFu && ua <= Ta));
                const int cb = (int)__popcll(__ballot(ub != 0xFFFFFFFFu && ub <= Tb));
                if (lane == 0) {
                    atomicAdd(&sm.tot[0][q], ca);
                    atomicAdd(&sm.tot[1][q], cb);
                }
            }
            __syncthreads();
#pragma unroll
            for (int q = 0; q < LNW; ++q) {
                const uint32_t Ta = sm.tw[0][q], Tb = sm.tw[1][q];
                if (Ta != 0xFFFFFFFFu && sm.tot[0][q] >= kl + 1 && Ta < tl) tl = Ta;
                if (Tb != 0xFFFFFFFFu && sm.tot[1][q] >= ku + 1 && Tb < tu) tu = Tb;
            }
            ok = tl != 0xFFFFFFFFu && tu != 0xFFFFFFFFu;
        }
        int clo = 0, chi = 0;
        if (ok) {
            // candidates by value compares against the largest / smallest double of the
            // threshold high word (+-inf at the ends, where the next keys would be NaNs);
            // value compares also take the other zero of a +-0 boundary, which keeps the
            // candidates a prefix / suffix of the sorted values
            const uint64_t kla = ((uint64_t)tl << 32) | 0xFFFFFFFFull;
            const uint64_t kub = ~(((uint64_t)tu << 32) | 0xFFFFFFFFull);
            const double tlo = kla >= dkey(INFINITY) ? INFINITY : kval(kla);
            const double thi = kub <= dkey(-INFINITY) ? -INFINITY : kval(kub);
            // wave totals from ballots (compares straight into lane masks, scalar counts),
            // then each wave's offset from the other waves' totals (one barrier)
            int wl = 0, wh = 0;
#pragma unroll
            for (int v = 0; v < VPT; ++v) {
                wl += (int)__popcll(__ballot(xv[v] <= tlo));
                wh += (int)__popcll(__ballot(xv[v] >= thi));
                // counts in order: otherwise the compiler forms all 2 x VPT ballot masks first
                // and spills them to VGPR lanes (~300 writelane / readlane VALU per wave)
                asm volatile("" : "+s"(wl), "+s"(wh));
            }
            if (lane == 0) {
                sm.wc[0][w] = wl;
                sm.wc[1][w] = wh;
            }
            __syncthreads();
            int ol = 0, oh = LCAP;
#pragma unroll
            for (int q = 0; q < LNW; ++q) {
                const int a0 = sm.wc[0][q], a1 = sm.wc[1][q];
                ol += q < w ? a0 : 0;
                oh += q < w ? a1 : 0;
                clo += a0;
                chi += a1;
            }
            // caps, and the rare overlap of the two sets (massive ties): redone by the fallback
            ok = clo <= LCAP && chi <= LCAP && clo + chi <= n && clo > kl && chi > ku;
            if (ok) {
#pragma unroll
                for (int v = 0; v < VPT; ++v) {
                    double x = xv[v];
                    asm volatile("" : "+v"(x));   // recompute (no SGPR masks kept from the count)
                    const uint64_t ml = __ballot(x <= tlo), mh = __ballot(x >= thi);
                    if (ml) {   // wave-uniform: most value slots hold no candidate
                        if (x <= tlo) sm.cand[ol + mask_rank(ml)] = x;
                        ol += (int)__popcll(ml);
                    }
                    if (mh) {
                        if (x >= thi) sm.cand[oh + mask_rank(mh)] = x;
                        oh += (int)__popcll(mh);
                    }
                }
                __syncthreads();
                // the four order statistics among the candidates: wave w sorts run w of each
                // tail (64 keys; the upper tail on complemented keys, so both count from their
                // end), then every candidate's merged rank = its run position + the entries
                // of the other runs before it (binary searches, ties by run); the lanes at
                // the target ranks store their keys
                uint64_t* ck = reinterpret_cast<uint64_t*>(sm.cand);
                const int e = w * WAVE + lane;
                uint64_t ka[1] = {e < clo ? dkey(sm.cand[e]) : SENT};
                uint64_t kb[1] = {e < chi ? ~dkey(sm.cand[LCAP + e]) : SENT};
                const int nrl = __builtin_amdgcn_readfirstlane((clo + WAVE - 1) / WAVE);
                const int nru = __builtin_amdgcn_readfirstlane((chi + WAVE - 1) / WAVE);
                // only the waves holding candidates sort (an all-sentinel run is sorted);
                // block-uniform counts, so the sorts run with the whole wave active
                if (FM_AB_LONG != 2 && w < nrl) wave_sort<1>(ka);
                if (FM_AB_LONG != 2 && w < nru) wave_sort<1>(kb);
                ck[e] = ka[0];   // in place: wave w owns entries [64 w, 64 w + 64) of each list
                ck[LCAP + e] = kb[0];
                if (tid < 4) sm.res[tid] = SENT;
                __syncthreads();
                if (ka[0] != SENT) {
                    int r = lane;
                    for (int u = 0; u < nrl; ++u)
                        if (u != w) r += merge_count(ck + u * WAVE, ka[0], u < w);
                    if (r == i0) sm.res[0] = ka[0];
                    if (r == j0) sm.res[1] = ka[0];
                }
                if (kb[0] != SENT) {
                    int r = lane;
                    for (int u = 0; u < nru; ++u)
                        if (u != w) r += merge_count(ck + LCAP + u * WAVE, kb[0], u < w);
                    if (r == n - 1 - i1) sm.res[2] = ~kb[0];
                    if (r == n - 1 - j1) sm.res[3] = ~kb[0];
                }
                __syncthreads();
                lo = qlerp(kval(sm.res[0]), kval(sm.res[1]), g0, a.lerp_mode);
                hi = qlerp(kval(sm.res[2]), kval(sm.res[3]), g1, a.lerp_mode);
            }
        }
    }
    if (!ok) {   // redone by the fix-up kernel
        if (tid == 0) sel_mark(a, o);
        return;
    }
    if (a.center != nullptr) {
        // Gram pivot: the midpoint of the cuts, else of the finite range, else 0
        double cen = 0.5 * (lo + hi);
        if (!isfinite(cen)) {   // block-uniform
            const uint64_t m1 = block_min_u64<LNW>(isfinite(mn) ? dkey(mn) : SENT, sm.hs.u64s);
            const uint64_t m2 = block_min_u64<LNW>(isfinite(mx) ? ~dkey(mx) : SENT, sm.hs.u64s + LNW);
            cen = m1 == SENT || m2 == SENT ? 0.0 : 0.5 * (kval(m1) + kval(~m2));
            if (!isfinite(cen)) cen = 0.0;
        }
        if (tid == 0) a.center[o] = cen;
    }
    if (tid == 0) {
        a.lo[o] = lo;
        a.hi[o] = hi;
        a.nvalid[o] = n;
        if (zero_cut(a, lo, hi)) sel_push(a, o);
    }
}

// ---- High-key tail kernel (the default for tail ranks without a row mask).
//
// The FP64 kernel above holds a unit's values in 80 VGPRs per thread, so only two 512-thread
// workgroups fit a CU and the chip idles its HBM while both compute.  The tails need far less:
// every step before the final candidate sort works on the HIGH 32 bits of the values' order
// keys (thread extrema, per-wave thresholds, ballot counts, compaction), and only the
// candidates' full values are gathered back from memory (a few hundred per unit).  40 VGPRs
// of keys per thread: three workgroups per CU, one unit each.  Per unit (round 6): the keys
// stream in as 16-byte slots (four rows per lane); each wave's tail threshold is its lane
// keys' q-th smallest by bit bisection; the candidates go straight into per-wave lists (no
// counting pass) and are re-indexed into 64-entry runs at the gather; the runs are sorted
// by the lane-mask 64-bit network and ranked by binary searches of the other runs, both
// tails side by side.  The SIMDs issue VALU in ~70 % of the kernel's cycles
// (profiles/r06/v11-v12): stage ablations on 1,000 x 20,000 x 15 put load + keys + counts at
// 0.21 ms of 0.48.
//
// (Thresholds from each thread's two smallest / largest keys instead of one measured slower:
// 0.72 vs 0.64 ms -- three more wave sorts per tail cost more than the fewer candidates save.)
//
// hkey: the dkey high word shifted so that -inf -> 0 and +inf -> HK_MAX, order-preserving over
// non-NaN values, and EVERY NaN lands above HK_MAX (positive NaNs above +inf, negative NaNs
// wrap past the top).  The one thing a high word cannot tell is +-inf from a NaN whose payload
// is all in the low word (high word 0x7FF00000 / 0xFFF00000): units holding either key
// (thread min 0 / thread max HK_MAX) are marked and redone by the exact streaming kernel.
#ifndef FM_HK_ABL
#define FM_HK_ABL 0   // timing ablations only (wrong cuts): 1 = stop after the thresholds, 2 = before the gather, 3 = after the counts
#endif
#ifndef FM_PAIR_KTH
#define FM_PAIR_KTH 1   // pair select: the tail threshold by bisection over unsorted lane extremes
#endif
#ifndef FM_HK_KTH
#define FM_HK_KTH 1   // per-wave thresholds by bit bisection (not a sort of the thread keys)
#endif
#ifndef FM_HK_WAVELIST
#define FM_HK_WAVELIST 1   // long-month candidates written straight into per-wave runs (no count pass)
#endif
#ifndef FM_HK_RIDE
#define FM_HK_RIDE 1   // a universe rides the high-key kernel's launch (one more grid column)
#endif
#ifndef FM_AB_NOFB
#define FM_AB_NOFB 0   // timing / probe builds only: no fallback launch after the long kernel
#endif
#ifndef FM_AB_LONG_F64
#define FM_AB_LONG_F64 0   // timing builds only: 1 = tails on the FP64-register kernel above
#endif
constexpr uint32_t HK_MAX = 0xFFE00001u;
constexpr uint32_t HK_NONE = 0xFFFFFFFFu;   // thread / threshold sentinel (no valid value)
__device__ __forceinline__ uint32_t hkey(uint32_t hi) {
    const uint32_t m = (uint32_t)((int32_t)hi >> 31) | 0x80000000u;
    return (hi ^ m) - 0x000FFFFFu;
}

struct LongHkSmem {
    uint64_t ck[2 * LCAP];       // candidate keys: lower tail, then upper tail at LCAP
    int cidx[2 * LCAP];          // candidate rows (compaction), same layout
    SelSmemT<LNW> hs;            // block reductions (and the riding universe's hist_select)
    uint32_t tw[2][LNW];
    int tot[2][LNW];
    int wc[2][LNW];
    uint64_t res[4];
};

// The high words of a unit into hk (raw; hkey is applied by the unit's own pass).  Slot v of
// thread t holds row hk_row(v, t): with FM_HK_X4, four consecutive rows per 16-byte load
// (row 4 LT (v / 4) + 4 t + v % 4: one descriptor per unit, a quarter of the load issue);
// otherwise row LT v + t, one 4-byte load per slot.  Rows past the month end read 0 through
// the descriptor's range check (checked per dword; masked later).
#ifndef FM_HK_X4
#define FM_HK_X4 1
#endif
__device__ __forceinline__ int hk_row(int v, int t) {
    return FM_HK_X4 ? (v >> 2) * (4 * LT) + 4 * t + (v & 3) : v * LT + t;
}

template <int VPT>
__device__ __forceinline__ void hk_load(const double* col, int L, uint32_t (&hk)[VPT]) {
    if constexpr (FM_HK_X4) {
        static_assert(VPT % 4 == 0, "hk_load: 16-byte slots");
        const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)col, 0, L * 8, 0x00020000);
        const uint32_t lb = (uint32_t)threadIdx.x * 32u + 4u;   // little-endian: byte 4 = high word
#pragma unroll
        for (int v = 0; v < VPT; ++v)
            hk[v] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rs, lb + (uint32_t)(v & 3) * 8u,
                                                                  (v >> 2) * (4 * LT * 8), 0);
    } else {
        const uint32_t lb = (uint32_t)threadIdx.x * 8u + 4u;
#pragma unroll
        for (int v = 0; v < VPT; ++v) {
            const int rem = L - v * LT;   // rows from this slot's first row to the month end
            const int nrec = rem > 0 ? (rem < LT ? rem : LT) * 8 : 0;
            const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)(col + (rem > 0 ? v * LT : 0)), 0, nrec,
                                                              0x00020000);
            hk[v] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rs, lb, 0, 0);
        }
    }
}

// ... or from the high-word plane (4 bytes per value read instead of 8)
template <int VPT>
__device__ __forceinline__ void hk_load_plane(const uint32_t* hp, int L, uint32_t (&hk)[VPT]) {
    if constexpr (FM_HK_X4) {
        const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)hp, 0, L * 4, 0x00020000);
        const uint32_t lb = (uint32_t)threadIdx.x * 16u;
#pragma unroll
        for (int v = 0; v < VPT / 4; ++v) {
            const auto q = __builtin_amdgcn_raw_buffer_load_b128(rs, lb, v * (4 * LT * 4), 0);
            hk[4 * v] = q[0];
            hk[4 * v + 1] = q[1];
            hk[4 * v + 2] = q[2];
            hk[4 * v + 3] = q[3];
        }
    } else {
        const uint32_t lb = (uint32_t)threadIdx.x * 4u;
#pragma unroll
        for (int v = 0; v < VPT; ++v) {
            const int rem = L - v * LT;
            const int nrec = rem > 0 ? (rem < LT ? rem : LT) * 4 : 0;
            const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)(hp + (rem > 0 ? v * LT : 0)), 0, nrec, 0x00020000);
            hk[v] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rs, lb, 0, 0);
        }
    }
}

// v with lane Q's value replaced by the uniform x (one v_writelane)
template <int Q>
__device__ __forceinline__ int writelane(int v, int x) {
    asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(v) : "s"(x), "i"(Q));
    return v;
}

// One (month, column) unit whose raw high words are in hk.
template <int VPT>
__device__ __forceinline__ void hk_unit(const SelArgs& a, int s, int c, uint32_t (&hk)[VPT], LongHkSmem& sm) {
    const int tid = (int)threadIdx.x, lane = lane_id();
    const int w = __builtin_amdgcn_readfirstlane(tid / WAVE);
    const int64_t o = (int64_t)c * a.nseg + s;
    const int64_t r0 = a.seg_off[s];
    const int L = (int)(a.seg_off[s + 1] - r0);
    const PCols col = sel_col(a, c, r0);
    // rows past the month end (read as 0 by the range check) -> HK_NONE; straight-line (a
    // scalar branch per slot split the block and pushed keys into scratch)
    const int lim = L - hk_row(0, tid);
#pragma unroll
    for (int v = 0; v < VPT; ++v) hk[v] = hk_row(v, 0) < lim ? hkey(hk[v]) : HK_NONE;
    // count of valid values (ballots: scalar counts), thread min key and max key (NaN keys are
    // above HK_MAX for the min; +0x1FFFFE moves them below every valid key for the max)
    int cw = 0;
    uint32_t kmn = HK_NONE, kmx2 = 0;
#pragma unroll
    for (int v = 0; v < VPT; ++v) {
        const uint32_t k = hk[v];
        cw += (int)__popcll(__ballot(k <= HK_MAX));
        kmn = min(kmn, k);
        kmx2 = max(kmx2, k + 0x1FFFFEu);
        // in order: otherwise the ballot masks are hoisted (SGPR spills) and every k2 kept
        asm volatile("" : "+s"(cw), "+v"(kmn), "+v"(kmx2));
    }
    const bool tvalid = kmn <= HK_MAX;   // this thread holds a valid value
    const uint32_t kmx = kmx2 - 0x1FFFFEu;
    const uint32_t ua = tvalid ? kmn : HK_NONE;            // lower-tail thread key
    const uint32_t ub = tvalid ? HK_MAX - kmx : HK_NONE;   // upper-tail thread key
    const bool amb = tvalid && (kmn == 0u || kmx == HK_MAX);
    if (tid < 2 * LNW) sm.tot[tid / LNW][tid % LNW] = 0;
    // valid count (low 16 bits per wave: <= 64 * VPT) and ambiguous-key threads, one reduction
    // (the ballot outside the lane-0 select: inside it, it would see lane 0's flag only)
    const int ambw = (int)__popcll(__ballot(amb));
    const int packed = block_sum<LNW>(lane == 0 ? cw + (ambw << 16) : 0, sm.hs.ints);
    const int n = packed & 0xFFFF;
    double lo = NAN, hi = NAN;
    bool ok = (packed >> 16) == 0;
    // phases: thresholds + compaction (cand), then ONE site that gathers the candidates and
    // issues the next unit's loads (every path reaches it), then the sort / merge
    bool cand = false, fast_done = false;   // fast_done: the candidates are in per-wave runs
    int i0 = 0, j0 = 0, i1 = 0, j1 = 0, clo = 0, chi = 0;
    double g0 = 0.0, g1 = 0.0;
#if FM_HK_ABL == 3
    lo = -1.0; hi = 1.0;
    if (false) {
#else
    if (ok && n >= a.min_count && n > 0) {   // block-uniform
#endif
        qranks(n, a.q_lo, a.lerp_mode, i0, j0, g0);
        qranks(n, a.q_hi, a.lerp_mode, i1, j1, g1);
        const int kl = j0, ku = n - 1 - i1;        // largest ranks needed from either end
        const int ql = kl / LNW + 1, qu = ku / LNW + 1;
        ok = ql <= WAVE && qu <= WAVE;
        uint32_t tl = HK_NONE, tu = HK_NONE;
        if (ok) {
#if FM_HK_KTH
            uint32_t ta, tb;   // the ql-th / qu-th smallest lane key, by bisection
            wave_kth_u32x2(ua, ql, ub, qu, ta, tb);
            if (lane == 0) {
                sm.tw[0][w] = ta;
                sm.tw[1][w] = tb;
            }
#else
            uint32_t ha[1] = {ua}, hb[1] = {ub};
            wave_sort32<1>(ha);
            wave_sort32<1>(hb);
            if (lane == 0) {
                sm.tw[0][w] = (uint32_t)__builtin_amdgcn_readlane((int)ha[0], ql - 1);
                sm.tw[1][w] = (uint32_t)__builtin_amdgcn_readlane((int)hb[0], qu - 1);
            }
#endif
            __syncthreads();
            // this wave's count under each wave's threshold, lane q holding threshold q's, one
            // LDS add per lane (a threshold of HK_NONE is never taken: its count is moot)
            int pa = 0, pb = 0;
            static_for<0, LNW>([&](auto qc) {
                constexpr int q = decltype(qc)::value;
                const uint32_t Ta = sm.tw[0][q], Tb = sm.tw[1][q];
                const int ca = (int)__popcll(__ballot(ua <= Ta)), cb = (int)__popcll(__ballot(ub <= Tb));
                pa = writelane<q>(pa, ca);
                pb = writelane<q>(pb, cb);
            });
            if (lane < LNW) {
                atomicAdd(&sm.tot[0][lane], pa);
                atomicAdd(&sm.tot[1][lane], pb);
            }
            __syncthreads();
#pragma unroll
            for (int q = 0; q < LNW; ++q) {
                const uint32_t Ta = sm.tw[0][q], Tb = sm.tw[1][q];
                if (Ta != HK_NONE && sm.tot[0][q] >= kl + 1 && Ta < tl) tl = Ta;
                if (Tb != HK_NONE && sm.tot[1][q] >= ku + 1 && Tb < tu) tu = Tb;
            }
            ok = tl != HK_NONE && tu != HK_NONE;
        }
#if FM_HK_ABL == 1
        if (ok) { lo = -1.0; hi = 1.0; fast_done = true; }
        if (false) {
#else
        if (ok && FM_HK_WAVELIST) {
#endif
            // candidates straight into per-wave lists: wave w writes its lower-tail rows to
            // cidx[64 w ..] and its upper-tail rows to cidx[LCAP + 64 w ..] (re-indexed into
            // 64-candidate runs at the gather below), no count pass for list offsets first.  A
            // wave holding more than 64 candidates of a tail (its writes wrap inside its own
            // list), or too many in all, sends the unit to the counted compaction with the
            // threshold refinement below, which rewrites every list.
            int wl = 0, wh = 0;
#pragma unroll
            for (int v = 0; v < VPT; ++v) {
                const uint32_t k = hk[v];
                const bool bl = k <= tl, bh = HK_MAX - k <= tu;
                const uint64_t ml = __ballot(bl), mh = __ballot(bh);
                if (ml) {   // wave-uniform
                    const int p = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(ml >> 32),
                                                                 __builtin_amdgcn_mbcnt_lo((uint32_t)ml, (uint32_t)wl));
                    if (bl) sm.cidx[w * WAVE + (p & (WAVE - 1))] = hk_row(v, tid);
                    wl += (int)__popcll(ml);
                }
                if (mh) {
                    const int p = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(mh >> 32),
                                                                 __builtin_amdgcn_mbcnt_lo((uint32_t)mh, (uint32_t)wh));
                    if (bh) sm.cidx[LCAP + w * WAVE + (p & (WAVE - 1))] = hk_row(v, tid);
                    wh += (int)__popcll(mh);
                }
            }
            if (lane == 0) {
                sm.wc[0][w] = wl;
                sm.wc[1][w] = wh;
            }
            __syncthreads();
            bool over = false;
            clo = chi = 0;
#pragma unroll
            for (int q = 0; q < LNW; ++q) {
                const int a0 = sm.wc[0][q], a1 = sm.wc[1][q];
                over = over || a0 > WAVE || a1 > WAVE;
                clo += a0;
                chi += a1;
            }
            fast_done = !over && clo + chi <= n && clo > kl && chi > ku;   // block-uniform
            if (fast_done) cand = true;
            else __syncthreads();   // every read of sm.wc above before the counted path rewrites it
        }
        if (ok && !fast_done) {
            // candidates: key <= tl (a prefix of the sorted values) / HK_MAX - key <= tu (a
            // suffix); NaN keys fail both (the subtraction wraps them above every tu)
            int ol = 0, oh = LCAP;
            for (int pass = 0; pass < 2; ++pass) {   // a second pass only after a refinement
                int wl = 0, wh = 0;
#pragma unroll
                for (int v = 0; v < VPT; ++v) {
                    uint32_t k = hk[v];
                    asm volatile("" : "+v"(k));   // no values derived in the count loop kept for here
                    wl += (int)__popcll(__ballot(k <= tl));
                    wh += (int)__popcll(__ballot(HK_MAX - k <= tu));
                    asm volatile("" : "+s"(wl), "+s"(wh));   // counts in order (no spilled masks)
                }
                if (lane == 0) {
                    sm.wc[0][w] = wl;
                    sm.wc[1][w] = wh;
                }
                __syncthreads();
                ol = 0;
                oh = LCAP;
                clo = chi = 0;
#pragma unroll
                for (int q = 0; q < LNW; ++q) {
                    const int a0 = sm.wc[0][q], a1 = sm.wc[1][q];
                    ol += q < w ? a0 : 0;
                    oh += q < w ? a1 : 0;
                    clo += a0;
                    chi += a1;
                }
                if (pass == 1 || !((clo > LCAP || chi > LCAP) && clo > kl && chi > ku)) break;   // block-uniform
                // more candidates than a list holds (the thread-minimum thresholds can overshoot
                // by hundreds): the smallest threshold whose VALUE count still reaches the rank,
                // by bisection on the keys (block counts; a few passes over the registers),
                // then recount -- instead of sending the unit to the streaming fix-up
                auto count_le = [&](uint32_t T, bool upper) -> int {
                    int c = 0;
#pragma unroll
                    for (int v = 0; v < VPT; ++v) {
                        uint32_t k = hk[v];
                        asm volatile("" : "+v"(k));
                        c += (int)__popcll(__ballot(upper ? HK_MAX - k <= T : k <= T));
                        asm volatile("" : "+s"(c));
                    }
                    return block_sum<LNW>(lane == 0 ? c : 0, sm.hs.ints);
                };
                auto refine = [&](uint32_t& T, int& cnt, int need, bool upper) {
                    uint32_t lo = 0, hi = T;
                    while (cnt > LCAP && lo < hi) {   // block-uniform
                        const uint32_t mid = lo + (hi - lo) / 2;
                        const int c = count_le(mid, upper);
                        if (c >= need) {
                            hi = mid;
                            cnt = c;
                        } else {
                            lo = mid + 1;
                        }
                    }
                    T = hi;
                };
                if (clo > LCAP) refine(tl, clo, kl + 1, false);
                if (chi > LCAP) refine(tu, chi, ku + 1, true);
                __syncthreads();   // every pass-0 read of sm.wc before the recount rewrites it
            }
            ok = clo <= LCAP && chi <= LCAP && clo + chi <= n && clo > kl && chi > ku;
            if (ok) {
#pragma unroll
                for (int v = 0; v < VPT; ++v) {
                    uint32_t k = hk[v];
                    asm volatile("" : "+v"(k));
                    const bool bl = k <= tl, bh = HK_MAX - k <= tu;
                    const uint64_t ml = __ballot(bl), mh = __ballot(bh);
                    const int row = hk_row(v, tid);
                    if (ml) {   // wave-uniform: most value slots hold no candidate
                        if (bl) sm.cidx[ol + mask_rank(ml)] = row;
                        ol += (int)__popcll(ml);
                    }
                    if (mh) {
                        if (bh) sm.cidx[oh + mask_rank(mh)] = row;
                        oh += (int)__popcll(mh);
                    }
                }
                __syncthreads();
                cand = true;
            }
        }
    }
#if FM_HK_ABL == 2
    if (cand) { lo = -1.0; hi = 1.0; cand = false; }
#endif
    if (cand) {   // block-uniform
        // gather the candidates' full values (a few hundred rows of the unit just read); wave
        // w sorts run w of each tail (64 keys; the upper tail on complemented keys), then every
        // candidate's merged rank = its run position + the entries of the other runs before it.
        // (Ordering the candidates by (high key, row) first and gathering only the tie groups at
        // the target ranks measured slower: 0.91-1.0 vs 0.66 ms on 1,000 x 20,000 x 15.)
        // candidate e of the merged list: cidx[e], or with per-wave runs the (e - prefix)-th
        // entry of the last wave whose count prefix is <= e (scalar prefixes, a few selects)
        const int e = w * WAVE + lane;
        const int nrl = __builtin_amdgcn_readfirstlane((clo + WAVE - 1) / WAVE);
        const int nru = __builtin_amdgcn_readfirstlane((chi + WAVE - 1) / WAVE);
        int il = e, iu = e;
        if (fast_done) {   // block-uniform
            int pl = 0, pu = 0;
#pragma unroll
            for (int q = 0; q < LNW; ++q) {
                if (e >= pl) il = e + (q * WAVE - pl);
                if (e >= pu) iu = e + (q * WAVE - pu);
                pl += sm.wc[0][q];
                pu += sm.wc[1][q];
            }
        }
        const bool vl = e < clo, vu = e < chi;
        const int rl = vl ? sm.cidx[il] : 0, ru = vu ? sm.cidx[LCAP + iu] : 0;
        const double xl = col[rl], xu = col[ru];
        uint64_t ka[1] = {vl ? dkey(xl) : SENT};
        uint64_t kb[1] = {vu ? ~dkey(xu) : SENT};
        if (w < nrl) wave_sort<1>(ka);
        if (w < nru) wave_sort<1>(kb);
        sm.ck[e] = ka[0];
        sm.ck[LCAP + e] = kb[0];
        if (tid < 4) sm.res[tid] = SENT;
        __syncthreads();
        // both tails' searches of run u side by side (independent LDS chains); a run past a
        // tail's count is all SENT and adds 0; SENT lanes count garbage and store nothing
        const int nr = nrl > nru ? nrl : nru;
        int ra = lane, rb = lane;
#pragma unroll
        for (int u = 0; u < LNW; ++u) {
            if (u < nr && u != w) {   // wave-uniform
                ra += merge_count(sm.ck + u * WAVE, ka[0], u < w);
                rb += merge_count(sm.ck + LCAP + u * WAVE, kb[0], u < w);
            }
        }
        if (ka[0] != SENT) {
            if (ra == i0) sm.res[0] = ka[0];
            if (ra == j0) sm.res[1] = ka[0];
        }
        if (kb[0] != SENT) {
            if (rb == n - 1 - i1) sm.res[2] = ~kb[0];
            if (rb == n - 1 - j1) sm.res[3] = ~kb[0];
        }
        __syncthreads();
        lo = qlerp(kval(sm.res[0]), kval(sm.res[1]), g0, a.lerp_mode);
        hi = qlerp(kval(sm.res[2]), kval(sm.res[3]), g1, a.lerp_mode);
    }
    if (!ok) {   // redone by the fix-up kernel
        if (tid == 0) sel_mark(a, o);
    } else {
        if (a.center != nullptr) {
            // Gram pivot: the midpoint of the cuts, else of the finite range (no +-inf here:
            // those units were marked above), else 0 -- the range re-read in full (rare: too
            // few values)
            double cen = 0.5 * (lo + hi);
            if (!isfinite(cen)) {   // block-uniform
                uint64_t m1 = SENT, m2 = SENT;
                for (int r = tid; r < L; r += LT) {
                    const double x = col[r];
                    if (isfinite(x)) {
                        m1 = dkey(x) < m1 ? dkey(x) : m1;
                        m2 = ~dkey(x) < m2 ? ~dkey(x) : m2;
                    }
                }
                m1 = block_min_u64<LNW>(m1, sm.hs.u64s);
                m2 = block_min_u64<LNW>(m2, sm.hs.u64s + LNW);
                cen = m1 == SENT || m2 == SENT ? 0.0 : 0.5 * (kval(m1) + kval(~m2));
                if (!isfinite(cen)) cen = 0.0;
            }
            if (tid == 0) a.center[o] = cen;
        }
        if (tid == 0) {
            a.lo[o] = lo;
            a.hi[o] = hi;
            a.nvalid[o] = n;
            if (zero_cut(a, lo, hi)) sel_push(a, o);
        }
    }
    __syncthreads();   // the LDS is rewritten by the next unit
}

// One unit per workgroup (grid months x (columns [+ 1 riding universe column])): 80 VGPRs, three
// workgroups per CU; the hardware refills a CU slot as a unit ends.  (A persistent grid with
// the next unit's loads in flight during the sort and merge measured slower: 0.75-0.79 vs
// 0.66 ms on the 1,000 x 20,000 x 15 panel, two workgroups per CU at 128 VGPRs.)
template <int VPT>
__global__ __launch_bounds__(LT, 6) void select_long_hk_kernel(SelArgs a) {
    __shared__ LongHkSmem sm;
    const int s = blockIdx.x, c = blockIdx.y;
    if (FM_HK_RIDE && c == a.ncols) {   // fm_select_universe: the month's NYSE breakpoints + levels
        universe_month_wg<LNW, HB, HCAP>(a, s, sm.hs);
        return;
    }
    uint32_t hk[VPT];
    if (a.hp != nullptr)
        hk_load_plane<VPT>(a.hp + (int64_t)c * a.pstride + a.seg_off[s], (int)(a.seg_off[s + 1] - a.seg_off[s]), hk);
    else
        hk_load<VPT>(a.cols + (int64_t)c * a.col_stride + a.seg_off[s], (int)(a.seg_off[s + 1] - a.seg_off[s]), hk);
    hk_unit<VPT>(a, s, c, hk, sm);
}


template <int VPT>
void launch_long(const SelArgs& a, hipStream_t st, bool mid) {
    if (mid)
        hipLaunchKernelGGL((select_long_kernel<VPT, true>), dim3(a.nseg, a.ncols), dim3(LT), 0, st, a);
    else if (FM_AB_LONG_F64 || FM_AB_LONG != 0)   // with a universe (a.ume), one more grid column
        hipLaunchKernelGGL((select_long_kernel<VPT, false>), dim3(a.nseg, a.ncols + (a.ume ? 1 : 0)), dim3(LT), 0,
                           st, a);
    else   // with a universe (a.ume), one more grid column: its months' NYSE breakpoints
        hipLaunchKernelGGL((select_long_hk_kernel<VPT>), dim3(a.nseg, a.ncols + (a.ume ? 1 : 0)), dim3(LT), 0, st, a);
}

// the tail thresholds serve ranks < 512 from either end; row masks and middle ranks take the
// histogram over all values (the MID kernel)
bool long_is_mid(const SelArgs& a, int max_seg_len) {
    const double span = (double)(max_seg_len > 0 ? max_seg_len - 1 : 0);
    return a.mask != nullptr || a.q_lo * span + 2.0 > (double)LT || (1.0 - a.q_hi) * span + 2.0 > (double)LT;
}

int launch_select_long(const SelArgs& a, int max_seg_len, hipStream_t st) {
    const int vpt = (max_seg_len + LT - 1) / LT;
    const bool mid = long_is_mid(a, max_seg_len);
    if (vpt <= 16) launch_long<16>(a, st, mid);
    else if (vpt <= 24) launch_long<24>(a, st, mid);
    else if (vpt <= 32) launch_long<32>(a, st, mid);
    else if (vpt <= LONG_VPT) launch_long<LONG_VPT>(a, st, mid);
    else {
        set_error("select long kernel: %d-row segments exceed %d", max_seg_len, LONG_VPT * LT);
        return FM_ETOOBIG;
    }
    return FM_OK;
}

template <int VPT>
void launch_select(const SelArgs& a, int ncols, hipStream_t st) {
    hipLaunchKernelGGL((select_kernel<VPT>), dim3(a.nseg, ncols), dim3(ST), 0, st, a);
}

__device__ __forceinline__ int64_t unit_of(const SelArgs& a, int64_t k) {
    const int64_t s = k / a.ncols, c = k - s * a.ncols;
    return c * a.nseg + s;
}

template <int VPL>
__device__ __forceinline__ int load_unit(const SelArgs& a, int64_t u, double (&xv)[VPL]) {
    const int s = (int)(u % a.nseg), c = (int)(u / a.nseg);
    const int64_t r0 = a.seg_off[s];
    const int L = (int)(a.seg_off[s + 1] - r0);
    load_seg_col<VPL>(a.cols + (int64_t)c * a.col_stride + r0, L, xv);
    return L;
}

// Persistent waves, software-pipelined over units u = gw, gw + nwaves, ...: the loads of the
// next unit are issued as soon as this unit's candidates are compacted into LDS, so they
// overlap the candidate sorts, the lerp and the stores (without the moments pass, which
// needs the values; then they are issued after it).
template <int VPL, bool EARLY>
__global__ __launch_bounds__(ST, 2) void select_wave_kernel(SelArgs a) {
    __shared__ double cbuf[SNW][2][WCAP];   // per wave: lower / upper tail candidates
    const int lane = lane_id();
    const int w = __builtin_amdgcn_readfirstlane((int)threadIdx.x / WAVE);
    const int64_t nunits = (int64_t)a.nseg * a.ncols;
    const int64_t nwt = (int64_t)gridDim.x * SNW;
    // Work order is month-major (k -> month k / ncols, column k % ncols) so the panel is
    // streamed month by month, the order fm_gram then reads back in reverse (its first
    // months are this kernel's last, still in the memory-side cache); outputs stay indexed
    // by u = column * nseg + month.
    int64_t k = (int64_t)blockIdx.x * SNW + w;
    if (k >= nunits) return;   // wave-uniform; no block barriers below
    int64_t u = unit_of(a, k);
    constexpr bool early = EARLY;   // no moments pass: prefetch right after compaction
    double xv[VPL];
    int L = load_unit<VPL>(a, u, xv);
    __builtin_amdgcn_sched_barrier(0);
    double* Ll = cbuf[w][0];
    double* Lh = cbuf[w][1];
    while (true) {
        const int64_t kn = k + nwt;
        const bool more = kn < nunits;
        const int64_t un = more ? unit_of(a, kn) : 0;
        int Ln = 0;
        const WaveCut r = wave_cut<VPL>(xv, L, a.q_lo, a.q_hi, a.min_count, a.lerp_mode, Ll, Lh, [&] {
            if (early && more) Ln = load_unit<VPL>(a, un, xv);
        });
        const double lo = r.lo, hi = r.hi, mn = r.mn;
        const int n = r.n;
        const bool ok = r.ok;
        if (!ok) {
            if (lane == 0) sel_mark(a, u);   // redone by the fix-up kernel
        } else {
            if (a.center != nullptr && lane == 0) a.center[u] = r.cen;
            if (!early) {
                // moments of the clipped values about a pivot inside the data (see
                // select_unit_wg)
                double p = isfinite(lo) ? lo : (isfinite(hi) ? hi : 0.0);
                if (!isfinite(lo) && !isfinite(hi)) {
                    double m2 = isfinite(mn) ? mn : NAN;
#pragma unroll
                    for (int o = 32; o > 0; o >>= 1) m2 = fmin(m2, __shfl_xor(m2, o, WAVE));
                    p = isfinite(m2) ? m2 : 0.0;
                }
                double s1 = 0.0, s2 = 0.0;
                if (isfinite(lo) && !isnan(hi)) {
                    // p == lo: hardware max/min send a NaN (absent) value to lo, so it adds
                    // d == 0 exactly; the same d as the general loop for every present value
#pragma unroll
                    for (int v = 0; v < VPL; ++v) {
                        const double d = hw_min(hw_max(xv[v], lo), hi) - lo;
                        s1 += d;
                        s2 = fma(d, d, s2);
                    }
                } else {
#pragma unroll
                    for (int v = 0; v < VPL; ++v) {
                        double x = xv[v];
                        if (x < lo) x = lo;
                        if (x > hi) x = hi;
                        const double d = isnan(x) ? 0.0 : x - p;
                        s1 += d;
                        s2 = fma(d, d, s2);
                    }
                }
                s1 = wave_sum(s1);
                s2 = wave_sum(s2);
                if (lane == 0) {
                    a.mean[u] = n > 0 ? p + s1 / (double)n : NAN;
                    if (a.sd) {
                        double var = n > 1 ? (s2 - s1 * (s1 / (double)n)) / (double)(n - 1) : NAN;
                        if (var < 0.0) var = 0.0;
                        a.sd[u] = n > 1 ? sqrt(var) : NAN;
                    }
                }
            }
            if (lane == 0) {
                a.lo[u] = lo;
                a.hi[u] = hi;
                if (a.nvalid) a.nvalid[u] = n;
                if (zero_cut(a, lo, hi)) sel_push(a, u);
            }
        }
        if (!more) break;
        if (!early) Ln = load_unit<VPL>(a, un, xv);
        k = kn;
        u = un;
        L = Ln;
    }
}

// ---------------------------------------------------------------------------------------
// Two waves per (segment, column) unit (a 128-thread workgroup per unit at a time): each wave
// holds HALF the segment (rows (2v + h) * 64 + lane), so a wave needs half the registers of
// select_wave_kernel, four waves per SIMD fit, and each wave sorts ONE tail:
//   1. per wave: count, lane minima / maxima, the 64 lane-minimum high words sorted (and the
//      complemented lane-maximum high words), all published in LDS;
//   2. wave 0: T_lo = the j0-th smallest of the 128 lane-minimum high words (merge ranks of
//      two sorted lists by binary search) and tau_lo = the largest lane minimum (of either
//      wave) with that high word; wave 1 the same for the upper tail;
//   3. per wave: values < tau_lo / > tau_hi compacted into its own LDS lists; the next
//      unit's loads are issued here;
//   4. wave 0 sorts the two low-tail lists together and reads ranks i0, j0; wave 1 the high
//      tail.
// A unit the tail path cannot decide (ranks >= 128, candidate overflow: rare for 1/99
// cuts) is marked (nvalid = -1) and redone by the workgroup kernel's fallback pass.  Keeping
// the histogram select out of this kernel keeps its register count (the values are held in
// registers) at the level the hot path needs.
struct PairSmem {
    uint32_t sk[2][2][WAVE];   // [wave][lo / hi][lane] sorted high words
    double ext[2][2][WAVE];    // [wave][min / max][lane] lane extrema
    double cand[2][2][WCAP];   // [wave][lo / hi] tail candidates
    int ni[2][4];
    double tv[2];
    double res[2];
    int okv[2];
};

template <int VPH>
__global__ __launch_bounds__(2 * WAVE) void select_pair_kernel(SelArgs a) {
    __shared__ PairSmem sm;
    const int lane = lane_id();
    const int h = __builtin_amdgcn_readfirstlane((int)threadIdx.x / WAVE);
    const int64_t nunits = (int64_t)a.nseg * a.ncols;
    int64_t k = blockIdx.x;
    if (k >= nunits) return;   // block-uniform
    // unit k = (month k / ncols, column k % ncols), walked by (month, column) steps of the
    // grid size: no 64-bit division per unit (unit_of's emulated divisions cost ~45 scalar /
    // vector instructions each, four per unit)
    const int ncols = a.ncols;
    const int G = (int)gridDim.x;
    const int dS = G / ncols, dC = G - (G / ncols) * ncols;
    int s_cur = (int)blockIdx.x / ncols;
    int c_cur = (int)blockIdx.x - s_cur * ncols;
    double xv[VPH];
    auto load = [&](int s, int c) -> int {
        const double* base = a.cols + (int64_t)c * a.col_stride;
        const int64_t r0 = a.seg_off[s];
        const int L = (int)(a.seg_off[s + 1] - r0);
        typedef const __attribute__((address_space(1))) char* gptr;
        const gptr b = (gptr)(base + r0);
        const uint32_t lastb = (uint32_t)(L > 0 ? L - 1 : 0) * 8u;
        uint32_t lb = (uint32_t)(h * WAVE + lane) * 8u;
        asm volatile("" : "+v"(lb));
#pragma unroll
        for (int v = 0; v < VPH; ++v) {
            const uint32_t off = lb + (uint32_t)(v * 2 * WAVE * 8);
            xv[v] = *(const __attribute__((address_space(1))) double*)(b + (off < lastb ? off : lastb));
        }
        return L;
    };
    // finite min / max of this wave's half of unit u, re-read from memory: only the rare
    // pivot fallback (no finite cut midpoint) needs it, and by then xv holds the next unit
    auto finite_range = [&](int s, int c, double& m1, double& m2) {
        const PCols base = sel_col(a, c, a.seg_off[s]);
        const int Lu = (int)(a.seg_off[s + 1] - a.seg_off[s]);
        m1 = NAN;
        m2 = NAN;
        for (int r = h * WAVE + lane; r < Lu; r += 2 * WAVE) {
            const double x = base[r];
            m1 = hw_min(m1, isfinite(x) ? x : NAN);
            m2 = hw_max(m2, isfinite(x) ? x : NAN);
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            m1 = hw_min(m1, xor_lanes_f64(m1, o));
            m2 = hw_max(m2, xor_lanes_f64(m2, o));
        }
    };
    int L = load(s_cur, c_cur);
    while (true) {
        const int64_t u = (int64_t)c_cur * a.nseg + s_cur;
        const int64_t kn = k + gridDim.x;
        const bool more = kn < nunits;
        int s_nx = s_cur + dS, c_nx = c_cur + dC;
        if (c_nx >= ncols) {
            c_nx -= ncols;
            ++s_nx;
        }
        int Ln = 0;
        int row0 = h * WAVE + lane;
        asm volatile("" : "+v"(row0));
        // ---- 1. this wave's half: count, lane extrema (NaN = absent / masked out)
        int nh = 0;
        double mn4[4] = {NAN, NAN, NAN, NAN}, mx4[4] = {NAN, NAN, NAN, NAN};
        // slots past the segment end -> NaN; only the slots past the unit's full 128-row
        // groups can hold such rows (a scalar branch per slot, kept a branch by the asm)
        const int vf = FM_AB_PAIR_MASKALL ? 0 : L / (2 * WAVE);
#pragma unroll
        for (int v = 0; v < VPH; ++v) {
            if (v >= vf) {
                double x = xv[v];
                asm volatile("" : "+v"(x));
                xv[v] = row0 + v * 2 * WAVE >= L ? (double)NAN : x;
            }
            const double x = xv[v];
            nh += (int)__popcll(__ballot(!isnan(x)));
            mn4[v & 3] = hw_min(mn4[v & 3], x);
            mx4[v & 3] = hw_max(mx4[v & 3], x);
        }
        const double mn = hw_min(hw_min(mn4[0], mn4[1]), hw_min(mn4[2], mn4[3]));
        const double mx = hw_max(hw_max(mx4[0], mx4[1]), hw_max(mx4[2], mx4[3]));
        nh = __builtin_amdgcn_readfirstlane(nh);
        const double q_lo = a.q_lo, q_hi = a.q_hi;
        const int mode = a.lerp_mode;
        const int minc = a.min_count;
        {
            const uint32_t ha = isnan(mn) ? 0xFFFFFFFFu : (uint32_t)(dkey(mn) >> 32);
            const uint32_t hb = isnan(mx) ? 0xFFFFFFFFu : (uint32_t)(~dkey(mx) >> 32);
            uint32_t ta[1] = {ha}, tb[1] = {hb};
            wave_sort32<1>(ta);
            wave_sort32<1>(tb);
            sm.sk[h][0][lane] = ta[0];
            sm.sk[h][1][lane] = tb[0];
            sm.ext[h][0][lane] = mn;
            sm.ext[h][1][lane] = mx;
        }
        if (lane == 0) sm.ni[h][0] = nh;
        __syncthreads();
        const int n = sm.ni[0][0] + sm.ni[1][0];
        const bool apply = n >= minc && n > 0;
        int i0 = 0, j0 = 0, i1 = 0, j1 = 0;
        double g0 = 0.0, g1 = 0.0;
        if (apply) {
            qranks(n, q_lo, mode, i0, j0, g0);
            qranks(n, q_hi, mode, i1, j1, g1);
        }
        bool ok = apply;
        if (ok) {
            // ---- 2. this wave's tail: h == 0 low (rank j0 over lane minima), h == 1 high
            const int kr = h == 0 ? j0 : n - 1 - i1;
            ok = kr < 2 * WAVE;
            if (ok) {
                const int t = h;   // list kind
                const uint32_t mine = sm.sk[0][t][lane], other = sm.sk[1][t][lane];
                // merged ranks: entries of list 0 precede equal entries of list 1
                const int r0 = lane + count_below_u32(sm.sk[1][t], mine, false);
                const int r1 = lane + count_below_u32(sm.sk[0][t], other, true);
                uint32_t T = 0xFFFFFFFFu;
                const uint64_t m0 = __ballot(r0 == kr), m1 = __ballot(r1 == kr);
                if (m0) T = (uint32_t)__builtin_amdgcn_readlane((int)mine, __builtin_ctzll(m0));
                else if (m1) T = (uint32_t)__builtin_amdgcn_readlane((int)other, __builtin_ctzll(m1));
                ok = T != 0xFFFFFFFFu;
                // tau: the extreme lane extremum (either wave) whose high word is T
                double best = NAN;
#pragma unroll
                for (int w2 = 0; w2 < 2; ++w2) {
                    const double e = sm.ext[w2][t][lane];
                    const uint32_t hw = isnan(e) ? 0xFFFFFFFFu
                                                 : (t == 0 ? (uint32_t)(dkey(e) >> 32) : (uint32_t)(~dkey(e) >> 32));
                    const double cv = hw == T ? e : NAN;
                    best = t == 0 ? hw_max(best, cv) : hw_min(best, cv);
                }
#pragma unroll
                for (int o = 32; o > 0; o >>= 1)
                    best = t == 0 ? hw_max(best, xor_lanes_f64(best, o)) : hw_min(best, xor_lanes_f64(best, o));
                if (lane == 0) sm.tv[h] = best;
            }
            if (lane == 0) sm.okv[h] = ok ? 1 : 0;
            __syncthreads();
            ok = sm.okv[0] != 0 && sm.okv[1] != 0;   // block-uniform
        }
        double lo = NAN, hi = NAN;
        bool prefetched = false;
        if (ok) {
            // ---- 3. compaction of this wave's half into its own lists
            int clo = 0, chi = 0;
            const double tlo = sm.tv[0], thi = sm.tv[1];
            double* Ll = sm.cand[h][0];
            double* Lh = sm.cand[h][1];
#pragma unroll
            for (int v = 0; v < VPH; ++v) {
                const bool bl = xv[v] < tlo, bh = xv[v] > thi;
                const uint64_t ml = __ballot(bl), mh = __ballot(bh);
                if (ml) {
                    if (bl) Ll[(clo + mask_rank(ml)) & (WCAP - 1)] = xv[v];
                    clo += (int)__popcll(ml);
                }
                if (mh) {
                    if (bh) Lh[(chi + mask_rank(mh)) & (WCAP - 1)] = -xv[v];   // ascending
                    chi += (int)__popcll(mh);
                }
            }
            if (lane == 0) {
                sm.ni[h][1] = clo;
                sm.ni[h][2] = chi;
            }
            // xv is dead from here on: the next unit's loads fly during the candidate sorts
            if (more) Ln = load(s_nx, c_nx);
            prefetched = true;
            __syncthreads();
            // ---- 4. one tail per wave over both halves' candidates
            const int t = h;
            const int c0 = sm.ni[0][1 + t], c1 = sm.ni[1][1 + t];
            const int cc = c0 + c1;
            const bool fits = c0 <= WCAP && c1 <= WCAP && cc <= 4 * WAVE;
            if (fits) {
                double va = NAN, vb = NAN;
                const int ra = t == 0 ? i0 : n - 1 - j1, rb = t == 0 ? j0 : n - 1 - i1;
                const double tau = t == 0 ? sm.tv[0] : -sm.tv[1];
                if (cc <= 2 * WAVE) pick_tail2<2>(sm.cand[0][t], c0, sm.cand[1][t], c1, ra, rb, tau, va, vb);
                else pick_tail2<4>(sm.cand[0][t], c0, sm.cand[1][t], c1, ra, rb, tau, va, vb);
                if (lane == 0) sm.res[h] = t == 0 ? qlerp(va, vb, g0, mode) : qlerp(-vb, -va, g1, mode);
            }
            if (lane == 0) sm.okv[h] = fits ? 1 : 0;
            __syncthreads();
            ok = sm.okv[0] != 0 && sm.okv[1] != 0;   // block-uniform
            lo = sm.res[0];
            hi = sm.res[1];
        }
        if (apply && !ok) {
            // redone by the fix-up kernel
            if (threadIdx.x == 0) sel_mark(a, u);
        } else if (h == 0) {
            double cen = 0.5 * (lo + hi);
            if (!isfinite(cen)) {
                double m1, m2;
                finite_range(s_cur, c_cur, m1, m2);
                if (lane == 0) sm.res[0] = m1, sm.res[1] = m2;
            }
            if (lane == 0) {
                if (a.center && isfinite(cen)) a.center[u] = cen;
                a.lo[u] = lo;
                a.hi[u] = hi;
                if (a.nvalid) a.nvalid[u] = n;
                if (zero_cut(a, lo, hi)) sel_push(a, u);
            }
        } else if (!isfinite(0.5 * (lo + hi))) {
            // wave 1's half of the finite range for the pivot fallback
            double m1, m2;
            finite_range(s_cur, c_cur, m1, m2);
            if (lane == 0) sm.tv[0] = m1, sm.tv[1] = m2;
        }
        if (more && !prefetched) Ln = load(s_nx, c_nx);   // the next unit's loads fly across the barrier
        __syncthreads();
        if ((ok || !apply) && a.center && !isfinite(0.5 * (lo + hi)) && threadIdx.x == 0) {
            // pivot fallback: the midpoint of the finite range (both halves), else 0
            const double m1 = hw_min(sm.res[0], sm.tv[0]), m2 = hw_max(sm.res[1], sm.tv[1]);
            double cen = 0.5 * (m1 + m2);
            a.center[u] = isfinite(cen) ? cen : 0.0;
        }
        __syncthreads();   // LDS state is rewritten by the next unit
        if (!more) break;
        k = kn;
        s_cur = s_nx;
        c_cur = c_nx;
        L = Ln;
    }
}


// ---------------------------------------------------------------------------------------
// Two-wave units on the HIGH-WORD plane (fm_select_args.hi_plane: the panel's high 32 bits,
// fm_split_planes): select_pair_kernel's structure with every step before the final pick on
// 32-bit order keys (hkey), so a unit reads half the bytes and holds half the registers:
//   1. per wave: valid count, lane min / max keys (a lane holding +-inf or a NaN whose payload
//      is all in the low word -- keys 0 / HK_MAX -- sends the unit to the fix-up kernel);
//   2. wave 0 / 1: T = the kr-th smallest of the 128 lane-extreme keys of its tail, so at
//      least kr + 1 values have keys <= T: the values with key <= T are a prefix of the sorted
//      order holding both target ranks;
//   3. per wave: (key, row) of those values compacted to LDS, both tails; the next unit's
//      loads are issued here;
//   4. wave t sorts tail t's candidates by (key, row) and gathers the FP64 values at the two
//      target ranks from the column (4 scattered loads per unit); when high words tie at those
//      ranks every tied candidate is gathered and the tie broken by the full keys.
// resident two-wave workgroups per CU (the register budget and the persistent grid): the keys
// take VPH VGPRs beside ~70 for the rest (the next unit's keys are in flight during the pick)
#ifndef FM_PAIR_HK_WGS
#define FM_PAIR_HK_WGS 0   // 0: by VPH
#endif
// 1: the next unit's loads are issued before the pick (its keys then stay live through it)
#ifndef FM_PAIR_HK_PF
#define FM_PAIR_HK_PF 1
#endif
// 1: the valid-key count as a per-lane carry count and one wave sum (0: a ballot per value)
#ifndef FM_PAIR_HK_LANECNT
#define FM_PAIR_HK_LANECNT 1
#endif
constexpr int pair_hk_wgs(int vph) {
    return FM_PAIR_HK_WGS > 0 ? FM_PAIR_HK_WGS : (vph <= 16 ? 12 : (vph <= 24 ? 10 : 8));
}
struct PairHkSmem {
    uint32_t sk[2][2][WAVE];     // [wave][lo / hi][lane] sorted lane-extreme keys
    uint64_t cand[2][2][WCAP];   // [wave][lo / hi] (key << 32 | row) candidates
    int ni[2][4];
    uint32_t tv[2];
    double res[2];
    double fr[2];   // wave 1's half of the finite range (pivot fallback)
    int okv[2];
};

// Values at ranks ra <= rb (rb <= ra + 1) of one tail's candidates L1 ++ L2 (c <= 64 R,
// (key << 32 | row) each); tail 1 holds complemented keys (ranks from the top).  Only the
// 32-bit keys are sorted (wave_sort32: a DPP exchange, min, max and lane-mask select per
// register and stage); the keys at the two ranks are read back by readlane, and when each of
// them belongs to exactly one candidate its row is found in the UNSORTED list by one ballot
// per register, so the rows never travel through the sort.  When high words tie at the
// target ranks, every tied candidate's full value is gathered and those are sorted (rare).
// (Round 5 sorted the 64-bit (key, row) words: about 650 VALU per wave for R = 2 against
// about 230 here.)  false: cannot decide (never expected).
template <int R>
__device__ __forceinline__ bool pick_hk(uint64_t* L1, int c1, const uint64_t* L2, int c2, int ra, int rb, int tail,
                                        const PCols col, double& va, double& vb) {
    const int lane = lane_id();
    const int c = c1 + c2;
    uint32_t key[R], row[R], sk[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int e = lane + WAVE * r;
        const uint64_t x = e < c1 ? L1[e] : (e < c ? L2[e - c1] : SENT);
        key[r] = (uint32_t)(x >> 32);   // padding: 0xFFFFFFFF, above every candidate key (<= HK_MAX)
        row[r] = (uint32_t)x;
        sk[r] = key[r];
    }
    wave_sort32<R>(sk);
    const uint32_t Ka = wave_at_u32<R>(sk, ra), Kb = wave_at_u32<R>(sk, rb);
    int p0 = 0, m = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        p0 += (int)__popcll(__ballot(key[r] < Ka));
        m += (int)__popcll(__ballot(key[r] >= Ka && key[r] <= Kb));
    }
    if (m == rb - ra + 1 && (ra == rb || Ka != Kb)) {
        // distinct high words at the target ranks: each key names one candidate
        auto row_of = [&](uint32_t K) -> uint32_t {
            uint32_t rw = 0;
            bool found = false;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const uint64_t mk = __ballot(key[r] == K);
                if (!found && mk != 0ull) {
                    rw = (uint32_t)__builtin_amdgcn_readlane((int)row[r], (int)__builtin_ctzll(mk));
                    found = true;
                }
            }
            return rw;
        };
        const uint32_t rwa = row_of(Ka), rwb = ra == rb ? rwa : row_of(Kb);
        va = col[rwa];
        vb = col[rwb];
        return true;
    }
    // high words tie at the target ranks: the full values of the candidates whose keys lie in
    // [Ka, Kb] (ranks p0 .. p0 + m - 1) into this wave's own (already loaded) list space
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    int base = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const bool in = key[r] >= Ka && key[r] <= Kb;
        const uint64_t mk = __ballot(in);
        if (in) {
            const double x = col[row[r]];
            L1[base + mask_rank(mk)] = tail == 0 ? dkey(x) : ~dkey(x);
        }
        base += (int)__popcll(mk);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    uint64_t w[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int e = lane + WAVE * r;
        w[r] = e < m ? L1[e] : SENT;
    }
    wave_sort<R>(w);
    auto atw = [&](int e) -> uint64_t {
        const int q = e >> 6, l = e & 63;
        uint64_t x = readlane_u64(w[0], l);
        static_for<1, R>([&](auto rc) {
            constexpr int r = decltype(rc)::value;
            const uint64_t t = readlane_u64(w[r], l);
            x = q == r ? t : x;
        });
        return x;
    };
    const uint64_t fa = atw(ra - p0), fb = atw(rb - p0);
    va = kval(tail == 0 ? fa : ~fa);
    vb = kval(tail == 0 ? fb : ~fb);
    return true;
}

template <int VPH>
__global__ __launch_bounds__(2 * WAVE, pair_hk_wgs(VPH) / 2) void select_pair_hk_kernel(SelArgs a) {
    __shared__ PairHkSmem sm;
    const int lane = lane_id();
    const int h = __builtin_amdgcn_readfirstlane((int)threadIdx.x / WAVE);
    const int64_t nunits = (int64_t)a.nseg * a.ncols;
    int64_t k = blockIdx.x;
    if (k >= nunits) return;   // block-uniform
    const int ncols = a.ncols;
    const int G = (int)gridDim.x;
    const int dS = G / ncols, dC = G - (G / ncols) * ncols;
    int s_cur = (int)blockIdx.x / ncols;
    int c_cur = (int)blockIdx.x - s_cur * ncols;
    uint32_t xk[VPH];
    // the unit's raw high words: one buffer descriptor per unit (its range check reads 0 past
    // the month end; masked after), the lane's byte offset the only VGPR
    auto load = [&](int s, int c) -> int {
        const int64_t r0 = a.seg_off[s];
        const int L = (int)(a.seg_off[s + 1] - r0);
        const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)(a.hp + (int64_t)c * a.pstride + r0), 0,
                                                          L > 0 ? L * 4 : 0, 0x00020000);
        uint32_t lb = (uint32_t)(h * WAVE + lane) * 4u;
        asm volatile("" : "+v"(lb));
#pragma unroll
        for (int v = 0; v < VPH; ++v)
            xk[v] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rs, lb + (uint32_t)(v * 2 * WAVE * 4), 0, 0);
        return L;
    };
    auto finite_range = [&](int s, int c, double& m1, double& m2) {
        const PCols base = sel_col(a, c, a.seg_off[s]);
        const int Lu = (int)(a.seg_off[s + 1] - a.seg_off[s]);
        m1 = NAN;
        m2 = NAN;
        for (int r = h * WAVE + lane; r < Lu; r += 2 * WAVE) {
            const double x = base[r];
            m1 = hw_min(m1, isfinite(x) ? x : NAN);
            m2 = hw_max(m2, isfinite(x) ? x : NAN);
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            m1 = hw_min(m1, xor_lanes_f64(m1, o));
            m2 = hw_max(m2, xor_lanes_f64(m2, o));
        }
    };
    int L = load(s_cur, c_cur);
    while (true) {
        const int64_t u = (int64_t)c_cur * a.nseg + s_cur;
        const int64_t kn = k + gridDim.x;
        const bool more = kn < nunits;
        int s_nx = s_cur + dS, c_nx = c_cur + dC;
        if (c_nx >= ncols) {
            c_nx -= ncols;
            ++s_nx;
        }
        int Ln = 0;
        const int row0 = h * WAVE + lane;
        // ---- 1. keys (rows past the month end -> HK_NONE), count, lane min / max keys
        const int lim = L - row0;
        int nh = 0;
        uint32_t kmn = HK_NONE, kmx2 = 0;
#if FM_PAIR_HK_LANECNT
        // invalid keys counted per lane from the wrap of the max's offset add (one add with
        // carry per value), one wave sum after the loop instead of a ballot per value
        int nbad = 0;
        // values in pairs: the lane min / max are one v_min3 / v_max3 per two values.  (A
        // second copy of this loop that range-tests only the last register -- the bench's
        // 5,000-row months fill the others -- pushed the kernel to 128 VGPRs with spills.)
        static_assert(VPH % 2 == 0, "pairs of registers");
#pragma unroll
        for (int v = 0; v < VPH; v += 2) {
            uint32_t kk[2], kx[2];
#pragma unroll
            for (int d = 0; d < 2; ++d) {
                const int vv = v + d;
                kk[d] = vv * 2 * WAVE < lim ? hkey(xk[vv]) : HK_NONE;
                xk[vv] = kk[d];
                // kk + 0x1FFFFE: NaN / absent keys wrap below every valid one (carry set)
                asm volatile("v_add_co_u32 %0, vcc, 0x1ffffe, %2\n\tv_addc_co_u32 %1, vcc, 0, %1, vcc"
                             : "=&v"(kx[d]), "+v"(nbad)
                             : "v"(kk[d])
                             : "vcc");
            }
            kmn = min(kmn, min(kk[0], kk[1]));
            kmx2 = max(kmx2, max(kx[0], kx[1]));
            asm volatile("" : "+v"(kmn), "+v"(kmx2));
        }
        nh = VPH * WAVE - wave_sum(nbad);
#else
#pragma unroll
        for (int v = 0; v < VPH; ++v) {
            const uint32_t kk = v * 2 * WAVE < lim ? hkey(xk[v]) : HK_NONE;
            xk[v] = kk;
            nh += (int)__popcll(__ballot(kk <= HK_MAX));
            kmn = min(kmn, kk);
            kmx2 = max(kmx2, kk + 0x1FFFFEu);   // NaN / absent keys wrap below every valid one
            asm volatile("" : "+s"(nh), "+v"(kmn), "+v"(kmx2));
        }
#endif
        const bool tvalid = kmn <= HK_MAX;
        const uint32_t kmx = kmx2 - 0x1FFFFEu;
        const bool amb = tvalid && (kmn == 0u || kmx == HK_MAX);
        {
            uint32_t ta[1] = {tvalid ? kmn : HK_NONE}, tb[1] = {tvalid ? HK_MAX - kmx : HK_NONE};
#if !FM_PAIR_KTH
            wave_sort32<1>(ta);
            wave_sort32<1>(tb);
#endif
            sm.sk[h][0][lane] = ta[0];
            sm.sk[h][1][lane] = tb[0];
        }
        const int ambw = (int)__popcll(__ballot(amb));
        if (lane == 0) {
            sm.ni[h][0] = nh;
            sm.ni[h][3] = ambw;
        }
        __syncthreads();
        const int n = sm.ni[0][0] + sm.ni[1][0];
        const int mode = a.lerp_mode;
        const bool apply = n >= a.min_count && n > 0;
        int i0 = 0, j0 = 0, i1 = 0, j1 = 0;
        double g0 = 0.0, g1 = 0.0;
        if (apply) {
            qranks(n, a.q_lo, mode, i0, j0, g0);
            qranks(n, a.q_hi, mode, i1, j1, g1);
        }
        bool ok = apply && sm.ni[0][3] + sm.ni[1][3] == 0;
        if (ok) {
            // ---- 2. this wave's tail threshold: the kr-th of the 128 lane-extreme keys
            const int t = h;
            const int kr = t == 0 ? j0 : n - 1 - i1;
            uint32_t T = HK_NONE;
#if FM_PAIR_KTH
            // (unsorted lane extremes of both halves; the (kr+1)-th smallest by bisection)
            if (kr < 2 * WAVE) T = wave_kth_u32_of2(sm.sk[0][t][lane], sm.sk[1][t][lane], kr + 1);
#else
            if (kr < 2 * WAVE) {
                const uint32_t mine = sm.sk[0][t][lane], other = sm.sk[1][t][lane];
                const int q0 = lane + count_below_u32(sm.sk[1][t], mine, false);
                const int q1 = lane + count_below_u32(sm.sk[0][t], other, true);
                const uint64_t m0 = __ballot(q0 == kr), m1 = __ballot(q1 == kr);
                if (m0) T = (uint32_t)__builtin_amdgcn_readlane((int)mine, __builtin_ctzll(m0));
                else if (m1) T = (uint32_t)__builtin_amdgcn_readlane((int)other, __builtin_ctzll(m1));
            }
#endif
            if (lane == 0) {
                sm.tv[h] = T;
                sm.okv[h] = T <= HK_MAX ? 1 : 0;
            }
            __syncthreads();
            ok = sm.okv[0] != 0 && sm.okv[1] != 0;   // block-uniform
        }
        double lo = NAN, hi = NAN;
        bool prefetched = false;
        if (ok) {
            // ---- 3. (key, row) candidates of both tails from this wave's half
            const uint32_t tlo = sm.tv[0], thi = sm.tv[1];
            int clo = 0, chi = 0;
            uint64_t* Ll = sm.cand[h][0];
            uint64_t* Lh = sm.cand[h][1];
#pragma unroll
            for (int v = 0; v < VPH; ++v) {
                const uint32_t kk = xk[v];
                const bool bl = kk <= tlo, bh = HK_MAX - kk <= thi;   // NaN / absent keys wrap above thi
                const uint64_t ml = __ballot(bl), mh = __ballot(bh);
                const uint64_t row = (uint64_t)(uint32_t)(row0 + v * 2 * WAVE);
                if (ml) {
                    if (bl) Ll[(clo + mask_rank(ml)) & (WCAP - 1)] = ((uint64_t)kk << 32) | row;
                    clo += (int)__popcll(ml);
                }
                if (mh) {
                    if (bh) Lh[(chi + mask_rank(mh)) & (WCAP - 1)] = ((uint64_t)(HK_MAX - kk) << 32) | row;
                    chi += (int)__popcll(mh);
                }
            }
            if (lane == 0) {
                sm.ni[h][1] = clo;
                sm.ni[h][2] = chi;
            }
            // xk is dead from here on: the next unit's loads fly during the sorts and gathers
            if (FM_PAIR_HK_PF && more) Ln = load(s_nx, c_nx);
            prefetched = FM_PAIR_HK_PF != 0;
            __syncthreads();
            // ---- 4. one tail per wave over both halves' candidates
            const int t = h;
            const int c0 = sm.ni[0][1 + t], c1 = sm.ni[1][1 + t];
            const int cc = c0 + c1;
            bool good = c0 <= WCAP && c1 <= WCAP && cc <= 4 * WAVE;
            if (good) {
                const PCols col = sel_col(a, c_cur, a.seg_off[s_cur]);
                const int ra = t == 0 ? i0 : n - 1 - j1, rb = t == 0 ? j0 : n - 1 - i1;
                double va = NAN, vb = NAN;
                if (cc <= WAVE) good = pick_hk<1>(sm.cand[0][t], c0, sm.cand[1][t], c1, ra, rb, t, col, va, vb);
                else if (cc <= 2 * WAVE) good = pick_hk<2>(sm.cand[0][t], c0, sm.cand[1][t], c1, ra, rb, t, col, va, vb);
                else good = pick_hk<4>(sm.cand[0][t], c0, sm.cand[1][t], c1, ra, rb, t, col, va, vb);
                // tail 1: ra / rb count from the top: va is the value at rank j1, vb at i1
                if (lane == 0) sm.res[h] = t == 0 ? qlerp(va, vb, g0, mode) : qlerp(vb, va, g1, mode);
            }
            if (lane == 0) sm.okv[h] = good ? 1 : 0;
            __syncthreads();
            ok = sm.okv[0] != 0 && sm.okv[1] != 0;   // block-uniform
            lo = sm.res[0];
            hi = sm.res[1];
        }
        if (apply && !ok) {
            if (threadIdx.x == 0) sel_mark(a, u);   // redone by the fix-up kernel
        } else if (h == 0) {
            double cen = 0.5 * (lo + hi);
            if (!isfinite(cen)) {
                double m1, m2;
                finite_range(s_cur, c_cur, m1, m2);
                if (lane == 0) sm.res[0] = m1, sm.res[1] = m2;
            }
            if (lane == 0) {
                if (a.center && isfinite(cen)) a.center[u] = cen;
                a.lo[u] = lo;
                a.hi[u] = hi;
                if (a.nvalid) a.nvalid[u] = n;
                if (zero_cut(a, lo, hi)) sel_push(a, u);
            }
        } else if (!isfinite(0.5 * (lo + hi))) {
            double m1, m2;
            finite_range(s_cur, c_cur, m1, m2);
            if (lane == 0) sm.fr[0] = m1, sm.fr[1] = m2;
        }
        if (more && !prefetched) Ln = load(s_nx, c_nx);
        __syncthreads();
        if ((ok || !apply) && a.center && !isfinite(0.5 * (lo + hi)) && threadIdx.x == 0) {
            const double m1 = hw_min(sm.res[0], sm.fr[0]), m2 = hw_max(sm.res[1], sm.fr[1]);
            double cen = 0.5 * (m1 + m2);
            a.center[u] = isfinite(cen) ? cen : 0.0;
        }
        __syncthreads();   // LDS state is rewritten by the next unit
        if (!more) break;
        k = kn;
        s_cur = s_nx;
        c_cur = c_nx;
        L = Ln;
    }
}

int select_wave_grid(int64_t nunits) {
    static int ncu = [] {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
            n = 256;
        return n;
    }();
    const int64_t need = (nunits + SNW - 1) / SNW;
    const int64_t cap = (int64_t)ncu * 2;   // two resident workgroups per CU
    return (int)(need < cap ? need : cap);
}

template <int VPH>
void launch_select_pair_hk(const SelArgs& a, hipStream_t st);

template <int VPH>
void launch_select_pair(const SelArgs& a, hipStream_t st) {
    if (a.hp != nullptr) {
        launch_select_pair_hk<VPH>(a, st);
        return;
    }
    static int ncu = [] {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
            n = 256;
        return n;
    }();
    const int64_t nunits = (int64_t)a.nseg * a.ncols;
    const int64_t cap = (int64_t)ncu * 8;   // eight 2-wave workgroups per CU (4 waves / SIMD)
    hipLaunchKernelGGL((select_pair_kernel<VPH>), dim3((unsigned)(nunits < cap ? nunits : cap)), dim3(2 * WAVE),
                       0, st, a);
}

template <int VPH>
void launch_select_pair_hk(const SelArgs& a, hipStream_t st) {
    static int ncu = [] {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
            n = 256;
        return n;
    }();
    const int64_t nunits = (int64_t)a.nseg * a.ncols;
    const int64_t cap = (int64_t)ncu * pair_hk_wgs(VPH);
    hipLaunchKernelGGL((select_pair_hk_kernel<VPH>), dim3((unsigned)(nunits < cap ? nunits : cap)), dim3(2 * WAVE),
                       0, st, a);
}

int launch_select_pair_vph(const SelArgs& a, int max_seg_len, hipStream_t st) {
    const int vph = (max_seg_len + 2 * WAVE - 1) / (2 * WAVE);
    if (vph <= 8) launch_select_pair<8>(a, st);
    else if (vph <= 16) launch_select_pair<16>(a, st);
    else if (vph <= 24) launch_select_pair<24>(a, st);
    else if (vph <= 32) launch_select_pair<32>(a, st);
    else if (vph <= 40) launch_select_pair<40>(a, st);
    else if (vph <= 48) launch_select_pair<48>(a, st);
    else {
        set_error("select pair kernel: %d-row segments exceed %d", max_seg_len, 48 * 2 * WAVE);
        return FM_ETOOBIG;
    }
    return FM_OK;
}

// A/B switch for timing builds only (-DFM_AB_SELECT_ONE_WAVE=1): the one-wave kernel
bool getenv_flag_one_wave() {
#ifdef FM_AB_SELECT_ONE_WAVE
    return FM_AB_SELECT_ONE_WAVE != 0;
#else
    return false;
#endif
}

template <int VPL>
void launch_select_wave(const SelArgs& a, hipStream_t st) {
    const int64_t nunits = (int64_t)a.nseg * a.ncols;
    if (a.mean == nullptr)
        hipLaunchKernelGGL((select_wave_kernel<VPL, true>), dim3((unsigned)select_wave_grid(nunits)), dim3(ST), 0, st, a);
    else
        hipLaunchKernelGGL((select_wave_kernel<VPL, false>), dim3((unsigned)select_wave_grid(nunits)), dim3(ST), 0, st, a);
}

// get_subsets' NYSE breakpoints AND the nested universe levels in one launch (reference
// src/calc_Lewellen_2014.py:69-105): one 256-thread workgroup per month holds the month's
// `me` in registers (VPT per thread, one coalesced read, the NYSE flags as a bit mask),
// finds the pandas groupby.quantile(q_a, q_b) order statistics of the NYSE rows (NaN me
// skipped) by the adaptive histogram select, lerps them the pandas way, and writes every
// row's level (me >= me_20) + (me >= me_50) from the same registers (NaN compares False).
#ifndef FM_AB_UNI_APART
#define FM_AB_UNI_APART 0   // timing builds only: the universe in its own launch before the select
#endif
#ifndef FM_AB_UNI_NOSELECT
#define FM_AB_UNI_NOSELECT 0   // timing builds only (tools/build_variant.sh): skip the order statistics
#endif
template <int VPT>
__device__ __forceinline__ void universe_month(const double* __restrict__ me, const uint8_t* __restrict__ nyse,
                                               const int64_t* __restrict__ seg_off, double qa, double qb,
                                               double* __restrict__ cut_a, double* __restrict__ cut_b,
                                               uint8_t* __restrict__ level, int s, SelSmem& sm) {
    static_assert(VPT <= 64, "universe_kernel: NYSE flags are one 64-bit mask per thread");
    FM_PROBE_AT(sel, 0);
    const int tid = threadIdx.x;
    const int64_t r0 = seg_off[s];
    const int L = (int)(seg_off[s + 1] - r0);
    const int last = L > 0 ? L - 1 : 0;
    double xm[VPT];
    uint64_t nb = 0;
#pragma unroll
    for (int v = 0; v < VPT; ++v) {   // unconditional (clamped) loads, masked after
        const int idx = tid + v * ST;
        const int ci = idx < L ? idx : last;
        const double x = me[r0 + ci];
        const uint8_t m = nyse[r0 + ci];
        xm[v] = idx < L ? x : NAN;
        if (idx < L && m != 0 && !isnan(x)) nb |= 1ull << v;
    }
    // each pass re-forms the masked value (opaque to the optimizer): kept across the
    // histogram passes, the per-value NaN tests become 2 x VPT SGPRs spilled to VGPR lanes
    auto for_each = [&](auto&& f) {
#pragma unroll
        for (int v = 0; v < VPT; ++v) {
            double x = ((nb >> v) & 1ull) ? xm[v] : NAN;
            asm volatile("" : "+v"(x));
            f(x);
        }
    };
    int cnt = 0;
    uint64_t kmn = SENT, kmx = 0;
    for_each([&](double x) {
        if (!isnan(x)) {
            ++cnt;
            const uint64_t k = dkey(x);
            kmn = k < kmn ? k : kmn;
            kmx = k > kmx ? k : kmx;
        }
    });
    // count, min and max in one exchange (one barrier; nothing of sm is in use yet)
    {
        const int c = wave_sum(cnt);
        const uint64_t mn = wave_min_u64(kmn), mx = wave_max_u64(kmx);
        const int w = tid / WAVE;
        if ((tid & (WAVE - 1)) == 0) {
            sm.ints[w] = c;
            sm.u64s[w] = mn;
            sm.u64s[SNW + w] = mx;
        }
    }
    __syncthreads();
    int n = sm.ints[0];
    kmn = sm.u64s[0];
    kmx = sm.u64s[SNW];
#pragma unroll
    for (int q = 1; q < SNW; ++q) {
        n += sm.ints[q];
        kmn = sm.u64s[q] < kmn ? sm.u64s[q] : kmn;
        kmx = sm.u64s[SNW + q] > kmx ? sm.u64s[SNW + q] : kmx;
    }
    double a = NAN, b = NAN;
    FM_PROBE_AT(sel, 1);
    if (n > 0) {   // block-uniform
        int rk[4];
        double g0, g1;
        qranks(n, qa, 1, rk[0], rk[1], g0);
        qranks(n, qb, 1, rk[2], rk[3], g1);
        uint64_t ko[4] = {kmn, kmn, kmx, kmx};
        if (!FM_AB_UNI_NOSELECT) hist_select(for_each, 4, rk, kmn, kmx, ko, sm);
        a = qlerp(kval(ko[0]), kval(ko[1]), g0, 1);
        b = qlerp(kval(ko[2]), kval(ko[3]), g1, 1);
    }
    FM_PROBE_AT(sel, 2);
    if (tid == 0) {
        cut_a[s] = a;
        cut_b[s] = b;
    }
#pragma unroll
    for (int v = 0; v < VPT; ++v) {
        const int idx = tid + v * ST;
        if (idx < L) level[r0 + idx] = (uint8_t)((xm[v] >= a ? 1 : 0) + (xm[v] >= b ? 1 : 0));
    }
    FM_PROBE_AT(sel, 3);
}

template <int VPT>
__global__ __launch_bounds__(ST, VPT <= 20 ? 3 : 1) void universe_kernel(const double* __restrict__ me,
                                                      const uint8_t* __restrict__ nyse,
                                                      const int64_t* __restrict__ seg_off, double qa,
                                                      double qb, double* __restrict__ cut_a,
                                                      double* __restrict__ cut_b,
                                                      uint8_t* __restrict__ level) {
    __shared__ SelSmem sm;
    universe_month<VPT>(me, nyse, seg_off, qa, qb, cut_a, cut_b, level, (int)blockIdx.x, sm);
}

}  // namespace
}  // namespace fm

extern "C" int fm_select_cuts(const double* cols, int64_t col_stride, int32_t ncols,
                              const int64_t* seg_off, int32_t nseg, int32_t max_seg_len,
                              const uint8_t* row_mask, double q_lo, double q_hi,
                              int32_t min_count, int32_t lerp_mode, double* lo, double* hi,
                              int32_t* nvalid, double* mean, double* sd, void* ws, void* stream) {
    fm_select_args a{};
    a.cols = cols;
    a.col_stride = col_stride;
    a.ncols = ncols;
    a.seg_off = seg_off;
    a.nseg = nseg;
    a.max_seg_len = max_seg_len;
    a.row_mask = row_mask;
    a.q_lo = q_lo;
    a.q_hi = q_hi;
    a.min_count = min_count;
    a.lerp_mode = lerp_mode;
    a.lo = lo;
    a.hi = hi;
    a.nvalid = nvalid;
    a.mean = mean;
    a.sd = sd;
    a.ws = ws;
    return fm_select(&a, stream);
}

extern "C" int64_t fm_select_ws_bytes(int32_t nseg, int32_t ncols, int32_t max_seg_len) {
    if (nseg < 0 || ncols < 0 || max_seg_len < 0) return -1;
    return fm::ws_bytes(nseg, ncols, max_seg_len);
}

namespace fm {
namespace {
// fm_select, optionally with get_subsets' NYSE breakpoints + level bytes (u != NULL): months of
// <= 5,120 rows on the register paths share the select fix-up's launch after the select; they
// ride the long-month high-key kernel's launch (6,145 .. 20,480-row months, tail ranks, no row
// mask: one more grid column); on the other paths (MID, streaming) the universe is launched
// on its own first (fm_universe, or the row-masked select), same outputs.
int select_impl(const fm_select_args* args, const fm_universe_args* u, void* stream);
}  // namespace
}  // namespace fm

extern "C" int fm_select(const fm_select_args* args, void* stream) {
    return fm::select_impl(args, nullptr, stream);
}

extern "C" int fm_select_universe(const fm_select_args* args, const fm_universe_args* u, void* stream) {
    using namespace fm;
    FM_REQUIRE(u != nullptr && u->me && u->nyse && u->cut_a && u->cut_b && u->level,
               "fm_select_universe: null universe pointer");
    FM_REQUIRE(u->q_a >= 0.0 && u->q_a <= 1.0 && u->q_b >= 0.0 && u->q_b <= 1.0,
               "fm_select_universe: quantiles must be in [0,1]");
    return select_impl(args, u, stream);
}

namespace fm {
namespace {
void set_universe(SelArgs& a, const fm_universe_args* u) {
    a.ume = u->me;
    a.unyse = u->nyse;
    a.uq_a = u->q_a;
    a.uq_b = u->q_b;
    a.ucut_a = u->cut_a;
    a.ucut_b = u->cut_b;
    a.ulevel = u->level;
}

// the universe by its own launches (months past the fused paths): fm_universe's one-launch
// kernel up to its register budget, else the row-masked pandas select of the NYSE `me` with
// the level bytes (streaming path: any length)
int universe_separately(const fm_select_args& x, const fm_universe_args* u, void* stream) {
    if (x.max_seg_len <= 64 * ST)
        return fm_universe(u->me, u->nyse, x.seg_off, x.nseg, x.max_seg_len, u->q_a, u->q_b, u->cut_a, u->cut_b,
                           u->level, stream);
    fm_select_args y{};
    y.cols = u->me;
    y.col_stride = 0;
    y.ncols = 1;
    y.seg_off = x.seg_off;
    y.nseg = x.nseg;
    y.max_seg_len = x.max_seg_len;
    y.row_mask = u->nyse;
    y.q_lo = u->q_a;
    y.q_hi = u->q_b;
    y.min_count = 1;
    y.lerp_mode = 1;
    y.lo = u->cut_a;
    y.hi = u->cut_b;
    y.level = u->level;
    y.ws = x.ws;
    return select_impl(&y, nullptr, stream);
}

int select_impl(const fm_select_args* args, const fm_universe_args* u, void* stream) {
    FM_REQUIRE(args != nullptr, "fm_select: null args");
    const fm_select_args& x = *args;
    const double* cols = x.cols;
    const int64_t* seg_off = x.seg_off;
    const int32_t ncols = x.ncols, nseg = x.nseg, max_seg_len = x.max_seg_len;
    const uint8_t* row_mask = x.row_mask;
    const int32_t* nvalid = x.nvalid;
    FM_REQUIRE((cols || (x.hi_plane && x.lo_plane)) && seg_off && x.lo && x.hi, "fm_select_cuts: null pointer");
    FM_REQUIRE(ncols > 0 && ncols <= 65535 && nseg >= 0, "fm_select_cuts: bad sizes");
    FM_REQUIRE(x.lerp_mode == 0 || x.lerp_mode == 1, "fm_select_cuts: lerp_mode must be 0 or 1");
    FM_REQUIRE(x.q_lo >= 0.0 && x.q_lo <= 1.0 && x.q_hi >= 0.0 && x.q_hi <= 1.0,
               "fm_select_cuts: quantiles must be in [0,1]");
    if (nseg == 0) return FM_OK;
    FM_REQUIRE(x.level == nullptr || ncols == 1, "fm_select: level needs a single column");
    FM_REQUIRE(x.ws != nullptr, "fm_select: ws (fm_select_ws_bytes bytes, zeroed once) is required");
    SelArgs a{cols,        x.col_stride, seg_off, nseg,     ncols, row_mask, x.q_lo, x.q_hi,
              x.min_count, x.lerp_mode,  x.lo,    x.hi,     x.nvalid, x.mean, x.sd,  x.center,
              nullptr,     x.level};
    a.ctl = (SelCtl*)x.ws;
    a.hp = x.hi_plane;
    a.pstride = x.plane_stride;
    a.lp = x.lo_plane;
    FM_REQUIRE(a.hp == nullptr || a.pstride > 0, "fm_select: hi_plane needs plane_stride > 0");
    FM_REQUIRE(a.lp == nullptr || a.hp != nullptr, "fm_select: lo_plane needs hi_plane");
    // a split panel without FP64 columns: only the plane-reading paths (the two-wave and
    // long-month high-key kernels, the workgroup / streaming fix-ups) can serve it
    const bool no_f64 = cols == nullptr;
    hipStream_t st = (hipStream_t)stream;
    const int vpt = (max_seg_len + ST - 1) / ST;
    const bool long_path = vpt > FM_SELECT_STREAM_VPT && max_seg_len <= LONG_VPT * LT && x.mean == nullptr &&
                           nvalid != nullptr && !FM_AB_SELECT_STREAM;
    // a universe rides the long-month kernel's launch (one more grid column) unless its tails
    // need the histogram (MID) kernel (riding the two-wave kernel's persistent workgroups
    // measured slower for short months: 118 vs 83 + 23 us on the bench panel,
    // profiles/r04/v2_kbench_fused_universe.log)
    const bool ride = u != nullptr && long_path && !long_is_mid(a, max_seg_len) &&
                      (FM_HK_RIDE || FM_AB_LONG_F64 || FM_AB_LONG != 0);
    // months of <= 20 x 256 rows on the register paths: the universe shares the fix-up's launch
    // after the select (one launch less; the two are independent)
    const bool with_fixup = u != nullptr && !ride && !long_path && vpt <= 20 && !FM_AB_UNI_APART;
    if (u != nullptr && !ride && !with_fixup) {
        const int rcu = universe_separately(x, u, stream);
        if (rcu != FM_OK) return rcu;
    }
    if (long_path) {
        // past the 256-thread paths' register budget: the 512-thread register-resident
        // kernel (one read per unit); the streaming kernel redoes the units it marked
        FM_REQUIRE(!no_f64 || (a.hp != nullptr && !long_is_mid(a, max_seg_len) && !FM_AB_LONG_F64 && FM_AB_LONG == 0),
                   "fm_select: this long-month path (row mask / middle ranks) needs FP64 columns");
        SelArgs al = a;
        if (ride) set_universe(al, u);
        const int rc = launch_select_long(al, max_seg_len, st);
        if (rc != FM_OK) return rc;
        FM_CHECK_LAUNCH("fm_select_cuts(long)");
        if (!FM_AB_NOFB) launch_fixup(a, max_seg_len, st);
        FM_CHECK_LAUNCH("fm_select_cuts(long fix-up)");
        // the level bytes by a streaming launch: writing them from the select kernel (a
        // re-read of the unmasked column, or unmasked registers + mask bits) measured no
        // faster, the register select being latency-bound at one workgroup per CU
        return a.level ? fm_universe_level(cols, seg_off, nseg, (int64_t)max_seg_len * nseg, x.lo, x.hi, x.level, stream)
                       : FM_OK;
    }
    if (vpt > FM_SELECT_STREAM_VPT) {
        // longer still, or row masks / moments: stream every unit from HBM / L2 for each
        // pass (exact, any length)
        hipLaunchKernelGGL(select_stream_kernel, dim3(nseg, ncols), dim3(ST), 0, st, a);
        FM_CHECK_LAUNCH("fm_select_cuts(stream)");
        launch_fixup(a, max_seg_len, st);
        FM_CHECK_LAUNCH("fm_select_cuts(stream fix-up)");
        return a.level ? fm_universe_level(cols, seg_off, nseg, (int64_t)max_seg_len * nseg, x.lo, x.hi, x.level, stream) : FM_OK;
    }
    // wave fast path: no row mask, segments of <= 96 * 64 rows, nvalid present (it carries
    // the fallback marks); the workgroup kernel then redoes the marked units only
    const int vpl = (max_seg_len + WAVE - 1) / WAVE;
#ifdef FM_AB_SELECT_WG
    const bool wave = false;   // A/B timing builds only: the workgroup-per-unit kernel for all
#else
    const bool wave = row_mask == nullptr && nvalid != nullptr && vpl <= 96;
#endif
    (void)vpl;
    FM_REQUIRE(!no_f64 || (wave && x.mean == nullptr && a.hp != nullptr) || !wave,
               "fm_select: moments on a split panel need FP64 columns");
    if (wave && x.mean == nullptr && vpl <= 96 && !getenv_flag_one_wave()) {
        // two waves per unit (the common Table-2 case: no moments)
        const int rc = launch_select_pair_vph(a, max_seg_len, st);
        if (rc != FM_OK) return rc;
        FM_CHECK_LAUNCH("fm_select_cuts(pair)");
    } else if (wave) {
        if (vpl <= 16) launch_select_wave<16>(a, st);
        else if (vpl <= 32) launch_select_wave<32>(a, st);
        else if (vpl <= 48) launch_select_wave<48>(a, st);
        else if (vpl <= 64) launch_select_wave<64>(a, st);
        else if (vpl <= 80) launch_select_wave<80>(a, st);
        else launch_select_wave<96>(a, st);
        FM_CHECK_LAUNCH("fm_select_cuts(wave)");
    }
    if (!wave) {   // one workgroup per unit (row masks, moments past the wave kernels)
        if (vpt <= 2) launch_select<2>(a, ncols, st);
        else if (vpt <= 4) launch_select<4>(a, ncols, st);
        else if (vpt <= 8) launch_select<8>(a, ncols, st);
        else if (vpt <= 16) launch_select<16>(a, ncols, st);
        else if (vpt <= 20) launch_select<20>(a, ncols, st);
        else launch_select<FM_SELECT_STREAM_VPT>(a, ncols, st);
        FM_CHECK_LAUNCH("fm_select_cuts");
    }
    if (with_fixup) {
        SelArgs au = a;
        set_universe(au, u);
        launch_fixup_universe(au, max_seg_len, st);
    } else {
        launch_fixup(a, max_seg_len, st);
    }
    FM_CHECK_LAUNCH("fm_select_cuts(fix-up)");
    return a.level ? fm_universe_level(cols, seg_off, nseg, (int64_t)max_seg_len * nseg, x.lo, x.hi, x.level, stream) : FM_OK;
}

}  // namespace
}  // namespace fm

extern "C" int fm_universe(const double* me, const uint8_t* nyse, const int64_t* seg_off, int32_t nseg,
                           int32_t max_seg_len, double q_a, double q_b, double* cut_a, double* cut_b,
                           uint8_t* level, void* stream) {
    using namespace fm;
    FM_REQUIRE(me && nyse && seg_off && cut_a && cut_b && level, "fm_universe: null pointer");
    FM_REQUIRE(nseg >= 0 && max_seg_len >= 0, "fm_universe: bad sizes");
    FM_REQUIRE(q_a >= 0.0 && q_a <= 1.0 && q_b >= 0.0 && q_b <= 1.0, "fm_universe: quantiles must be in [0,1]");
    if (max_seg_len > 64 * ST) {
        set_error("fm_universe: %d-row months exceed %d (use fm_select_cuts + fm_universe_level)",
                  max_seg_len, 64 * ST);
        return FM_ETOOBIG;
    }
    if (nseg == 0) return FM_OK;
    hipStream_t st = (hipStream_t)stream;
    const int vpt = (max_seg_len + ST - 1) / ST;
    if (vpt <= 8) hipLaunchKernelGGL(universe_kernel<8>, dim3(nseg), dim3(ST), 0, st, me, nyse, seg_off, q_a, q_b, cut_a, cut_b, level);
    else if (vpt <= 20) hipLaunchKernelGGL(universe_kernel<20>, dim3(nseg), dim3(ST), 0, st, me, nyse, seg_off, q_a, q_b, cut_a, cut_b, level);
    else if (vpt <= 32) hipLaunchKernelGGL(universe_kernel<32>, dim3(nseg), dim3(ST), 0, st, me, nyse, seg_off, q_a, q_b, cut_a, cut_b, level);
    else hipLaunchKernelGGL(universe_kernel<64>, dim3(nseg), dim3(ST), 0, st, me, nyse, seg_off, q_a, q_b, cut_a, cut_b, level);
    FM_CHECK_LAUNCH("fm_universe");
    return FM_OK;
}

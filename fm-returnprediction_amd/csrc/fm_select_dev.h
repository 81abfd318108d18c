// Device-side building blocks of the exact order-statistic selection (fm_select):
// order-preserving keys, wave bitonic sorts over DPP / permlane exchanges, the exact MSB
// radix select, the workgroup tail selection and the numpy / pandas interpolation
// (anonymous namespace: each including translation unit gets its own copy).  Compiled with -ffp-contract=off (exact lerps).
#pragma once
#include <math.h>

#include "fm_common.h"

// ablation knobs: timing builds only (tools/kbench.py), never the shipped library
#ifndef FM_AB_SEL_NOSORT
#define FM_AB_SEL_NOSORT 0
#endif
#ifndef FM_AB_SEL_NOCOMPACT
#define FM_AB_SEL_NOCOMPACT 0
#endif
#ifndef FM_AB_SEL_NOLOAD
#define FM_AB_SEL_NOLOAD 0
#endif

namespace fm {
namespace {

constexpr int ST = 256;
constexpr int SNW = ST / WAVE;
constexpr int CAND_CAP = 2048;

constexpr int HB = 2048;     // hist_select: bins per level
constexpr int HCAP = 256;    // hist_select: keys per candidate list (one wave sorts them)

// fm_select_args.ws header (zeroed by the caller once; every fm_select leaves it zeroed):
// the worklist of units the fix-up kernel redoes exactly.
struct SelCtl {
    uint32_t nwork;   // worklist length
    uint32_t done;    // fix-up workgroups finished (the last one resets both)
    uint32_t pad[62];
    uint32_t work[1];   // [nseg * ncols] unit ids (column * nseg + month)
};

// Shared scratch of the workgroup select paths for NW-wave workgroups.
template <int NW>
struct SelSmemT {
    uint64_t buf[CAND_CAP];
    uint32_t hist[HB];
    uint64_t u64s[2 * NW];
    double dbl[2 * NW];
    int ints[NW > 8 ? NW : 8];
    uint64_t bc[4];
    int hs[4 * 3];           // hist_select: located (bin, count below, count in bin) per target
    uint32_t hcnt[4];        // hist_select: candidate list fill counters
};
using SelSmem = SelSmemT<SNW>;

struct SelArgs {
    const double* cols;
    int64_t col_stride;
    const int64_t* seg_off;
    int nseg;
    int ncols;
    const uint8_t* mask;
    double q_lo, q_hi;
    int min_count;
    int lerp_mode;
    double* lo;
    double* hi;
    int32_t* nvalid;
    double* mean;
    double* sd;
    double* center;
    double* prm;   // optional LDS [3][32]: thread 0 also stores lo, hi, center of column c there
    uint8_t* level;   // fm_select_args.level (written by fm_universe_level after the cuts)
    // fm_select_universe: get_subsets' NYSE breakpoints + level bytes of every month, done by
    // one more grid column of the long-month high-key kernel or by the first nseg workgroups
    // of the select fix-up's launch (ume == NULL: none)
    const double* ume = nullptr;
    const uint8_t* unyse = nullptr;
    double uq_a = 0.0, uq_b = 0.0;
    double* ucut_a = nullptr;
    double* ucut_b = nullptr;
    uint8_t* ulevel = nullptr;
    // fm_select_args.ws: the fix-up worklist (units a fast kernel could not finish, and units
    // whose numpy cut is exactly zero); NULL inside the fix-up kernel itself
    SelCtl* ctl = nullptr;
    // fm_select_args.hi_plane: the columns' high 32-bit words ([ncols][pstride]); the two-wave
    // and long-month kernels then read 4 bytes per value
    const uint32_t* hp = nullptr;
    int64_t pstride = 0;
    // fm_select_args.lo_plane: with hp, the low words; cols may then be NULL (a split panel
    // without FP64 columns): the gathers and fix-up paths read values through sel_col
    const uint32_t* lp = nullptr;
};

// Column c of the panel from row r0 on, as FP64 values or from the two planes
__device__ __forceinline__ PCols sel_col(const SelArgs& a, int c, int64_t r0) {
    if (a.cols != nullptr) return PCols{a.cols + (int64_t)c * a.col_stride + r0, nullptr, 0};
    return PCols{nullptr, a.hp + (int64_t)c * a.pstride + r0, (int64_t)(a.lp - a.hp)};
}

// One lane: unit u goes on the fix-up kernel's worklist (and is marked, nvalid = -1, when the
// kernel could not finish it).  A call pushes each of its nseg * ncols units at most once, so
// the list (sized for them) cannot overflow -- unless an earlier call's entries were left
// behind (its fix-up launch never ran: an error between the two launches).  Entries past the
// list's capacity are then dropped here, and the fix-up skips ids outside this call's units.
__device__ __forceinline__ void sel_push(const SelArgs& a, int64_t u) {
    if (a.ctl != nullptr) {
        const uint32_t i = atomicAdd(&a.ctl->nwork, 1u);
        if (i < (uint32_t)((int64_t)a.nseg * a.ncols)) a.ctl->work[i] = (uint32_t)u;
    }
}
__device__ __forceinline__ void sel_mark(const SelArgs& a, int64_t u) {
    if (a.nvalid) a.nvalid[u] = -1;
    sel_push(a, u);
}
// A numpy cut that is exactly +-0: its sign is numpy's partition order's business (the
// fix-up kernel replays it when the unit holds both signed zeros).  pandas' groupby.quantile
// (lerp mode 1) orders equal values by an unstable argsort that numpy dispatches to its SIMD
// sort on AVX-512 hosts; that order is not reproduced (only the sign of an exactly-zero NYSE
// `me` breakpoint could differ, and market equity is positive).
__device__ __forceinline__ bool zero_cut(const SelArgs& a, double lo, double hi) {
    return a.lerp_mode == 0 && a.ctl != nullptr && (lo == 0.0 || hi == 0.0);
}

__device__ __forceinline__ uint64_t key_of(double x) { return isnan(x) ? SENT : dkey(x); }

// General path: exact key at ascending rank `rank` (0-based) among the valid values, by an
// MSB-first 8-bit radix select over keys formed on the fly from the register values (no
// key array, so the general path adds no registers to the tail fast path).
template <int VPT>
__device__ __forceinline__ uint64_t radix_rank(const double (&xv)[VPT], int rank, SelSmem& sm) {
    uint64_t prefix = 0, pmask = 0;
    int rem = rank;
#pragma unroll 1
    for (int shift = 56; shift >= 0; shift -= 8) {
        for (int i = threadIdx.x; i < 256; i += ST) sm.hist[i] = 0;
        __syncthreads();
#pragma unroll
        for (int v = 0; v < VPT; ++v) {
            double x = xv[v];
            asm volatile("" : "+v"(x));   // keep the key per pass (no hoisted key array)
            const uint64_t k = key_of(x);
            if (k != SENT && (k & pmask) == prefix) atomicAdd(&sm.hist[(k >> shift) & 255u], 1u);
        }
        __syncthreads();
        if (threadIdx.x < WAVE) {
            const int l = threadIdx.x;
            const int h0 = sm.hist[4 * l], h1 = sm.hist[4 * l + 1], h2 = sm.hist[4 * l + 2],
                      h3 = sm.hist[4 * l + 3];
            const int s = h0 + h1 + h2 + h3;
            const int incl = wave_incl_scan(s);
            const int excl = incl - s;
            if (excl <= rem && rem < incl) {
                int c = excl, b = 4 * l;
                if (c + h0 <= rem) {
                    c += h0;
                    ++b;
                    if (c + h1 <= rem) {
                        c += h1;
                        ++b;
                        if (c + h2 <= rem) {
                            c += h2;
                            ++b;
                        }
                    }
                }
                sm.ints[0] = b;
                sm.ints[1] = rem - c;
            }
        }
        __syncthreads();
        const int sel = sm.ints[0];
        rem = sm.ints[1];
        prefix |= (uint64_t)sel << shift;
        pmask |= 0xFFull << shift;
        __syncthreads();
    }
    return prefix;
}

// Keys at ranks ri <= rj (rj == ri or ri + 1) by radix select; block-uniform.
template <int VPT>
__device__ __forceinline__ void radix_pair(const double (&xv)[VPT], int ri, int rj, uint64_t& ki,
                                           uint64_t& kj, SelSmem& sm) {
    ki = radix_rank<VPT>(xv, ri, sm);
    if (rj == ri) {
        kj = ki;
        return;
    }
    int le = 0;
    uint64_t nxt = SENT;
#pragma unroll
    for (int v = 0; v < VPT; ++v) {
        double x = xv[v];
        asm volatile("" : "+v"(x));
        const uint64_t k = key_of(x);
        le += k <= ki ? 1 : 0;
        if (k > ki && k < nxt) nxt = k;
    }
    le = block_sum<SNW>(le, sm.ints);
    nxt = block_min_u64<SNW>(nxt, sm.u64s);
    kj = le >= rj + 1 ? ki : nxt;
}

// Bitonic stage (k, j) for register r (element e = lane + 64 r): lane l keeps the minimum
// iff ((l & j) == 0) == ((e & k) == 0).  As a compile-time 64-bit lane mask the role costs
// one s_mov_b64 instead of per-stage lane arithmetic.
template <int K, int J, int Rr>
__host__ __device__ constexpr uint64_t bitonic_min_mask() {
    uint64_t m = 0;
    for (int l = 0; l < WAVE; ++l)
        if (((l & J) == 0) == (((l + WAVE * Rr) & K) == 0)) m |= 1ull << l;
    return m;
}
// mask bit set ? if1 : if0 (v_cndmask with an SGPR-pair condition)
__device__ __forceinline__ uint32_t cnd_u32(uint64_t m, uint32_t if0, uint32_t if1) {
    uint32_t r;
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(if0), "v"(if1), "s"(m));
    return r;
}
// The compile-time lane mask M in an SGPR pair, materialized right here (two s_mov_b32):
// as plain constants the compiler hoists every stage's mask out of the unit loop and, short
// of SGPRs, spills them to VGPR lanes -- a v_readlane pair (VALU) per bitonic stage instead
// of two scalar moves.
template <uint64_t M>
__device__ __forceinline__ uint64_t lane_mask() {
    uint32_t lo, hi;
    asm volatile("s_mov_b32 %0, %2\n\ts_mov_b32 %1, %3" : "=s"(lo), "=s"(hi)
                 : "i"((uint32_t)M), "i"((uint32_t)(M >> 32)));
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ double cnd_f64(uint64_t m, double if0, double if1) {
    const uint64_t a = (uint64_t)__double_as_longlong(if0), b = (uint64_t)__double_as_longlong(if1);
    const uint32_t lo = cnd_u32(m, (uint32_t)a, (uint32_t)b);
    const uint32_t hi = cnd_u32(m, (uint32_t)(a >> 32), (uint32_t)(b >> 32));
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
// {own, partner at lane ^ J} as an unordered pair: for J in {16, 32} a permlane swap of a
// register with itself leaves each lane holding both; for J < 16 (own, DPP partner)
template <int J>
__device__ __forceinline__ void xor_pair_f64(double x, double& p0, double& p1) {
    const uint64_t b = (uint64_t)__double_as_longlong(x);
    if constexpr (J >= 16) {
        const uint32_t lo = (uint32_t)b, hi = (uint32_t)(b >> 32);
        uint32_t l0, l1, h0, h1;
        if constexpr (J == 16) {
            const auto rl = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
            const auto rh = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
            l0 = rl[0], l1 = rl[1], h0 = rh[0], h1 = rh[1];
        } else {
            const auto rl = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
            const auto rh = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
            l0 = rl[0], l1 = rl[1], h0 = rh[0], h1 = rh[1];
        }
        p0 = __longlong_as_double((long long)(((uint64_t)h0 << 32) | l0));
        p1 = __longlong_as_double((long long)(((uint64_t)h1 << 32) | l1));
    } else {
        p0 = x;
        p1 = __longlong_as_double((long long)(((uint64_t)xor_lanes<J>((uint32_t)(b >> 32)) << 32) |
                                              xor_lanes<J>((uint32_t)b)));
    }
}
template <int J>
__device__ __forceinline__ void xor_pair_u32(uint32_t x, uint32_t& p0, uint32_t& p1) {
    if constexpr (J == 16) {
        const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
        p0 = r[0], p1 = r[1];
    } else if constexpr (J == 32) {
        const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
        p0 = r[0], p1 = r[1];
    } else {
        p0 = x, p1 = xor_lanes<J>(x);
    }
}

template <int R, int K, int J>
__device__ __forceinline__ void bitonic_f64_stages(double (&v)[R]) {
    if constexpr (J >= WAVE) {   // register-local: the role depends on r only
        constexpr int rj = J / WAVE;
        static_for<0, R>([&](auto rc) {
            constexpr int r = decltype(rc)::value;
            if constexpr ((r & rj) == 0) {
                constexpr bool up = ((WAVE * r) & K) == 0;
                const double mn = hw_min(v[r], v[r | rj]), mx = hw_max(v[r], v[r | rj]);
                v[r] = up ? mn : mx;
                v[r | rj] = up ? mx : mn;
            }
        });
    } else {
        static_for<0, R>([&](auto rc) {
            constexpr int r = decltype(rc)::value;
            double p0, p1;
            xor_pair_f64<J>(v[r], p0, p1);
            const double mn = hw_min(p0, p1), mx = hw_max(p0, p1);
            v[r] = cnd_f64(lane_mask<bitonic_min_mask<K, J, r>()>(), mx, mn);
        });
    }
    if constexpr (J > 1) bitonic_f64_stages<R, K, J / 2>(v);
}

// Non-NaN doubles (element e = lane + 64 r in register r): bitonic sort ascending with the
// hardware min / max (no 64-bit integer compares and selects).  Cross-lane stages exchange
// through DPP / permlane swaps (no LDS round trip); min and max are both computed and a
// constant lane mask picks one (inline asm is convergent: a conditional one would branch).
template <int R, int K = 2>
__device__ __forceinline__ void wave_sort_f64(double (&v)[R]) {
    bitonic_f64_stages<R, K, K / 2>(v);
    if constexpr (K < WAVE * R) wave_sort_f64<R, K * 2>(v);
}

template <int R, int K, int J>
__device__ __forceinline__ void bitonic_u32_stages(uint32_t (&v)[R]) {
    if constexpr (J >= WAVE) {   // register-local: the role depends on r only
        constexpr int rj = J / WAVE;
        static_for<0, R>([&](auto rc) {
            constexpr int r = decltype(rc)::value;
            if constexpr ((r & rj) == 0) {
                constexpr bool up = ((WAVE * r) & K) == 0;
                const uint32_t a = v[r], b = v[r | rj];
                const uint32_t mn = a < b ? a : b, mx = a < b ? b : a;
                v[r] = up ? mn : mx;
                v[r | rj] = up ? mx : mn;
            }
        });
    } else {
        static_for<0, R>([&](auto rc) {
            constexpr int r = decltype(rc)::value;
            uint32_t p0, p1;
            xor_pair_u32<J>(v[r], p0, p1);
            const uint32_t mn = p0 < p1 ? p0 : p1, mx = p0 < p1 ? p1 : p0;
            v[r] = cnd_u32(lane_mask<bitonic_min_mask<K, J, r>()>(), mx, mn);
        });
    }
    if constexpr (J > 1) bitonic_u32_stages<R, K, J / 2>(v);
}

// 32-bit keys: one wave sorts its 64 R values ascending (element e = lane + 64 r in register
// r): one DPP / permlane exchange, a min, a max and a lane-mask select per register and
// stage below 64, a register-local min / max at and above it (R = 1: 21 stages; R = 2: 28).
template <int R, int K = 2>
__device__ __forceinline__ void wave_sort32(uint32_t (&v)[R]) {
    static_assert(R == 1 || R == 2 || R == 4, "wave_sort32: 1, 2 or 4 registers");
    bitonic_u32_stages<R, K, K / 2>(v);
    if constexpr (K < WAVE * R) wave_sort32<R, K * 2>(v);
}

// 64-bit keys, the same scheme: the partner by DPP / permlane (per 32-bit half), ONE 64-bit
// compare into a lane mask, and the lane's role as a compile-time mask -- a lane takes the
// partner iff (partner < own) == (the lane keeps the minimum): an s_xnor and two v_cndmask
// per register and stage (the generic wave_sort spends lane arithmetic and four selects).
template <int R, int K, int J>
__device__ __forceinline__ void bitonic_u64_stages(uint64_t (&v)[R]) {
    if constexpr (J >= WAVE) {
        constexpr int rj = J / WAVE;
        static_for<0, R>([&](auto rc) {
            constexpr int r = decltype(rc)::value;
            if constexpr ((r & rj) == 0) {
                constexpr bool up = ((WAVE * r) & K) == 0;
                const uint64_t a = v[r], b = v[r | rj];
                const uint64_t mn = a < b ? a : b, mx = a < b ? b : a;
                v[r] = up ? mn : mx;
                v[r | rj] = up ? mx : mn;
            }
        });
    } else {
        static_for<0, R>([&](auto rc) {
            constexpr int r = decltype(rc)::value;
            const uint64_t p = xor_lane<J>(v[r]);
            const uint64_t lt = __ballot(p < v[r]);
            const uint64_t take = ~(lt ^ lane_mask<bitonic_min_mask<K, J, r>()>());
            const uint32_t lo = cnd_u32(take, (uint32_t)v[r], (uint32_t)p);
            const uint32_t hi = cnd_u32(take, (uint32_t)(v[r] >> 32), (uint32_t)(p >> 32));
            v[r] = ((uint64_t)hi << 32) | lo;
        });
    }
    if constexpr (J > 1) bitonic_u64_stages<R, K, J / 2>(v);
}

// One wave sorts its 64 R 64-bit keys ascending (element e = lane + 64 r in register r); the
// whole wave must be active (the compare is a ballot).
template <int R, int K = 2>
__device__ __forceinline__ void wave_sort64(uint64_t (&v)[R]) {
    bitonic_u64_stages<R, K, K / 2>(v);
    if constexpr (K < WAVE * R) wave_sort64<R, K * 2>(v);
}

// The q-th smallest (1-based, q <= 128) of the 128 keys a, b held by the wave's lanes: the
// same bisection, two ballot counts per bit
__device__ __forceinline__ uint32_t wave_kth_u32_of2(uint32_t a, uint32_t b, int q) {
    uint32_t t = 0;
#pragma unroll
    for (int bit = 31; bit >= 0; --bit) {
        const uint32_t m = t | ((1u << bit) - 1u);
        const int c = (int)__popcll(__ballot(a <= m)) + (int)__popcll(__ballot(b <= m));
        t |= c < q ? (1u << bit) : 0u;
    }
    return t;
}

// Bitonic sort (ascending) of the 64*R keys held by one wave (element e = lane + 64*r in
// register r); the whole wave active
template <int R>
__device__ __forceinline__ void wave_sort(uint64_t (&v)[R]) {
    wave_sort64<R>(v);
}

// The q-th smallest (1-based, q <= 64) of the wave's lane keys a, and the r-th of b: MSB-first
// bisection on the key bits, one ballot count per bit and key (uniform results; no sort)
__device__ __forceinline__ void wave_kth_u32x2(uint32_t a, int q, uint32_t b, int r, uint32_t& ka, uint32_t& kb) {
    uint32_t ta = 0, tb = 0;
#pragma unroll
    for (int bit = 31; bit >= 0; --bit) {
        const uint32_t m = (1u << bit) - 1u;
        const int ca = (int)__popcll(__ballot(a <= (ta | m)));
        const int cb = (int)__popcll(__ballot(b <= (tb | m)));
        ta |= ca < q ? (1u << bit) : 0u;
        tb |= cb < r ? (1u << bit) : 0u;
    }
    ka = ta;
    kb = tb;
}

// Element e (wave-uniform, < 64 R) of a wave-distributed u32 array: one readlane per register,
// the register picked by scalar selects.
template <int R>
__device__ __forceinline__ uint32_t wave_at_u32(const uint32_t (&v)[R], int e) {
    const int q = e >> 6, l = e & 63;
    uint32_t x = (uint32_t)__builtin_amdgcn_readlane((int)v[0], l);
    static_for<1, R>([&](auto rc) {
        constexpr int r = decltype(rc)::value;
        const uint32_t t = (uint32_t)__builtin_amdgcn_readlane((int)v[r], l);
        x = q == r ? t : x;
    });
    return x;
}

// Sort buf[0..c) (c <= 64*R) in place with one wave; entries c..64R-1 become SENT.
template <int R>
__device__ __forceinline__ void wave_sort_lds(uint64_t* buf, int c) {
    const int lane = lane_id();
    uint64_t v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int e = lane + WAVE * r;
        v[r] = e < c ? buf[e] : SENT;
    }
    wave_sort<R>(v);
#pragma unroll
    for (int r = 0; r < R; ++r) buf[lane + WAVE * r] = v[r];
}

// ---------------------------------------------------------------------------------------
// hist_select: exact keys at up to four ascending ranks by an adaptive histogram over the
// order-preserving uint64 keys (a two-level radix select with data-dependent digits).
//   level 1: the key range [kmin, kmax] is cut into <= HB bins of 2^shift consecutive keys
//            (bin = (key - kmin) >> shift, monotone, no rounding anywhere); one LDS
//            histogram pass, one block scan, each target rank located in its bin;
//   then:    every located bin holding <= HCAP keys is compacted into an LDS list (one
//            list per distinct bin) and sorted by one wave; a bigger bin is refined by the
//            next level on that bin's key range (11 more bits each level; a bin of width 1
//            holds one distinct key, which is the answer).
// `for_each(f)` calls f(x) for each of this thread's values (NaN = absent): register-resident
// values or a grid-stride stream over HBM (long segments), the same code either way.  n,
// kmin, kmax describe the non-NaN values; block-uniform control flow; barriers inside.
// probe builds of fm_select.hip only (tools/tail_probe.py): phase marks of hist_select
#if FM_PROBE && defined(FM_HS_PROBE_ON)
#define FM_HS_PROBE(slot) FM_PROBE_AT(sel, slot)
#else
#define FM_HS_PROBE(slot) \
    do {                  \
    } while (0)
#endif
template <int NW, int HBN, int CAP, typename Sm, typename ForEach>
__device__ __forceinline__ void hist_select_t(ForEach&& for_each, int nr, const int* rk, uint64_t kmin,
                                              uint64_t kmax, uint64_t* out, Sm& sm) {
    constexpr int NT = NW * WAVE;
    const int tid = threadIdx.x;
    uint64_t tlo[4], thi[4];
    int tr[4];
    bool done[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        tlo[t] = kmin;
        thi[t] = kmax;
        tr[t] = t < nr ? rk[t] : 0;
        done[t] = t >= nr;
        out[t] = kmin;
    }
    bool shrink[4] = {false, false, false, false};
    // at most 4 groups x 8 levels (>= 8 bits each) are ever needed; the bound only guards
    for (int it = 0; it < 32; ++it) {
        int t0 = -1;
#pragma unroll
        for (int t = 3; t >= 0; --t)
            if (!done[t]) t0 = t;
        if (t0 < 0) break;   // block-uniform
        uint64_t lo = tlo[0], hi = thi[0];
        bool shr = false;
#pragma unroll
        for (int t = 0; t < 4; ++t)
            if (t == t0) lo = tlo[t], hi = thi[t], shr = shrink[t];
        bool grp[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) grp[t] = !done[t] && tlo[t] == lo && thi[t] == hi;
        if (shr) {
            // a refined bin: shrink its range to the keys actually present (a bin of equal
            // keys -- ties -- is answered right here)
            uint64_t mn = SENT, mx = 0;
            for_each([&](double x) {
                if (!isnan(x)) {
                    const uint64_t k = dkey(x);
                    if (k >= lo && k <= hi) {
                        mn = k < mn ? k : mn;
                        mx = k > mx ? k : mx;
                    }
                }
            });
            mn = block_min_u64<NW>(mn, sm.u64s);
            mx = block_max_u64<NW>(mx, sm.u64s + NW);
#pragma unroll
            for (int t = 0; t < 4; ++t)
                if (grp[t]) {
                    tlo[t] = mn;
                    thi[t] = mx;
                    shrink[t] = false;
                    if (mn == mx) {
                        out[t] = mn;
                        done[t] = true;
                    }
                }
            lo = mn;
            hi = mx;
            if (mn == mx) continue;   // block-uniform
        }
        const uint64_t span = hi - lo;
        constexpr int LB = HBN == 2048 ? 11 : HBN == 1024 ? 10 : HBN == 512 ? 9 : 8;
        static_assert((1 << LB) == HBN, "hist_select: HBN must be 256 .. 2048, a power of two");
        const int shift = span < (uint64_t)HBN ? 0 : 64 - __clzll(span) - LB;   // span >> shift < HBN
        for (int i = tid; i < HBN; i += NT) sm.hist[i] = 0u;
        __syncthreads();
        for_each([&](double x) {
            if (!isnan(x)) {
                const uint64_t k = dkey(x);
                if (k >= lo && k <= hi) atomicAdd(&sm.hist[(uint32_t)((k - lo) >> shift)], 1u);
            }
        });
        __syncthreads();
        FM_HS_PROBE(4);
        // block scan: thread tid owns bins [8 tid, 8 tid + 8)
        constexpr int BPT = HBN / NT;
        uint32_t h[BPT];
        int loc = 0;
#pragma unroll
        for (int j = 0; j < BPT; ++j) {
            h[j] = sm.hist[BPT * tid + j];
            loc += (int)h[j];
        }
        int tot = 0;
        int run = block_excl_scan<NW>(loc, sm.ints, &tot);
#pragma unroll
        for (int j = 0; j < BPT; ++j) {
#pragma unroll
            for (int t = 0; t < 4; ++t)
                if (grp[t] && run <= tr[t] && tr[t] < run + (int)h[j]) {
                    sm.hs[3 * t] = BPT * tid + j;
                    sm.hs[3 * t + 1] = run;
                    sm.hs[3 * t + 2] = (int)h[j];
                }
            run += (int)h[j];
        }
        __syncthreads();
        FM_HS_PROBE(5);
        uint64_t blo[4], bhi[4];
        int lst[4], lrank[4], lcnt[4];
        bool any_list = false;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            lst[t] = -1;
            lrank[t] = 0;
            lcnt[t] = 0;
            blo[t] = bhi[t] = 0;
            if (!grp[t]) continue;
            const int b = sm.hs[3 * t], below = sm.hs[3 * t + 1], cnt = sm.hs[3 * t + 2];
            const uint64_t wm1 = shift == 0 ? 0ull : (1ull << shift) - 1ull;
            blo[t] = lo + ((uint64_t)b << shift);
            bhi[t] = hi - blo[t] < wm1 ? hi : blo[t] + wm1;
            if (blo[t] == bhi[t]) {           // one distinct key in the bin: it is the answer
                out[t] = blo[t];
                done[t] = true;
            } else if (cnt <= CAP) {         // compact + sort
                lrank[t] = tr[t] - below;
                lcnt[t] = cnt;
                any_list = true;
            } else {                          // refine the bin at the next level
                tlo[t] = blo[t];
                thi[t] = bhi[t];
                tr[t] -= below;
                shrink[t] = true;
            }
        }
        if (!any_list) continue;
        // one list per distinct bin (targets i and i+1 usually share one)
        int nl = 0;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const bool listed = grp[t] && !done[t] && tlo[t] == lo && thi[t] == hi && lcnt[t] > 0;
            if (!listed) continue;
            int u = -1;
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (q < t && lst[q] >= 0 && blo[q] == blo[t]) u = lst[q];
            lst[t] = u >= 0 ? u : nl++;
        }
        if (tid < 4) sm.hcnt[tid] = 0u;
        __syncthreads();
        uint64_t ulo[4], uhi[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) ulo[u] = 1, uhi[u] = 0;   // empty ranges
#pragma unroll
        for (int t = 0; t < 4; ++t)
            if (lst[t] >= 0) {
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    if (u == lst[t]) ulo[u] = blo[t], uhi[u] = bhi[t];
            }
        for_each([&](double x) {
            if (!isnan(x)) {
                const uint64_t k = dkey(x);
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    if (u < nl && k >= ulo[u] && k <= uhi[u]) {   // nl: block-uniform (usually 2)
                        const uint32_t pos = atomicAdd(&sm.hcnt[u], 1u);
                        if (pos < (uint32_t)CAP) sm.buf[u * CAP + pos] = k;
                    }
            }
        });
        __syncthreads();
        FM_HS_PROBE(6);
        for (int w = tid / WAVE; w < nl; w += NW) {   // one wave per list
            const int c = (int)sm.hcnt[w];
            uint64_t* L = sm.buf + w * CAP;
            if (c <= WAVE) wave_sort_lds<1>(L, c);
            else if (CAP <= 2 * WAVE || c <= 2 * WAVE) wave_sort_lds<(CAP <= 2 * WAVE ? 2 : 2)>(L, c);
            else wave_sort_lds<(CAP > 2 * WAVE ? 4 : 2)>(L, c);
        }
        __syncthreads();
        FM_HS_PROBE(7);
#pragma unroll
        for (int t = 0; t < 4; ++t)
            if (lst[t] >= 0) {
                out[t] = sm.buf[lst[t] * CAP + lrank[t]];
                done[t] = true;
            }
        __syncthreads();   // lists and histogram are reused by the next level / caller
    }
}

template <int NW = SNW, typename ForEach>
__device__ __forceinline__ void hist_select(ForEach&& for_each, int nr, const int* rk, uint64_t kmin,
                                            uint64_t kmax, uint64_t* out, SelSmemT<NW>& sm) {
    hist_select_t<NW, HB, HCAP>(for_each, nr, rk, kmin, kmax, out, sm);
}

// Number of entries of the ascending list L[0..64) that precede v in the merged order:
// entries < v, or <= v when the list's wave comes first (ties broken by wave).
__device__ __forceinline__ int merge_count(const uint64_t* L, uint64_t v, bool inclusive) {
    int lo = 0;
#pragma unroll
    for (int step = 32; step > 0; step >>= 1) {
        const uint64_t x = L[lo + step - 1];
        lo += (x < v || (inclusive && x == v)) ? step : 0;
    }
    const uint64_t x = L[lo < WAVE ? lo : WAVE - 1];
    lo += (lo < WAVE && (x < v || (inclusive && x == v))) ? 1 : 0;
    return lo;
}

// Both winsorize tails at once, on the FP64 values xv (NaN = absent): keys at ranks
// li <= lj (lower tail) and hi_i <= hi_j (upper tail) among n valid values, thread minima
// mn / maxima mx.  Returns false (block-uniform, nothing written) when the fast path does
// not apply; the caller then takes the general path.
//   tau_lo = the lj-th smallest of the 256 thread minima (exact: per-wave bitonic sort,
//   then each lane's rank in the merged order by binary search in the other waves' lists).
//   lj+1 threads own a value <= tau_lo, so s[lj] <= tau_lo, and only the values < tau_lo
//   (a few more than lj) can precede it: they are compacted with one packed scan and
//   sorted by one wave.  The upper tail is the same on complemented keys of the maxima.
template <int VPT, int NW = SNW>
__device__ __forceinline__ bool select_tails(const double (&xv)[VPT], double mn, double mx, int n,
                                             int li, int lj, int hi_i, int hi_j, uint64_t& k0,
                                             uint64_t& k1, uint64_t& k2, uint64_t& k3, SelSmemT<NW>& sm) {
    constexpr int NT = NW * WAVE;
    // candidate list capacity per tail (4 * 64 keys; 8 * 64 for the 8-wave long-month path)
    constexpr int CC = NW >= 8 ? 8 * WAVE : 4 * WAVE;
    static_assert(2 * NT + 2 * (CAND_CAP / 4) <= CAND_CAP && CC <= CAND_CAP / 4, "select_tails: LDS layout");
    const int ci = n - 1 - hi_j, cj = n - 1 - hi_i;   // upper-tail ranks in complemented order
    if (lj >= NT || cj >= NT) return false;
    uint64_t a[1] = {isnan(mn) ? SENT : dkey(mn)};
    uint64_t b[1] = {isnan(mx) ? SENT : ~dkey(mx)};
    wave_sort<1>(a);
    wave_sort<1>(b);
    const int w = threadIdx.x / WAVE, lane = lane_id();
    uint64_t* Llo = sm.buf + CAND_CAP - 2 * NT;         // [NW][64] sorted thread minima
    uint64_t* Lhi = sm.buf + CAND_CAP - NT;             // [NW][64] sorted complemented maxima
    __syncthreads();   // sm.buf may still be read by a previous phase
    Llo[w * WAVE + lane] = a[0];
    Lhi[w * WAVE + lane] = b[0];
    if (threadIdx.x < 2) sm.bc[threadIdx.x] = SENT;
    __syncthreads();
    // merged rank of this lane's entries (ranks >= lane, so only lanes <= lj / cj matter)
    if (lane <= lj && a[0] != SENT) {
        int r = lane;
#pragma unroll
        for (int u = 0; u < NW; ++u)
            if (u != w) r += merge_count(Llo + u * WAVE, a[0], u < w);
        if (r == lj) sm.bc[0] = a[0];
    }
    if (lane <= cj && b[0] != SENT) {
        int r = lane;
#pragma unroll
        for (int u = 0; u < NW; ++u)
            if (u != w) r += merge_count(Lhi + u * WAVE, b[0], u < w);
        if (r == cj) sm.bc[1] = b[0];
    }
    __syncthreads();
    const uint64_t tlo_k = sm.bc[0], thi_k = sm.bc[1];
    if (tlo_k == SENT || thi_k == SENT) return false;   // fewer valid thread minima than needed
    const double tlo = kval(tlo_k), thi = kval(~thi_k);
    int cnt = 0;
#pragma unroll
    for (int v = 0; v < VPT; ++v) cnt += (xv[v] < tlo ? 1 : 0) + (xv[v] > thi ? 0x10000 : 0);
    int tot = 0;
    const int off = block_excl_scan<NW>(cnt, sm.ints, &tot);
    const int clo = tot & 0xFFFF, chi = tot >> 16;
    constexpr int HALF = CAND_CAP / 4;
    if (clo > CC || chi > CC) return false;   // block-uniform
    {
        int ol = off & 0xFFFF, oh = HALF + (off >> 16);
#pragma unroll
        for (int v = 0; v < VPT; ++v) {
            // recompute the compares (the counting pass's would stay live as SGPR masks)
            double x = xv[v];
            asm volatile("" : "+v"(x));
            if (x < tlo) sm.buf[ol++] = dkey(x);
            if (x > thi) sm.buf[oh++] = ~dkey(x);
        }
        __syncthreads();
    }
    if (w == 0) {
        if (clo <= WAVE) wave_sort_lds<1>(sm.buf, clo);
        else if (clo <= 2 * WAVE) wave_sort_lds<2>(sm.buf, clo);
        else if (CC <= 4 * WAVE || clo <= 4 * WAVE) wave_sort_lds<4>(sm.buf, clo);
        else wave_sort_lds<(CC > 4 * WAVE ? 8 : 4)>(sm.buf, clo);
    } else if (w == 1) {
        if (chi <= WAVE) wave_sort_lds<1>(sm.buf + HALF, chi);
        else if (chi <= 2 * WAVE) wave_sort_lds<2>(sm.buf + HALF, chi);
        else if (CC <= 4 * WAVE || chi <= 4 * WAVE) wave_sort_lds<4>(sm.buf + HALF, chi);
        else wave_sort_lds<(CC > 4 * WAVE ? 8 : 4)>(sm.buf + HALF, chi);
    }
    __syncthreads();
    k0 = li < clo ? sm.buf[li] : tlo_k;
    k1 = lj < clo ? sm.buf[lj] : tlo_k;
    const uint64_t ca = ci < chi ? sm.buf[HALF + ci] : thi_k;
    const uint64_t cb = cj < chi ? sm.buf[HALF + cj] : thi_k;
    k3 = ~ca;   // rank hi_j (complemented rank ci)
    k2 = ~cb;   // rank hi_i
    return true;
}

// numpy 'linear' (mode 0, function_base._quantile/_lerp) or pandas group_quantile (mode 1)
__device__ __forceinline__ void qranks(int n, double q, int mode, int& i, int& j, double& g) {
    if (mode == 0) {
        const double vi = (double)(n - 1) * q;
        if (vi >= (double)(n - 1)) {
            i = j = n - 1;
            g = vi + 1.0;  // numpy: gamma = vi - (-1)
        } else {
            const double f = floor(vi);
            i = (int)f;
            j = i + 1;
            g = vi - f;
        }
    } else {
        const double qi = q * (double)(n - 1);
        i = (int)qi;
        g = qi - floor(qi);
        j = g == 0.0 ? i : i + 1;
    }
}

__device__ __forceinline__ double qlerp(double a, double b, double g, int mode) {
    if (mode == 0) {
        const double d = b - a;
        return g >= 0.5 ? b - d * (1.0 - g) : a + d * g;
    }
    return g == 0.0 ? a : a + (b - a) * g;
}

// One (segment, column) unit on a 256-thread workgroup: the general path (any ranks, row
// masks, up to 96 * 256 rows).  Block-uniform control flow.
template <int VPT, int NW = SNW, bool MARK = false>
__device__ __forceinline__ void select_unit_wg(const SelArgs& a, int s, int c, SelSmemT<NW>& sm) {
    constexpr int NT = NW * WAVE;
    const int64_t r0 = a.seg_off[s];
    const int L = (int)(a.seg_off[s + 1] - r0);
    const double* src = a.cols + (int64_t)c * a.col_stride + r0;
    // Unconditional loads (index clamped, masked after): a load under a runtime condition
    // makes hipcc wait vmcnt(0) per load and serializes the HBM round trips.
    // Wave-uniform base (SGPRs) + the lane's 32-bit byte offset: no 64-bit address per load.
    typedef const __attribute__((address_space(1))) char* gptr;
    const uint32_t lastb = (uint32_t)(L > 0 ? L - 1 : 0) * 8u;
    uint32_t lb = (uint32_t)threadIdx.x * 8u;
    asm volatile("" : "+v"(lb));
    double xv[VPT];
    if (a.cols == nullptr) {   // block-uniform: a split panel without FP64 columns (fix-up path)
        const PCols pc = sel_col(a, c, r0);
#pragma unroll
        for (int v = 0; v < VPT; ++v) {
            const uint32_t off = lb + (uint32_t)(v * NT * 8);
            const uint32_t oc = off < lastb ? off : lastb;
            const double x = pc[oc >> 3];
            const bool m = a.mask == nullptr || a.mask[r0 + (oc >> 3)] != 0;
            xv[v] = (off <= lastb && L > 0 && m) ? x : NAN;
        }
    } else if (a.mask == nullptr) {   // block-uniform
#pragma unroll
        for (int v = 0; v < VPT; ++v) {
            const uint32_t off = lb + (uint32_t)(v * NT * 8);
            const double x = *(const __attribute__((address_space(1))) double*)((gptr)src + (off < lastb ? off : lastb));
            xv[v] = off <= lastb && L > 0 ? x : NAN;
        }
    } else {
        const gptr mb = (gptr)(a.mask + r0);
#pragma unroll
        for (int v = 0; v < VPT; ++v) {
            const uint32_t off = lb + (uint32_t)(v * NT * 8);
            const uint32_t oc = off < lastb ? off : lastb;
            const double x = *(const __attribute__((address_space(1))) double*)((gptr)src + oc);
            const uint8_t m = *(mb + (oc >> 3));
            xv[v] = (off <= lastb && L > 0 && m != 0) ? x : NAN;
        }
    }
    // thread count / min / max (NaN-ignoring hardware min / max)
    int cnt = 0;
    double mn = NAN, mx = NAN;
#pragma unroll
    for (int v = 0; v < VPT; ++v) {
        cnt += isnan(xv[v]) ? 0 : 1;
        mn = hw_min(mn, xv[v]);
        mx = hw_max(mx, xv[v]);
    }
    const int n = block_sum<NW>(cnt, sm.ints);
    double lo = NAN, hi = NAN;
    const bool apply = n >= a.min_count && n > 0;
    if (apply) {
        int i0, j0, i1, j1;
        double g0, g1;
        qranks(n, a.q_lo, a.lerp_mode, i0, j0, g0);
        qranks(n, a.q_hi, a.lerp_mode, i1, j1, g1);
        uint64_t k0, k1, k2, k3;
        const bool fast = select_tails<VPT, NW>(xv, mn, mx, n, i0, j0, i1, j1, k0, k1, k2, k3, sm);
        if (MARK && !fast) {
            // MARK: the rare unit the tail path cannot finish is redone by a fallback pass
            if (threadIdx.x == 0) sel_mark(a, (int64_t)c * a.nseg + s);
            return;
        }
        if (!MARK && !fast) {
            // any ranks (pandas middle quantiles, overflowing tails): adaptive histogram
            uint64_t kmn = SENT, kmx = 0;
#pragma unroll
            for (int v = 0; v < VPT; ++v)
                if (!isnan(xv[v])) {
                    const uint64_t k = dkey(xv[v]);
                    kmn = k < kmn ? k : kmn;
                    kmx = k > kmx ? k : kmx;
                }
            kmn = block_min_u64<NW>(kmn, sm.u64s);
            kmx = block_max_u64<NW>(kmx, sm.u64s + NW);
            const int rk[4] = {i0, j0, i1, j1};
            uint64_t ko[4];
            hist_select<NW>([&](auto&& f) {
#pragma unroll
                for (int v = 0; v < VPT; ++v) f(xv[v]);
            }, 4, rk, kmn, kmx, ko, sm);
            k0 = ko[0], k1 = ko[1], k2 = ko[2], k3 = ko[3];
        }
        lo = qlerp(kval(k0), kval(k1), g0, a.lerp_mode);
        hi = qlerp(kval(k2), kval(k3), g1, a.lerp_mode);
    }
    if (a.center != nullptr) {
        // Gram pivot: the midpoint of the cuts, else of the values' range, else 0 (block-
        // uniform branch: lo / hi are block-uniform)
        double cen = 0.5 * (lo + hi);
        if (!isfinite(cen)) {
            const double m1 = block_min_f64<NW>(isfinite(mn) ? mn : NAN, sm.dbl);
            const double m2 = -block_min_f64<NW>(isfinite(mx) ? -mx : NAN, sm.dbl);
            cen = 0.5 * (m1 + m2);
            if (!isfinite(cen)) cen = 0.0;
        }
        if (threadIdx.x == 0) a.center[(int64_t)c * a.nseg + s] = cen;
    }
    if (!MARK && a.mean != nullptr) {   // (MARK callers route moment requests elsewhere)
        // Moments of the clipped values (pandas clip ignores NaN bounds).  One pass about a
        // pivot p inside the data (a finite cut, else the smallest finite value):
        // mean = p + S1/n, var = (S2 - S1^2/n)/(n-1).
        double p = isfinite(lo) ? lo : (isfinite(hi) ? hi : 0.0);
        if (!isfinite(lo) && !isfinite(hi)) {
            // no cuts (short month): pivot = the smallest finite value
            double m2 = isfinite(mn) ? mn : NAN;
            p = block_min_f64<NW>(m2, sm.dbl);
            if (!isfinite(p)) p = 0.0;
        }
        double s1 = 0.0, s2 = 0.0;
#pragma unroll
        for (int v = 0; v < VPT; ++v) {
            double x = xv[v];
            if (x < lo) x = lo;
            if (x > hi) x = hi;
            const double d = isnan(x) ? 0.0 : x - p;
            s1 += d;
            s2 = fma(d, d, s2);
        }
        double2 r = block_sum2<NW>(s1, s2, sm.dbl);
        if (threadIdx.x == 0) {
            const double mu = n > 0 ? p + r.x / (double)n : NAN;
            a.mean[(int64_t)c * a.nseg + s] = mu;
            if (a.sd) {
                double var = n > 1 ? (r.y - r.x * (r.x / (double)n)) / (double)(n - 1) : NAN;
                if (var < 0.0) var = 0.0;
                a.sd[(int64_t)c * a.nseg + s] = n > 1 ? sqrt(var) : NAN;
            }
        }
    }
    if (threadIdx.x == 0) {
        const int64_t o = (int64_t)c * a.nseg + s;
        a.lo[o] = lo;
        a.hi[o] = hi;
        if (a.nvalid) a.nvalid[o] = n;
        if (zero_cut(a, lo, hi)) sel_push(a, o);
        if (a.prm) {
            a.prm[c] = lo;
            a.prm[32 + c] = hi;
            a.prm[64 + c] = a.center ? a.center[o] : 0.0;
        }
    }
}

// fallback == 0: one unit per workgroup (grid nseg x ncols).  fallback == 1: a fixed grid
// that walks every unit and redoes those the wave kernel marked with nvalid == -1.

// ---------------------------------------------------------------------------------------
// Wave-per-unit fast path for the winsorize tails (no row mask): one wave holds a whole
// (segment, column) in registers (VPL values per lane, element lane + 64 v), so there is
// no workgroup barrier at all and twice as many units per CU are in flight as with the
// workgroup kernel.  Per unit:
//   * n, lane minima / maxima; tau_lo = the lj-th smallest lane minimum (one 64-key wave
//     bitonic sort): lj+1 lanes own a value <= tau_lo, so s[lj] <= tau_lo, and only the
//     values < tau_lo can precede it.  Same for the upper tail on complemented keys.
//   * those candidates (about 1.8% of n at n = 5000) are compacted by ballot + mbcnt into
//     the wave's LDS list and sorted by a 128-key wave bitonic sort; the order statistics
//     are read at wave-uniform positions.
// Units the fast path cannot finish (ranks >= 64, more than 128 candidates, fewer lanes
// with a valid value than the rank) get nvalid = -1 and are redone by the workgroup
// kernel's fallback pass.  Results are exact order statistics either way.
constexpr int WCAP = 256;

// Values at ascending ranks ra <= rb among the c candidates L[0..c) (c <= 64 R), or tau
// when a rank is >= c (then the order statistic is tau itself, a data value).
template <int R>
__device__ __forceinline__ void pick_tail(const double* L, int c, int ra, int rb, double tau, double& va,
                                          double& vb) {
    const int lane = lane_id();
    double v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int e = lane + WAVE * r;
        v[r] = e < c ? L[e] : INFINITY;
    }
    wave_sort_f64<R>(v);
    auto at = [&](int e) -> double {
        // lane e & 63 of every register read out (scalar), then a scalar pick of register
        // e >> 6: selecting the register first becomes a dynamically indexed stack array
        // (scratch round trips)
        const int q = e >> 6, l = e & 63;
        uint64_t x = readlane_u64((uint64_t)__double_as_longlong(v[0]), l);
        static_for<1, R>([&](auto rc) {
            constexpr int r = decltype(rc)::value;
            const uint64_t t = readlane_u64((uint64_t)__double_as_longlong(v[r]), l);
            x = q == r ? t : x;
        });
        return __longlong_as_double((long long)x);
    };
    va = ra < c ? at(ra) : tau;
    vb = rb < c ? at(rb) : tau;
}

// pick_tail over the concatenation of two LDS candidate lists L1[0..c1) ++ L2[0..c2)
template <int R>
__device__ __forceinline__ void pick_tail2(const double* L1, int c1, const double* L2, int c2, int ra, int rb,
                                           double tau, double& va, double& vb) {
    const int lane = lane_id();
    const int c = c1 + c2;
    double v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int e = lane + WAVE * r;
        v[r] = e < c1 ? L1[e] : (e < c ? L2[e - c1] : INFINITY);
    }
    wave_sort_f64<R>(v);
    auto at = [&](int e) -> double {
        // lane e & 63 of every register read out (scalar), then a scalar pick of register
        // e >> 6: selecting the register first becomes a dynamically indexed stack array
        // (scratch round trips)
        const int q = e >> 6, l = e & 63;
        uint64_t x = readlane_u64((uint64_t)__double_as_longlong(v[0]), l);
        static_for<1, R>([&](auto rc) {
            constexpr int r = decltype(rc)::value;
            const uint64_t t = readlane_u64((uint64_t)__double_as_longlong(v[r]), l);
            x = q == r ? t : x;
        });
        return __longlong_as_double((long long)x);
    };
    va = ra < c ? at(ra) : tau;
    vb = rb < c ? at(rb) : tau;
}

// Number of entries of the ascending u32 list L[0..64) below v (inclusive: <= v).
__device__ __forceinline__ int count_below_u32(const uint32_t* L, uint32_t v, bool inclusive) {
    int lo = 0;
#pragma unroll
    for (int step = 32; step > 0; step >>= 1) {
        const uint32_t x = L[lo + step - 1];
        lo += (x < v || (inclusive && x == v)) ? step : 0;
    }
    const uint32_t x = L[lo < WAVE ? lo : WAVE - 1];
    lo += (lo < WAVE && (x < v || (inclusive && x == v))) ? 1 : 0;
    return lo;
}



// ---------------------------------------------------------------------------------------
// One (segment, column) unit held by ONE wave (element lane + 64 v in register v, NaN =
// absent): both winsorize tails without any workgroup barrier.
//   * n, lane minima / maxima; tau_lo = the j0-th smallest lane minimum (one 64-key wave
//     bitonic sort of the keys' high words): j0+1 lanes own a value <= tau_lo, so
//     s[j0] <= tau_lo, and only the values < tau_lo can precede it.  Same for the upper
//     tail on complemented keys.
//   * those candidates (about 1.8% of n at n = 5000) are compacted by ballot + mbcnt into
//     the wave's LDS lists Ll / Lh (WCAP each) and sorted by a 128-key wave bitonic sort;
//     the order statistics are read at wave-uniform positions.
// `freed()` runs as soon as xv is no longer needed (the caller's prefetch of its next
// unit).  ok == false (ranks >= 64, more than WCAP candidates, fewer lanes with a valid
// value than the rank): nothing is decided, the caller takes an exact fallback.  The
// pivot `cen` is the midpoint of the cuts, else of the finite range, else 0.
struct WaveCut {
    double lo, hi, cen, mn, mx;
    int n;
    bool ok;
};

template <int VPL, typename F>
__device__ __forceinline__ WaveCut wave_cut(double (&xv)[VPL], int L, double q_lo, double q_hi,
                                            int min_count, int lerp_mode, double* Ll, double* Lh,
                                            F&& freed) {
    const int lane = lane_id();
    // min / max with 4 independent accumulators each (the chains would otherwise serialize
    // on the f64 latency); the count is scalar: ballot + popcount per row, no VALU
    int n = 0;
    double mn4[4] = {NAN, NAN, NAN, NAN}, mx4[4] = {NAN, NAN, NAN, NAN};
    const int vfull = L / WAVE;   // rows v < vfull lie inside the segment (wave-uniform)
    int lo_ = lane;
    asm volatile("" : "+v"(lo_));   // keep lane + v * WAVE from being hoisted
#pragma unroll
    for (int v = 0; v < VPL; ++v) {
        if (v >= vfull && lo_ + v * WAVE >= L) xv[v] = NAN;   // past the segment end
        n += (int)__popcll(__ballot(!isnan(xv[v])));
        mn4[v & 3] = hw_min(mn4[v & 3], xv[v]);   // NaN-ignoring, no canonicalized copy of xv
        mx4[v & 3] = hw_max(mx4[v & 3], xv[v]);
    }
    WaveCut r;
    r.mn = hw_min(hw_min(mn4[0], mn4[1]), hw_min(mn4[2], mn4[3]));
    r.mx = hw_max(hw_max(mx4[0], mx4[1]), hw_max(mx4[2], mx4[3]));
    r.n = n = __builtin_amdgcn_readfirstlane(n);
    r.lo = r.hi = NAN;
    r.ok = true;
    const bool apply = n >= min_count && n > 0;
    int i0 = 0, j0 = 0, i1 = 0, j1 = 0, clo = 0, chi = 0;
    double g0 = 0.0, g1 = 0.0, tlo = NAN, thi = NAN;
    if (apply) {
        qranks(n, q_lo, lerp_mode, i0, j0, g0);
        qranks(n, q_hi, lerp_mode, i1, j1, g1);
        const int cj = n - 1 - i1;   // upper rank in complemented order
        r.ok = j0 < WAVE && cj < WAVE;
        if (r.ok) {
            // tau from the high 32 bits of the keys (half the cost of a 64-bit sort): the
            // j0-th smallest high word T bounds j0+1 lane minima by key (T << 32 | ~0)
            const uint32_t ha = isnan(r.mn) ? 0xFFFFFFFFu : (uint32_t)(dkey(r.mn) >> 32);
            const uint32_t hb = isnan(r.mx) ? 0xFFFFFFFFu : (uint32_t)(~dkey(r.mx) >> 32);
            uint32_t ta[1] = {ha};
            uint32_t tb[1] = {hb};
            wave_sort32<1>(ta);
            wave_sort32<1>(tb);
            const uint32_t Ta = (uint32_t)__builtin_amdgcn_readlane((int)ta[0], j0);
            const uint32_t Tb = (uint32_t)__builtin_amdgcn_readlane((int)tb[0], cj);
            r.ok = Ta != 0xFFFFFFFFu && Tb != 0xFFFFFFFFu;
            if (r.ok) {
                // tau = the largest lane minimum whose high word is Ta: at least j0+1 lane
                // minima are <= it, and it is a data value, so ties at tau (e.g. many
                // exact zeros) stay out of the candidates instead of overflowing them
                tlo = ha == Ta ? r.mn : NAN;
                thi = hb == Tb ? r.mx : NAN;
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) {   // whole wave active: DPP / permlane
                    tlo = hw_max(tlo, xor_lanes_f64(tlo, o));
                    thi = hw_min(thi, xor_lanes_f64(thi, o));
                }
                // wave-uniform running counts; overflow is checked once
#pragma unroll
                for (int v = 0; v < VPL; ++v) {
                    if (FM_AB_SEL_NOCOMPACT) break;
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
                r.ok = clo <= WCAP && chi <= WCAP;
            }
        }
    }
    freed();   // xv is free from here on
    if (apply && r.ok) {
        double v0, v1, v2, v3;
        const int ci = n - 1 - j1, cj = n - 1 - i1;
        // LDS executes one wave's DS instructions in order; only the compiler's reordering
        // must be fenced
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // the candidates are never NaN: sort them as doubles (hardware min/max; equal values,
        // +0 / -0 included, are interchangeable for the result)
        if (FM_AB_SEL_NOSORT) {
            v0 = v1 = tlo;
            v2 = v3 = -thi;
        } else if (clo <= 2 * WAVE && chi <= 2 * WAVE) {
            pick_tail<2>(Ll, clo, i0, j0, tlo, v0, v1);
            pick_tail<2>(Lh, chi, ci, cj, -thi, v3, v2);
        } else {   // heavy tails: rare, 256 candidates
            pick_tail<4>(Ll, clo, i0, j0, tlo, v0, v1);
            pick_tail<4>(Lh, chi, ci, cj, -thi, v3, v2);
        }
        r.lo = qlerp(v0, v1, g0, lerp_mode);
        r.hi = qlerp(-v2, -v3, g1, lerp_mode);   // upper tail was stored negated
        // keep the LDS lists intact until every lane has read them (the next unit rewrites)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    // Gram pivot: the midpoint of the cuts, else of the values' range, else 0
    r.cen = 0.5 * (r.lo + r.hi);
    if (r.ok && !isfinite(r.cen)) {
        double m1 = isfinite(r.mn) ? r.mn : NAN, m2 = isfinite(r.mx) ? r.mx : NAN;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            m1 = hw_min(m1, xor_lanes_f64(m1, o));
            m2 = hw_max(m2, xor_lanes_f64(m2, o));
        }
        r.cen = 0.5 * (m1 + m2);
        if (!isfinite(r.cen)) r.cen = 0.0;
    }
    return r;
}

// Issue the loads of one segment column into xv (element lane + 64 v; nothing is used
// here: clamped 32-bit byte offsets from an SGPR base, masking happens at use, so the loads
// stay in flight while the caller keeps working).
template <int VPL>
__device__ __forceinline__ void load_seg_col(const double* src, int L, double (&xv)[VPL]) {
    typedef const __attribute__((address_space(1))) char* gptr;   // global_load, SGPR base
    const gptr b = (gptr)src;
    const uint32_t lastb = (uint32_t)(L > 0 ? L - 1 : 0) * 8u;
    // opaque lane offset: otherwise the loop-invariant per-row offsets are hoisted out of
    // the caller's unit loop and held in VGPRs for its whole length
    uint32_t lb = (uint32_t)lane_id() * 8u;
    asm volatile("" : "+v"(lb));
#pragma unroll
    for (int v = 0; v < VPL; ++v) {
        const uint32_t off = lb + (uint32_t)(v * WAVE * 8);
        if (FM_AB_SEL_NOLOAD)
            xv[v] = (double)((off * 2654435761u) >> 12) * 1e-6 + (double)(size_t)src * 1e-30;
        else
            xv[v] = *(const __attribute__((address_space(1))) double*)(b + (off < lastb ? off : lastb));
    }
}

}  // namespace
}  // namespace fm

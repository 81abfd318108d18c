// fm_select_cuts: exact per-(month, column) order statistics on gfx950.
//
// Replaces np.percentile(vals, 1/99) in winsorize (reference src/calc_Lewellen_2014.py:
// 519-523) and pandas groupby(...).quantile([.2,.5]) of NYSE `me` in get_subsets (:74-82).
//
// One 256-thread workgroup per (segment, column).  The segment's values live in
// registers as order-preserving uint64 keys (VPT per thread, one coalesced HBM read).
// Ranks near either tail (the 1%/99% winsorize cuts: rank ~n/100) take a fast path:
//   * the k-th smallest value is bounded above by tau = the k-th smallest of the 256
//     per-thread minima (k threads each own >= 1 value <= tau), so c_le(tau) >= k+1;
//   * at most k threads hold values < tau, so the candidates {x < tau} are few (about
//     k); they are compacted to LDS and ranked there by counting (no sort, few barriers).
// Middle ranks (pandas 0.2/0.5) and any overflow use an exact 8-bit LSD-free radix select
// (MSB-first histogram narrowing) over the register keys.  Results are the exact order
// statistics, so the interpolated cut is bit-identical to numpy/pandas given the same
// no-FMA lerp (this file is compiled with -ffp-contract=off).
#include <math.h>

#include "fm_common.h"

namespace fm {
namespace {

constexpr int ST = 256;
constexpr int SNW = ST / WAVE;
constexpr int CAND_CAP = 2048;

struct SelSmem {
    uint64_t buf[CAND_CAP];
    uint32_t hist[256];
    uint64_t u64s[SNW];
    double dbl[SNW];
    int ints[8];
    uint64_t bc[4];
};

struct SelArgs {
    const double* cols;
    int64_t col_stride;
    const int64_t* seg_off;
    int nseg;
    const uint8_t* mask;
    double q_lo, q_hi;
    int min_count;
    int lerp_mode;
    double* lo;
    double* hi;
    int32_t* nvalid;
    double* mean;
    double* sd;
};

// Exact key of the element at ascending rank `rank` (0-based) among non-SENT keys.
template <int VPT>
__device__ __forceinline__ uint64_t radix_rank(const uint64_t (&keys)[VPT], int rank, SelSmem& sm) {
    uint64_t prefix = 0, pmask = 0;
    int rem = rank;
    for (int shift = 56; shift >= 0; shift -= 8) {
        for (int i = threadIdx.x; i < 256; i += ST) sm.hist[i] = 0;
        __syncthreads();
#pragma unroll
        for (int v = 0; v < VPT; ++v) {
            const uint64_t k = keys[v];
            if (k != SENT && (k & pmask) == prefix) atomicAdd(&sm.hist[(k >> shift) & 255u], 1u);
        }
        __syncthreads();
        if (threadIdx.x < WAVE) {
            const int l = threadIdx.x;
            const int h0 = sm.hist[4 * l], h1 = sm.hist[4 * l + 1], h2 = sm.hist[4 * l + 2],
                      h3 = sm.hist[4 * l + 3];
            const int s = h0 + h1 + h2 + h3;
            int incl = s;
#pragma unroll
            for (int o = 1; o < WAVE; o <<= 1) {
                int y = __shfl_up(incl, o, WAVE);
                if (l >= o) incl += y;
            }
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

// Counting rank among LDS values buf[0..M): ascending, ties broken by index (unique ranks).
__device__ __forceinline__ int lds_rank(const uint64_t* buf, int M, uint64_t v, int self) {
    int r = 0;
    for (int u = 0; u < M; ++u) {
        const uint64_t x = buf[u];
        r += (x < v || (x == v && u < self)) ? 1 : 0;
    }
    return r;
}

// Keys at ascending ranks ri <= rj (< n) with the tail fast path; block-uniform.
// tau = the rj-th smallest of the 256 per-thread minima (found by counting ranks, no sort)
// bounds s[rj] from above; the few keys < tau are compacted to LDS and ranked by counting.
template <int VPT>
__device__ __forceinline__ void select_low(const uint64_t (&keys)[VPT], int ri, int rj, uint64_t& ki,
                           uint64_t& kj, SelSmem& sm) {
    bool done = false;
    if (rj < ST) {
        uint64_t m = SENT;
#pragma unroll
        for (int v = 0; v < VPT; ++v) m = keys[v] < m ? keys[v] : m;
        __syncthreads();
        sm.buf[threadIdx.x] = m;
        if (threadIdx.x == 0) sm.bc[0] = SENT;
        __syncthreads();
        if (lds_rank(sm.buf, ST, m, threadIdx.x) == rj) sm.bc[0] = m;
        __syncthreads();
        const uint64_t tau = sm.bc[0];
        if (tau != SENT) {
            int lt = 0;
#pragma unroll
            for (int v = 0; v < VPT; ++v) lt += keys[v] < tau ? 1 : 0;
            int c_lt = 0;
            const int off = block_excl_scan<SNW>(lt, sm.ints, &c_lt);
            if (ri >= c_lt) {
                ki = kj = tau;
                done = true;
            } else if (c_lt <= CAND_CAP) {
                int o = off;
                __syncthreads();
#pragma unroll
                for (int v = 0; v < VPT; ++v)
                    if (keys[v] < tau) sm.buf[o++] = keys[v];
                __syncthreads();
                for (int i = threadIdx.x; i < c_lt; i += ST) {
                    const uint64_t v = sm.buf[i];
                    const int r = lds_rank(sm.buf, c_lt, v, i);
                    if (r == ri) sm.bc[1] = v;
                    if (r == rj) sm.bc[2] = v;
                }
                __syncthreads();
                ki = sm.bc[1];
                kj = rj < c_lt ? sm.bc[2] : tau;
                __syncthreads();
                done = true;
            }
        }
    }
    if (!done) {
        ki = radix_rank<VPT>(keys, ri, sm);
        if (rj == ri) {
            kj = ki;
        } else {
            int le = 0;
            uint64_t nxt = SENT;
#pragma unroll
            for (int v = 0; v < VPT; ++v) {
                le += keys[v] <= ki ? 1 : 0;
                if (keys[v] > ki && keys[v] < nxt) nxt = keys[v];
            }
            le = block_sum<SNW>(le, sm.ints);
            nxt = block_min_u64<SNW>(nxt, sm.u64s);
            kj = le >= rj + 1 ? ki : nxt;
        }
    }
}

// Keys at ranks ri <= rj, choosing the lower-tail, upper-tail (complemented keys) or
// radix path.  `keys` is restored on return.
template <int VPT>
__device__ __forceinline__ void select_ranks(uint64_t (&keys)[VPT], int n, int ri, int rj, uint64_t& ki,
                             uint64_t& kj, SelSmem& sm) {
    if (rj < ST || (n - 1 - ri) >= ST) {
        select_low<VPT>(keys, ri, rj, ki, kj, sm);
        return;
    }
#pragma unroll
    for (int v = 0; v < VPT; ++v) keys[v] = keys[v] == SENT ? SENT : ~keys[v];
    uint64_t a, b;
    select_low<VPT>(keys, n - 1 - rj, n - 1 - ri, a, b, sm);
    kj = ~a;
    ki = ~b;
#pragma unroll
    for (int v = 0; v < VPT; ++v) keys[v] = keys[v] == SENT ? SENT : ~keys[v];
}

// Bitonic sort (ascending) of the 64*R keys held by one wave: element e = lane + 64*r lives
// in register r of lane e&63.  Cross-lane stages exchange through ds_bpermute; the j=64
// stage of R=2 is register-local.
template <int R>
__device__ __forceinline__ void wave_sort(uint64_t (&v)[R]) {
    const int lane = lane_id();
#pragma unroll
    for (int k = 2; k <= WAVE * R; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
            if (j >= WAVE) {
                const int rj = j / WAVE;
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    if (r & rj) continue;
                    const bool up = (((lane + WAVE * r) & k) == 0);
                    const uint64_t a = v[r], b = v[r | rj];
                    const uint64_t mn = a < b ? a : b, mx = a < b ? b : a;
                    v[r] = up ? mn : mx;
                    v[r | rj] = up ? mx : mn;
                }
            } else {
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const uint64_t p = (uint64_t)__shfl_xor((long long)v[r], j, WAVE);
                    const bool up = (((lane + WAVE * r) & k) == 0);
                    const bool lower = (lane & j) == 0;
                    const bool take_min = lower == up;
                    const uint64_t mn = p < v[r] ? p : v[r], mx = p < v[r] ? v[r] : p;
                    v[r] = take_min ? mn : mx;
                }
            }
        }
    }
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

// Both winsorize tails at once: keys at ranks li <= lj (lower tail) and hi_i <= hi_j (upper
// tail), n valid keys.  Returns false (nothing written, block-uniform) when the fast path
// does not apply; the caller then uses select_ranks.
//   tau_lo = max over the 4 waves of the wave's k-th smallest thread minimum,
//   k = ceil((lj+1)/4): 4k >= lj+1 distinct keys are <= tau_lo, so s[lj] <= tau_lo, and
//   only the keys < tau_lo (about lj of them) can precede it.  Same for the upper tail on
//   complemented keys.  Candidates are compacted with one packed scan and sorted by one
//   wave per tail.
template <int VPT>
__device__ __forceinline__ bool select_tails(const uint64_t (&keys)[VPT], int n, int li, int lj,
                                             int hi_i, int hi_j, uint64_t& k0, uint64_t& k1,
                                             uint64_t& k2, uint64_t& k3, SelSmem& sm) {
    const int ci = n - 1 - hi_j, cj = n - 1 - hi_i;   // upper-tail ranks in complemented order
    if (lj >= ST - 3 || cj >= ST - 3) return false;
    uint64_t mn = SENT, cmn = SENT;
#pragma unroll
    for (int v = 0; v < VPT; ++v) {
        const uint64_t k = keys[v];
        const uint64_t ck = k == SENT ? SENT : ~k;
        mn = k < mn ? k : mn;
        cmn = ck < cmn ? ck : cmn;
    }
    uint64_t a[1] = {mn}, b[1] = {cmn};
    wave_sort<1>(a);
    wave_sort<1>(b);
    const int w = threadIdx.x / WAVE, lane = lane_id();
    const int klo = (lj + 4) / 4, khi = (cj + 4) / 4;
    __syncthreads();   // sm.bc / sm.buf may still be read by a previous phase
    if (lane == klo - 1) sm.buf[CAND_CAP - 8 + w] = a[0];
    if (lane == khi - 1) sm.buf[CAND_CAP - 4 + w] = b[0];
    __syncthreads();
    uint64_t tlo = 0, thi = 0;
#pragma unroll
    for (int i = 0; i < SNW; ++i) {
        const uint64_t x = sm.buf[CAND_CAP - 8 + i], y = sm.buf[CAND_CAP - 4 + i];
        tlo = x > tlo ? x : tlo;
        thi = y > thi ? y : thi;
    }
    if (tlo == SENT || thi == SENT) return false;   // some wave lacks k valid thread minima
    int cnt = 0;
#pragma unroll
    for (int v = 0; v < VPT; ++v) {
        const uint64_t k = keys[v];
        const uint64_t ck = k == SENT ? SENT : ~k;
        cnt += (k < tlo ? 1 : 0) + (ck < thi ? 0x10000 : 0);
    }
    int tot = 0;
    const int off = block_excl_scan<SNW>(cnt, sm.ints, &tot);
    const int clo = tot & 0xFFFF, chi = tot >> 16;
    constexpr int HALF = CAND_CAP / 2;
    if (clo > 2 * WAVE || chi > 2 * WAVE) return false;   // block-uniform
    {
        int ol = off & 0xFFFF, oh = HALF + (off >> 16);
        __syncthreads();
#pragma unroll
        for (int v = 0; v < VPT; ++v) {
            const uint64_t k = keys[v];
            const uint64_t ck = k == SENT ? SENT : ~k;
            if (k < tlo) sm.buf[ol++] = k;
            if (ck < thi) sm.buf[oh++] = ck;
        }
        __syncthreads();
    }
    if (w == 0) {
        if (clo <= WAVE) wave_sort_lds<1>(sm.buf, clo);
        else wave_sort_lds<2>(sm.buf, clo);
    } else if (w == 1) {
        if (chi <= WAVE) wave_sort_lds<1>(sm.buf + HALF, chi);
        else wave_sort_lds<2>(sm.buf + HALF, chi);
    }
    __syncthreads();
    k0 = li < clo ? sm.buf[li] : tlo;
    k1 = lj < clo ? sm.buf[lj] : tlo;
    const uint64_t ca = ci < chi ? sm.buf[HALF + ci] : thi;
    const uint64_t cb = cj < chi ? sm.buf[HALF + cj] : thi;
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

template <int VPT>
__global__ __launch_bounds__(ST) void select_kernel(SelArgs a) {
    __shared__ SelSmem sm;
    const int s = blockIdx.x;
    const int c = blockIdx.y;
    const int64_t r0 = a.seg_off[s];
    const int L = (int)(a.seg_off[s + 1] - r0);
    const double* src = a.cols + (int64_t)c * a.col_stride + r0;
    uint64_t keys[VPT];
    int cnt = 0;
    // Unconditional loads (index clamped, masked after): a load under a runtime condition
    // makes hipcc wait vmcnt(0) per load and serializes the HBM round trips.
    const int last = L > 0 ? L - 1 : 0;
    double xv[VPT];
#pragma unroll
    for (int v = 0; v < VPT; ++v) {
        const int idx = threadIdx.x + v * ST;
        xv[v] = L > 0 ? src[idx < L ? idx : last] : NAN;
    }
    uint8_t mk[VPT];
    if (a.mask != nullptr) {
#pragma unroll
        for (int v = 0; v < VPT; ++v) {
            const int idx = threadIdx.x + v * ST;
            mk[v] = L > 0 ? a.mask[r0 + (idx < L ? idx : last)] : 0;
        }
    }
#pragma unroll
    for (int v = 0; v < VPT; ++v) {
        const int idx = threadIdx.x + v * ST;
        const bool on = idx < L && (a.mask == nullptr || mk[v] != 0) && !isnan(xv[v]);
        const uint64_t k = on ? dkey(xv[v]) : SENT;
        keys[v] = k;
        cnt += on ? 1 : 0;
    }
    const int n = block_sum<SNW>(cnt, sm.ints);
    double lo = NAN, hi = NAN;
    const bool apply = n >= a.min_count && n > 0;
    if (apply) {
        int i0, j0, i1, j1;
        double g0, g1;
        qranks(n, a.q_lo, a.lerp_mode, i0, j0, g0);
        qranks(n, a.q_hi, a.lerp_mode, i1, j1, g1);
        uint64_t k0, k1, k2, k3;
        if (!select_tails<VPT>(keys, n, i0, j0, i1, j1, k0, k1, k2, k3, sm)) {
            select_ranks<VPT>(keys, n, i0, j0, k0, k1, sm);
            select_ranks<VPT>(keys, n, i1, j1, k2, k3, sm);
        }
        lo = qlerp(kval(k0), kval(k1), g0, a.lerp_mode);
        hi = qlerp(kval(k2), kval(k3), g1, a.lerp_mode);
    }
    if (a.mean != nullptr) {
        // moments of the clipped values (pandas clip ignores NaN bounds)
        double sum = 0.0;
#pragma unroll
        for (int v = 0; v < VPT; ++v) {
            if (keys[v] == SENT) continue;
            double x = kval(keys[v]);
            if (apply) {
                if (x < lo) x = lo;
                if (x > hi) x = hi;
            }
            sum += x;
        }
        sum = block_sum<SNW>(sum, sm.dbl);
        const double mu = n > 0 ? sum / (double)n : NAN;
        double ss = 0.0;
#pragma unroll
        for (int v = 0; v < VPT; ++v) {
            if (keys[v] == SENT) continue;
            double x = kval(keys[v]);
            if (apply) {
                if (x < lo) x = lo;
                if (x > hi) x = hi;
            }
            const double d = x - mu;
            ss += d * d;
        }
        ss = block_sum<SNW>(ss, sm.dbl);
        if (threadIdx.x == 0) {
            a.mean[(int64_t)c * a.nseg + s] = mu;
            if (a.sd) a.sd[(int64_t)c * a.nseg + s] = n > 1 ? sqrt(ss / (double)(n - 1)) : NAN;
        }
    }
    if (threadIdx.x == 0) {
        const int64_t o = (int64_t)c * a.nseg + s;
        a.lo[o] = lo;
        a.hi[o] = hi;
        if (a.nvalid) a.nvalid[o] = n;
    }
}

template <int VPT>
void launch_select(const SelArgs& a, int ncols, hipStream_t st) {
    dim3 grid(a.nseg, ncols);
    hipLaunchKernelGGL(select_kernel<VPT>, grid, dim3(ST), 0, st, a);
}

}  // namespace
}  // namespace fm

extern "C" int fm_select_cuts(const double* cols, int64_t col_stride, int32_t ncols,
                              const int64_t* seg_off, int32_t nseg, int32_t max_seg_len,
                              const uint8_t* row_mask, double q_lo, double q_hi,
                              int32_t min_count, int32_t lerp_mode, double* lo, double* hi,
                              int32_t* nvalid, double* mean, double* sd, void* stream) {
    using namespace fm;
    FM_REQUIRE(cols && seg_off && lo && hi, "fm_select_cuts: null pointer");
    FM_REQUIRE(ncols > 0 && ncols <= 65535 && nseg >= 0, "fm_select_cuts: bad sizes");
    FM_REQUIRE(lerp_mode == 0 || lerp_mode == 1, "fm_select_cuts: lerp_mode must be 0 or 1");
    FM_REQUIRE(q_lo >= 0.0 && q_lo <= 1.0 && q_hi >= 0.0 && q_hi <= 1.0,
               "fm_select_cuts: quantiles must be in [0,1]");
    if (nseg == 0) return FM_OK;
    SelArgs a{cols, col_stride, seg_off, nseg, row_mask, q_lo, q_hi, min_count, lerp_mode,
              lo, hi, nvalid, mean, sd};
    hipStream_t st = (hipStream_t)stream;
    const int vpt = (max_seg_len + ST - 1) / ST;
    if (vpt <= 2) launch_select<2>(a, ncols, st);
    else if (vpt <= 4) launch_select<4>(a, ncols, st);
    else if (vpt <= 8) launch_select<8>(a, ncols, st);
    else if (vpt <= 16) launch_select<16>(a, ncols, st);
    else if (vpt <= 24) launch_select<24>(a, ncols, st);
    else if (vpt <= 32) launch_select<32>(a, ncols, st);
    else if (vpt <= 48) launch_select<48>(a, ncols, st);
    else if (vpt <= 64) launch_select<64>(a, ncols, st);
    else if (vpt <= 96) launch_select<96>(a, ncols, st);
    else {
        set_error("fm_select_cuts: segment of %d rows exceeds the %d-row register budget",
                  max_seg_len, 96 * ST);
        return FM_ETOOBIG;
    }
    FM_CHECK_LAUNCH("fm_select_cuts");
    return FM_OK;
}

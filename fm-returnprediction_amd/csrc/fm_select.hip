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
    double dbl[2 * SNW];
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
template <int VPT>
__device__ __forceinline__ bool select_tails(const double (&xv)[VPT], double mn, double mx, int n,
                                             int li, int lj, int hi_i, int hi_j, uint64_t& k0,
                                             uint64_t& k1, uint64_t& k2, uint64_t& k3, SelSmem& sm) {
    const int ci = n - 1 - hi_j, cj = n - 1 - hi_i;   // upper-tail ranks in complemented order
    if (lj >= ST || cj >= ST) return false;
    uint64_t a[1] = {isnan(mn) ? SENT : dkey(mn)};
    uint64_t b[1] = {isnan(mx) ? SENT : ~dkey(mx)};
    wave_sort<1>(a);
    wave_sort<1>(b);
    const int w = threadIdx.x / WAVE, lane = lane_id();
    uint64_t* Llo = sm.buf + CAND_CAP - 8 * WAVE;       // [4][64] sorted thread minima
    uint64_t* Lhi = sm.buf + CAND_CAP - 4 * WAVE;       // [4][64] sorted complemented maxima
    __syncthreads();   // sm.buf may still be read by a previous phase
    Llo[w * WAVE + lane] = a[0];
    Lhi[w * WAVE + lane] = b[0];
    if (threadIdx.x < 2) sm.bc[threadIdx.x] = SENT;
    __syncthreads();
    // merged rank of this lane's entries (ranks >= lane, so only lanes <= lj / cj matter)
    if (lane <= lj && a[0] != SENT) {
        int r = lane;
#pragma unroll
        for (int u = 0; u < SNW; ++u)
            if (u != w) r += merge_count(Llo + u * WAVE, a[0], u < w);
        if (r == lj) sm.bc[0] = a[0];
    }
    if (lane <= cj && b[0] != SENT) {
        int r = lane;
#pragma unroll
        for (int u = 0; u < SNW; ++u)
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
    const int off = block_excl_scan<SNW>(cnt, sm.ints, &tot);
    const int clo = tot & 0xFFFF, chi = tot >> 16;
    constexpr int HALF = CAND_CAP / 4;
    if (clo > 4 * WAVE || chi > 4 * WAVE) return false;   // block-uniform
    {
        int ol = off & 0xFFFF, oh = HALF + (off >> 16);
#pragma unroll
        for (int v = 0; v < VPT; ++v) {
            if (xv[v] < tlo) sm.buf[ol++] = dkey(xv[v]);
            if (xv[v] > thi) sm.buf[oh++] = ~dkey(xv[v]);
        }
        __syncthreads();
    }
    if (w == 0) {
        if (clo <= WAVE) wave_sort_lds<1>(sm.buf, clo);
        else if (clo <= 2 * WAVE) wave_sort_lds<2>(sm.buf, clo);
        else wave_sort_lds<4>(sm.buf, clo);
    } else if (w == 1) {
        if (chi <= WAVE) wave_sort_lds<1>(sm.buf + HALF, chi);
        else if (chi <= 2 * WAVE) wave_sort_lds<2>(sm.buf + HALF, chi);
        else wave_sort_lds<4>(sm.buf + HALF, chi);
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

template <int VPT>
__global__ __launch_bounds__(ST) void select_kernel(SelArgs a) {
    __shared__ SelSmem sm;
    const int s = blockIdx.x;
    const int c = blockIdx.y;
    const int64_t r0 = a.seg_off[s];
    const int L = (int)(a.seg_off[s + 1] - r0);
    const double* src = a.cols + (int64_t)c * a.col_stride + r0;
    // Unconditional loads (index clamped, masked after): a load under a runtime condition
    // makes hipcc wait vmcnt(0) per load and serializes the HBM round trips.
    const int last = L > 0 ? L - 1 : 0;
    const uint8_t* mbase = a.mask ? a.mask + r0 : (const uint8_t*)src;
    const int mand = a.mask ? 0xFF : 0, mor = a.mask ? 0 : 1;
    double xv[VPT];
#pragma unroll
    for (int v = 0; v < VPT; ++v) {
        const int idx = threadIdx.x + v * ST;
        const int ci = idx < L ? idx : last;
        const double x = src[ci];
        const int m = (mbase[ci] & mand) | mor;
        xv[v] = (idx < L && m != 0) ? x : NAN;
    }
    // thread count / min / max (fmin/fmax ignore NaN)
    int cnt = 0;
    double mn = NAN, mx = NAN;
#pragma unroll
    for (int v = 0; v < VPT; ++v) {
        cnt += isnan(xv[v]) ? 0 : 1;
        mn = fmin(mn, xv[v]);
        mx = fmax(mx, xv[v]);
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
        if (!select_tails<VPT>(xv, mn, mx, n, i0, j0, i1, j1, k0, k1, k2, k3, sm)) {
            radix_pair<VPT>(xv, i0, j0, k0, k1, sm);
            radix_pair<VPT>(xv, i1, j1, k2, k3, sm);
        }
        lo = qlerp(kval(k0), kval(k1), g0, a.lerp_mode);
        hi = qlerp(kval(k2), kval(k3), g1, a.lerp_mode);
    }
    if (a.mean != nullptr) {
        // Moments of the clipped values (pandas clip ignores NaN bounds).  One pass about a
        // pivot p inside the data (a finite cut, else the smallest finite value):
        // mean = p + S1/n, var = (S2 - S1^2/n)/(n-1).
        double p = isfinite(lo) ? lo : (isfinite(hi) ? hi : 0.0);
        if (!isfinite(lo) && !isfinite(hi)) {
            // no cuts (short month): pivot = the smallest finite value
            double m2 = isfinite(mn) ? mn : NAN;
            p = block_min_f64<SNW>(m2, sm.dbl);
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
        double2 r = block_sum2<SNW>(s1, s2, sm.dbl);
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
    else if (vpt <= 20) launch_select<20>(a, ncols, st);
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

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

#include "fm_select_dev.h"

namespace fm {
namespace {

template <int VPT, bool FB>
__global__ __launch_bounds__(ST) void select_kernel(SelArgs a) {
    __shared__ SelSmem sm;
    if (!FB) {
        select_unit_wg<VPT>(a, blockIdx.x, blockIdx.y, sm);
        return;
    }
    // Each workgroup scans a contiguous range of units with one coalesced load of the marks
    // per 256 units (a unit-by-unit scan would pay one memory round trip per unit), then
    // redoes the marked ones, lowest unit first (each thread clears its own mark).
    const int64_t nunits = (int64_t)a.nseg * a.ncols;
    const int64_t per = (nunits + gridDim.x - 1) / gridDim.x;
    const int64_t u0 = (int64_t)blockIdx.x * per, u1 = u0 + per < nunits ? u0 + per : nunits;
    for (int64_t b = u0; b < u1; b += ST) {
        const int64_t u = b + threadIdx.x;
        bool mark = u < u1 && a.nvalid[u] == -1;
        while (true) {
            const uint64_t pick = block_min_u64<SNW>(mark ? (uint64_t)u : SENT, sm.u64s);
            if (pick == SENT) break;   // block-uniform
            if ((uint64_t)u == pick) mark = false;
            __syncthreads();
            select_unit_wg<VPT>(a, (int)(pick % a.nseg), (int)(pick / a.nseg), sm);
            __syncthreads();
        }
    }
}

// Segments longer than the register budget (> 96 * 256 rows: a daily-frequency panel, a
// huge cross-section): one workgroup per (segment, column) STREAMS the segment from HBM for
// every pass instead of holding it in registers -- count / key range, the adaptive
// histogram (hist_select: one histogram pass per level, one compaction pass), then the
// moments if asked.  Exact order statistics, same lerps, same pivot as the register paths.
__global__ __launch_bounds__(ST) void select_stream_kernel(SelArgs a) {
    __shared__ SelSmem sm;
    const int s = blockIdx.x, c = blockIdx.y;
    const int64_t r0 = a.seg_off[s];
    const int64_t L = a.seg_off[s + 1] - r0;
    const double* src = a.cols + (int64_t)c * a.col_stride + r0;
    const uint8_t* msk = a.mask ? a.mask + r0 : nullptr;
    auto for_each = [&](auto&& f) {
        for (int64_t i = threadIdx.x; i < L; i += ST) {
            const double x = src[i];
            f((msk == nullptr || msk[i] != 0) ? x : NAN);
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
    }
}

template <int VPT>
void launch_select(const SelArgs& a, int ncols, hipStream_t st, bool fallback) {
    if (fallback)
        hipLaunchKernelGGL((select_kernel<VPT, true>), dim3(256), dim3(ST), 0, st, a);
    else
        hipLaunchKernelGGL((select_kernel<VPT, false>), dim3(a.nseg, ncols), dim3(ST), 0, st, a);
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
            if (lane == 0 && a.nvalid) a.nvalid[u] = -1;   // redone by the fallback pass
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
            }
        }
        if (!more) break;
        if (!early) Ln = load_unit<VPL>(a, un, xv);
        k = kn;
        u = un;
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

template <int VPL>
void launch_select_wave(const SelArgs& a, hipStream_t st) {
    const int64_t nunits = (int64_t)a.nseg * a.ncols;
    if (a.mean == nullptr)
        hipLaunchKernelGGL((select_wave_kernel<VPL, true>), dim3((unsigned)select_wave_grid(nunits)), dim3(ST), 0, st, a);
    else
        hipLaunchKernelGGL((select_wave_kernel<VPL, false>), dim3((unsigned)select_wave_grid(nunits)), dim3(ST), 0, st, a);
}

}  // namespace
}  // namespace fm

extern "C" int fm_select_cuts(const double* cols, int64_t col_stride, int32_t ncols,
                              const int64_t* seg_off, int32_t nseg, int32_t max_seg_len,
                              const uint8_t* row_mask, double q_lo, double q_hi,
                              int32_t min_count, int32_t lerp_mode, double* lo, double* hi,
                              int32_t* nvalid, double* mean, double* sd, void* stream) {
    const fm_select_args a{cols,    col_stride, ncols,    seg_off, nseg, max_seg_len, row_mask, q_lo,
                           q_hi,    min_count,  lerp_mode, lo,     hi,   nvalid,      mean,     sd,
                           nullptr};
    return fm_select(&a, stream);
}

extern "C" int fm_select(const fm_select_args* args, void* stream) {
    using namespace fm;
    FM_REQUIRE(args != nullptr, "fm_select: null args");
    const fm_select_args& x = *args;
    const double* cols = x.cols;
    const int64_t* seg_off = x.seg_off;
    const int32_t ncols = x.ncols, nseg = x.nseg, max_seg_len = x.max_seg_len;
    const uint8_t* row_mask = x.row_mask;
    const int32_t* nvalid = x.nvalid;
    FM_REQUIRE(cols && seg_off && x.lo && x.hi, "fm_select_cuts: null pointer");
    FM_REQUIRE(ncols > 0 && ncols <= 65535 && nseg >= 0, "fm_select_cuts: bad sizes");
    FM_REQUIRE(x.lerp_mode == 0 || x.lerp_mode == 1, "fm_select_cuts: lerp_mode must be 0 or 1");
    FM_REQUIRE(x.q_lo >= 0.0 && x.q_lo <= 1.0 && x.q_hi >= 0.0 && x.q_hi <= 1.0,
               "fm_select_cuts: quantiles must be in [0,1]");
    if (nseg == 0) return FM_OK;
    SelArgs a{cols,        x.col_stride, seg_off, nseg,     ncols, row_mask, x.q_lo, x.q_hi,
              x.min_count, x.lerp_mode,  x.lo,    x.hi,     x.nvalid, x.mean, x.sd,  x.center};
    hipStream_t st = (hipStream_t)stream;
    const int vpt = (max_seg_len + ST - 1) / ST;
    if (vpt > 96) {
        // longer than the register budget: stream every unit from HBM (exact, any length)
        hipLaunchKernelGGL(select_stream_kernel, dim3(nseg, ncols), dim3(ST), 0, st, a);
        FM_CHECK_LAUNCH("fm_select_cuts(stream)");
        return FM_OK;
    }
    // wave fast path: no row mask, segments of <= 96 * 64 rows, nvalid present (it carries
    // the fallback marks); the workgroup kernel then redoes the marked units only
    const int vpl = (max_seg_len + WAVE - 1) / WAVE;
    const bool wave = row_mask == nullptr && nvalid != nullptr && vpl <= 96;
    if (wave) {
        if (vpl <= 16) launch_select_wave<16>(a, st);
        else if (vpl <= 32) launch_select_wave<32>(a, st);
        else if (vpl <= 48) launch_select_wave<48>(a, st);
        else if (vpl <= 64) launch_select_wave<64>(a, st);
        else if (vpl <= 80) launch_select_wave<80>(a, st);
        else launch_select_wave<96>(a, st);
        FM_CHECK_LAUNCH("fm_select_cuts(wave)");
    }
#ifdef FM_SELECT_DIAG_NO_FALLBACK
    // diagnostic builds only (-DFM_SELECT_DIAG_NO_FALLBACK, tools/select_marks.py): leave the
    // wave kernel's fallback marks (nvalid == -1) in place; results are then incomplete.
    // The shipped library is never built with it.
    if (wave) return FM_OK;
#endif
    if (vpt <= 2) launch_select<2>(a, ncols, st, wave);
    else if (vpt <= 4) launch_select<4>(a, ncols, st, wave);
    else if (vpt <= 8) launch_select<8>(a, ncols, st, wave);
    else if (vpt <= 16) launch_select<16>(a, ncols, st, wave);
    else if (vpt <= 20) launch_select<20>(a, ncols, st, wave);
    else if (vpt <= 24) launch_select<24>(a, ncols, st, wave);
    else if (vpt <= 32) launch_select<32>(a, ncols, st, wave);
    else if (vpt <= 48) launch_select<48>(a, ncols, st, wave);
    else if (vpt <= 64) launch_select<64>(a, ncols, st, wave);
    else launch_select<96>(a, ncols, st, wave);
    FM_CHECK_LAUNCH("fm_select_cuts");
    return FM_OK;
}

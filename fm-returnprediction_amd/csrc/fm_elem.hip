// Streaming per-segment kernels: clip (winsorize write-back), standardize, universe
// levels, Gram pivots, synthetic panel generation, and a bandwidth probe.
#include <math.h>

#include "fm_common.h"

namespace fm {
namespace {

constexpr int ET = 256;

// One workgroup per (segment, column) tile of rows; blockIdx.z splits long segments.
__global__ __launch_bounds__(ET) void clip_kernel(const double* __restrict__ src,
                                                  double* __restrict__ dst, int64_t stride,
                                                  const int64_t* __restrict__ seg_off, int nseg,
                                                  const double* __restrict__ lo,
                                                  const double* __restrict__ hi) {
    const int s = blockIdx.x, c = blockIdx.y;
    const int64_t r0 = seg_off[s], r1 = seg_off[s + 1];
    const double l = lo[(int64_t)c * nseg + s], h = hi[(int64_t)c * nseg + s];
    const int64_t base = (int64_t)c * stride;
    for (int64_t r = r0 + blockIdx.z * ET + threadIdx.x; r < r1; r += (int64_t)gridDim.z * ET) {
        double x = src[base + r];
        // pandas clip: NaN values stay NaN, NaN bounds are ignored
        if (x < l) x = l;
        if (x > h) x = h;
        dst[base + r] = x;
    }
}

__global__ __launch_bounds__(ET) void standardize_kernel(const double* __restrict__ src,
                                                         double* __restrict__ dst, int64_t stride,
                                                         const int64_t* __restrict__ seg_off,
                                                         int nseg, const double* __restrict__ mean,
                                                         const double* __restrict__ sd) {
    const int s = blockIdx.x, c = blockIdx.y;
    const int64_t r0 = seg_off[s], r1 = seg_off[s + 1];
    const double mu = mean[(int64_t)c * nseg + s], sg = sd[(int64_t)c * nseg + s];
    const int64_t base = (int64_t)c * stride;
    for (int64_t r = r0 + blockIdx.z * ET + threadIdx.x; r < r1; r += (int64_t)gridDim.z * ET)
        dst[base + r] = (src[base + r] - mu) / sg;
}

__global__ __launch_bounds__(ET) void level_kernel(const double* __restrict__ me,
                                                   const int64_t* __restrict__ seg_off,
                                                   const double* __restrict__ ca,
                                                   const double* __restrict__ cb,
                                                   uint8_t* __restrict__ level) {
    const int s = blockIdx.x;
    const int64_t r0 = seg_off[s], r1 = seg_off[s + 1];
    const double a = ca[s], b = cb[s];
    for (int64_t r = r0 + blockIdx.z * ET + threadIdx.x; r < r1; r += (int64_t)gridDim.z * ET) {
        const double x = me[r];
        // src/calc_Lewellen_2014.py:95-96: NaN comparisons are False
        level[r] = (uint8_t)((x >= a ? 1 : 0) + (x >= b ? 1 : 0));
    }
}

// Pivot for the shifted Gram: mean of the first <= 256 finite values of the segment.
__global__ __launch_bounds__(WAVE) void pilot_kernel(const double* __restrict__ cols,
                                                     int64_t stride,
                                                     const int64_t* __restrict__ seg_off,
                                                     int nseg, double* __restrict__ shift) {
    const int s = blockIdx.x, c = blockIdx.y;
    const int64_t r0 = seg_off[s], r1 = seg_off[s + 1];
    const int64_t n = r1 - r0 < 256 ? r1 - r0 : 256;
    double sum = 0.0;
    int cnt = 0;
    for (int64_t i = threadIdx.x; i < n; i += WAVE) {
        const double x = cols[(int64_t)c * stride + r0 + i];
        if (isfinite(x)) {
            sum += x;
            ++cnt;
        }
    }
    sum = wave_sum(sum);
    cnt = wave_sum(cnt);
    if (threadIdx.x == 0) shift[(int64_t)c * nseg + s] = cnt > 0 ? sum / (double)cnt : 0.0;
}

// ---- synthetic panel: must match fmcore/synth.py operation for operation -----------------
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z ^= z >> 30;
    z *= 0xBF58476D1CE4E5B9ull;
    z ^= z >> 27;
    z *= 0x94D049BB133111EBull;
    z ^= z >> 31;
    return z;
}
__device__ __forceinline__ uint64_t cell_hash(uint64_t seed, uint64_t m, uint64_t f, uint64_t col) {
    uint64_t h = mix64(seed ^ (col << 40));
    h = mix64(h + m * 0x9E3779B97F4A7C15ull);
    h = mix64(h + f * 0xD1B54A32D192ED03ull);
    return h;
}
__device__ __forceinline__ double hash_u(uint64_t h) {
    return ((double)(h >> 11) + 0.5) * 0x1p-53;
}
__device__ __forceinline__ double t2(double u) {
    const double num = 2.0 * u - 1.0;
    const double den = sqrt((2.0 * u) * (1.0 - u));
    return num / den;
}

struct GenConst {
    double mu[15], sd[15], load[14];
};
__constant__ GenConst g_gen = {
    // WINSOR_VARS order: retx, log_size, log_bm, return_12_2, log_issues_12, accruals_final,
    // roa, log_assets_growth, dy, log_return_13_36, log_issues_36, beta, rolling_std_252,
    // debt_price, sales_price  (Table-1 Avg/Std, reference src/test_calc_Lewellen_2014.py:51-65)
    {0.0127, 4.63, -0.51, 0.13, 0.04, -0.02, 0.01, 0.12, 0.02, 0.24, 0.11, 0.96, 0.15, 0.83, 2.53},
    {0.1479, 1.93, 0.84, 0.48, 0.12, 0.10, 0.14, 0.26, 0.02, 0.58, 0.25, 0.55, 0.08, 1.59, 3.56},
    {-0.0030, 0.0035, 0.0040, -0.0010, -0.0025, 0.0020, -0.0015, 0.0005, 0.0010, -0.0020, 0.0003,
     -0.0005, 0.0004, 0.0012}};

__global__ __launch_bounds__(ET) void gen_kernel(uint64_t seed, int64_t month0, int nmonths,
                                                 int nfirms, uint64_t nan_thr, uint64_t me_nan_thr,
                                                 uint64_t nyse_thr, uint64_t dy_thr,
                                                 double* __restrict__ cols, int64_t stride,
                                                 double* __restrict__ me,
                                                 uint8_t* __restrict__ nyse,
                                                 uint32_t* __restrict__ hip_, uint32_t* __restrict__ lop,
                                                 int64_t pstride) {
    const int64_t cell = (int64_t)blockIdx.x * ET + threadIdx.x;
    const int64_t ncell = (int64_t)nmonths * nfirms;
    if (cell >= ncell) return;
    const uint64_t m = (uint64_t)(month0 + cell / nfirms);
    const uint64_t f = (uint64_t)(cell % nfirms);
    double x[15];
    double zsum = 0.0;
#pragma unroll
    for (int j = 0; j < 14; ++j) {
        const double mu = g_gen.mu[1 + j], sd = g_gen.sd[1 + j];
        double v = mu + sd * (t2(hash_u(cell_hash(seed, m, f, 1 + j))) * 0.5);
        if (j == 7 && cell_hash(seed, m, f, 68) < dy_thr) v = 0.0;  // dy: 30% exact zeros
        x[1 + j] = v;
        const double z = (v - mu) / sd;
        const double term = g_gen.load[j] * z;
        zsum = j == 0 ? term : zsum + term;
    }
    x[0] = (g_gen.mu[0] + zsum) + g_gen.sd[0] * (t2(hash_u(cell_hash(seed, m, f, 0))) * 0.5);
#pragma unroll
    for (int k = 0; k < 15; ++k) {
        double v = x[k];
        if (nan_thr != 0 && cell_hash(seed, m, f, 32 + k) < nan_thr) v = NAN;
        if (cols != nullptr) cols[(int64_t)k * stride + cell] = v;
        if (hip_ != nullptr) {   // the split layout, written here instead of by a later pass
            const uint64_t u = (uint64_t)__double_as_longlong(v);
            hip_[(int64_t)k * pstride + cell] = (uint32_t)(u >> 32);
            lop[(int64_t)k * pstride + cell] = (uint32_t)u;
        }
    }
    double mev = 10.0 / hash_u(cell_hash(seed, m, f, 64));
    if (me_nan_thr != 0 && cell_hash(seed, m, f, 65) < me_nan_thr) mev = NAN;
    me[cell] = mev;
    nyse[cell] = cell_hash(seed, m, f, 66) < nyse_thr ? 1 : 0;
}

// The achievable HBM READ rate (bench.py's measured_read_peak for the read-dominated Gram):
// 16-byte loads, PU of them in flight per thread, grid-stride over the buffer; the sum keeps
// the loads.  n must be a multiple of 2 (double2 pairs) for the full rate; an odd tail is
// read by thread 0.
constexpr int PU = 4;
__global__ __launch_bounds__(ET) void probe_kernel(const double* __restrict__ src, int64_t n,
                                                   double* __restrict__ out) {
    __shared__ double red[ET / WAVE];
    const double2* s2 = reinterpret_cast<const double2*>(src);
    const int64_t np = n / 2;
    const int64_t stride = (int64_t)gridDim.x * ET;
    double s = 0.0;
    int64_t i = (int64_t)blockIdx.x * ET + threadIdx.x;
    for (; i + (PU - 1) * stride < np; i += PU * stride) {
        double2 v[PU];
#pragma unroll
        for (int u = 0; u < PU; ++u) v[u] = s2[i + u * stride];
#pragma unroll
        for (int u = 0; u < PU; ++u) s += v[u].x + v[u].y;
    }
    for (; i < np; i += stride) s += s2[i].x + s2[i].y;
    if (blockIdx.x == 0 && threadIdx.x == 0 && (n & 1)) s += src[n - 1];
    s = block_sum<ET / WAVE>(s, red);
    if (threadIdx.x == 0) atomicAdd(out, s);
}

// The achievable HBM COPY rate (read + write bytes): the same grid-stride 16-byte stream,
// each pair stored to dst (bench.py's measured_copy_peak).  An odd tail by thread 0.
__global__ __launch_bounds__(ET) void copy_probe_kernel(const double* __restrict__ src, double* __restrict__ dst,
                                                        int64_t n) {
    const double2* s2 = reinterpret_cast<const double2*>(src);
    double2* d2 = reinterpret_cast<double2*>(dst);
    const int64_t np = n / 2;
    const int64_t stride = (int64_t)gridDim.x * ET;
    int64_t i = (int64_t)blockIdx.x * ET + threadIdx.x;
    for (; i + (PU - 1) * stride < np; i += PU * stride) {
        double2 v[PU];
#pragma unroll
        for (int u = 0; u < PU; ++u) v[u] = s2[i + u * stride];
#pragma unroll
        for (int u = 0; u < PU; ++u) d2[i + u * stride] = v[u];
    }
    for (; i < np; i += stride) d2[i] = s2[i];
    if (blockIdx.x == 0 && threadIdx.x == 0 && (n & 1)) dst[n - 1] = src[n - 1];
}

// The FP64 panel as two 32-bit planes (high words, low words): the selects order values by
// their high words alone (half the bytes), and the Gram re-reads the high plane right after
// them, from the memory-side cache.  16-byte loads (two rows), 8-byte stores per plane.
__global__ __launch_bounds__(ET) void split_planes_kernel(const double* __restrict__ cols, int64_t stride,
                                                          int ncols, int64_t nrows, uint32_t* __restrict__ hi,
                                                          uint32_t* __restrict__ lo, int64_t pstride) {
    const int64_t npair = (nrows + 1) / 2;
    const int64_t total = npair * ncols;
    for (int64_t i = (int64_t)blockIdx.x * ET + threadIdx.x; i < total; i += (int64_t)gridDim.x * ET) {
        const int64_t c = i / npair, p = i - c * npair, r = 2 * p;
        const double* src = cols + c * stride + r;
        uint32_t* h = hi + c * pstride + r;
        uint32_t* l = lo + c * pstride + r;
        if (r + 1 < nrows && (((uintptr_t)src | (uintptr_t)h | (uintptr_t)l) & 7) == 0 && (((uintptr_t)src) & 15) == 0) {
            const double2 v = *(const double2*)src;
            const uint64_t a = (uint64_t)__double_as_longlong(v.x), b = (uint64_t)__double_as_longlong(v.y);
            *(uint2*)h = make_uint2((uint32_t)(a >> 32), (uint32_t)(b >> 32));
            *(uint2*)l = make_uint2((uint32_t)a, (uint32_t)b);
        } else {
            for (int64_t k = r; k < r + 2 && k < nrows; ++k) {
                const uint64_t a = (uint64_t)__double_as_longlong(cols[c * stride + k]);
                hi[c * pstride + k] = (uint32_t)(a >> 32);
                lo[c * pstride + k] = (uint32_t)a;
            }
        }
    }
}

int zsplit(int64_t max_len) {
    // split long segments so every launch has >= ~2k workgroups in flight on 256 CUs
    int64_t z = (max_len + 4 * ET - 1) / (4 * ET);
    return (int)(z < 1 ? 1 : (z > 64 ? 64 : z));
}

}  // namespace
}  // namespace fm

extern "C" int fm_clip(const double* src, double* dst, int64_t col_stride, int32_t ncols,
                       const int64_t* seg_off, int32_t nseg, int64_t nrows, const double* lo,
                       const double* hi, void* stream) {
    using namespace fm;
    FM_REQUIRE(src && dst && seg_off && lo && hi, "fm_clip: null pointer");
    FM_REQUIRE(ncols > 0 && ncols <= 65535, "fm_clip: bad ncols");
    if (nseg == 0) return FM_OK;
    dim3 grid(nseg, ncols, zsplit(nrows / nseg + 1));
    hipLaunchKernelGGL(clip_kernel, grid, dim3(ET), 0, (hipStream_t)stream, src, dst, col_stride,
                       seg_off, nseg, lo, hi);
    FM_CHECK_LAUNCH("fm_clip");
    return FM_OK;
}

extern "C" int fm_standardize(const double* src, double* dst, int64_t col_stride, int32_t ncols,
                              const int64_t* seg_off, int32_t nseg, int64_t nrows,
                              const double* mean, const double* sd, void* stream) {
    using namespace fm;
    FM_REQUIRE(src && dst && seg_off && mean && sd, "fm_standardize: null pointer");
    FM_REQUIRE(ncols > 0 && ncols <= 65535, "fm_standardize: bad ncols");
    if (nseg == 0) return FM_OK;
    dim3 grid(nseg, ncols, zsplit(nrows / (nseg ? nseg : 1) + 1));
    hipLaunchKernelGGL(standardize_kernel, grid, dim3(ET), 0, (hipStream_t)stream, src, dst,
                       col_stride, seg_off, nseg, mean, sd);
    FM_CHECK_LAUNCH("fm_standardize");
    return FM_OK;
}

extern "C" int fm_universe_level(const double* me, const int64_t* seg_off, int32_t nseg,
                                 int64_t nrows, const double* cut_a, const double* cut_b,
                                 uint8_t* level, void* stream) {
    using namespace fm;
    FM_REQUIRE(me && seg_off && cut_a && cut_b && level, "fm_universe_level: null pointer");
    if (nseg == 0) return FM_OK;
    dim3 grid(nseg, 1, zsplit(nrows / (nseg ? nseg : 1) + 1));
    hipLaunchKernelGGL(level_kernel, grid, dim3(ET), 0, (hipStream_t)stream, me, seg_off, cut_a,
                       cut_b, level);
    FM_CHECK_LAUNCH("fm_universe_level");
    return FM_OK;
}

extern "C" int fm_pilot_shift(const double* cols, int64_t col_stride, int32_t ncols,
                              const int64_t* seg_off, int32_t nseg, double* shift, void* stream) {
    using namespace fm;
    FM_REQUIRE(cols && seg_off && shift, "fm_pilot_shift: null pointer");
    FM_REQUIRE(ncols > 0 && ncols <= 65535, "fm_pilot_shift: bad ncols");
    if (nseg == 0) return FM_OK;
    hipLaunchKernelGGL(pilot_kernel, dim3(nseg, ncols), dim3(WAVE), 0, (hipStream_t)stream, cols,
                       col_stride, seg_off, nseg, shift);
    FM_CHECK_LAUNCH("fm_pilot_shift");
    return FM_OK;
}

static uint64_t rate_thr(double r) {
    if (r <= 0.0) return 0;
    return (uint64_t)(r * 18446744073709551616.0);
}

extern "C" int fm_gen_panel_planes(uint64_t seed, int64_t month0, int32_t nmonths, int32_t nfirms,
                                   double nan_rate, double nyse_rate, double* cols, int64_t col_stride,
                                   uint32_t* hi, uint32_t* lo, int64_t plane_stride, double* me, uint8_t* nyse,
                                   void* stream) {
    using namespace fm;
    FM_REQUIRE((cols || hi) && me && nyse && (hi == nullptr) == (lo == nullptr), "fm_gen_panel: null pointer");
    FM_REQUIRE(nmonths >= 0 && nfirms > 0, "fm_gen_panel: bad sizes");
    FM_REQUIRE(nan_rate >= 0.0 && nan_rate < 1.0 && nyse_rate > 0.0 && nyse_rate < 1.0,
               "fm_gen_panel: rates must be in [0,1)");
    const int64_t ncell = (int64_t)nmonths * nfirms;
    FM_REQUIRE(cols == nullptr || col_stride >= ncell, "fm_gen_panel: col_stride < nmonths*nfirms");
    FM_REQUIRE(hi == nullptr || plane_stride >= ncell, "fm_gen_panel: plane_stride < nmonths*nfirms");
    if (ncell == 0) return FM_OK;
    const int64_t nblk = (ncell + ET - 1) / ET;
    hipLaunchKernelGGL(gen_kernel, dim3((unsigned)nblk), dim3(ET), 0, (hipStream_t)stream, seed,
                       month0, nmonths, nfirms, rate_thr(nan_rate), rate_thr(0.25 * nan_rate),
                       rate_thr(nyse_rate), rate_thr(0.3), cols, col_stride, me, nyse, hi, lo, plane_stride);
    FM_CHECK_LAUNCH("fm_gen_panel");
    return FM_OK;
}

extern "C" int fm_gen_panel(uint64_t seed, int64_t month0, int32_t nmonths, int32_t nfirms,
                            double nan_rate, double nyse_rate, double* cols, int64_t col_stride,
                            double* me, uint8_t* nyse, void* stream) {
    using namespace fm;
    FM_REQUIRE(cols && me && nyse, "fm_gen_panel: null pointer");
    FM_REQUIRE(nmonths >= 0 && nfirms > 0, "fm_gen_panel: bad sizes");
    FM_REQUIRE(nan_rate >= 0.0 && nan_rate < 1.0 && nyse_rate > 0.0 && nyse_rate < 1.0,
               "fm_gen_panel: rates must be in [0,1)");
    const int64_t ncell = (int64_t)nmonths * nfirms;
    FM_REQUIRE(col_stride >= ncell, "fm_gen_panel: col_stride < nmonths*nfirms");
    if (ncell == 0) return FM_OK;
    const int64_t nblk = (ncell + ET - 1) / ET;
    hipLaunchKernelGGL(gen_kernel, dim3((unsigned)nblk), dim3(ET), 0, (hipStream_t)stream, seed,
                       month0, nmonths, nfirms, rate_thr(nan_rate), rate_thr(0.25 * nan_rate),
                       rate_thr(nyse_rate), rate_thr(0.3), cols, col_stride, me, nyse, nullptr, nullptr, 0);
    FM_CHECK_LAUNCH("fm_gen_panel");
    return FM_OK;
}

extern "C" int fm_split_planes(const double* cols, int64_t col_stride, int32_t ncols, int64_t nrows,
                               uint32_t* hi, uint32_t* lo, int64_t plane_stride, void* stream) {
    using namespace fm;
    FM_REQUIRE(cols && hi && lo, "fm_split_planes: null pointer");
    FM_REQUIRE(ncols >= 0 && nrows >= 0 && col_stride >= nrows && plane_stride >= nrows,
               "fm_split_planes: bad sizes");
    if (ncols == 0 || nrows == 0) return FM_OK;
    hipLaunchKernelGGL(split_planes_kernel, dim3(4096), dim3(ET), 0, (hipStream_t)stream, cols, col_stride, ncols,
                       nrows, hi, lo, plane_stride);
    FM_CHECK_LAUNCH("fm_split_planes");
    return FM_OK;
}

namespace fm {
namespace {
__global__ __launch_bounds__(ET) void merge_planes_kernel(const uint32_t* __restrict__ hi, const uint32_t* __restrict__ lo,
                                                          int64_t pstride, int ncols, int64_t nrows,
                                                          double* __restrict__ cols, int64_t stride) {
    const int64_t total = nrows * ncols;
    for (int64_t i = (int64_t)blockIdx.x * ET + threadIdx.x; i < total; i += (int64_t)gridDim.x * ET) {
        const int64_t c = i / nrows, r = i - c * nrows;
        cols[c * stride + r] =
            __longlong_as_double((long long)(((uint64_t)hi[c * pstride + r] << 32) | lo[c * pstride + r]));
    }
}
}  // namespace
}  // namespace fm

extern "C" int fm_merge_planes(const uint32_t* hi, const uint32_t* lo, int64_t plane_stride, int32_t ncols,
                               int64_t nrows, double* cols, int64_t col_stride, void* stream) {
    using namespace fm;
    FM_REQUIRE(cols && hi && lo, "fm_merge_planes: null pointer");
    FM_REQUIRE(ncols >= 0 && nrows >= 0 && col_stride >= nrows && plane_stride >= nrows, "fm_merge_planes: bad sizes");
    if (ncols == 0 || nrows == 0) return FM_OK;
    hipLaunchKernelGGL(merge_planes_kernel, dim3(4096), dim3(ET), 0, (hipStream_t)stream, hi, lo, plane_stride, ncols,
                       nrows, cols, col_stride);
    FM_CHECK_LAUNCH("fm_merge_planes");
    return FM_OK;
}

extern "C" int fm_stream_probe(const double* src, int64_t n, double* out, void* stream) {
    using namespace fm;
    FM_REQUIRE(src && out, "fm_stream_probe: null pointer");
    FM_REQUIRE(((uintptr_t)src & 15) == 0, "fm_stream_probe: src must be 16-byte aligned");
    hipLaunchKernelGGL(probe_kernel, dim3(256 * 8), dim3(ET), 0, (hipStream_t)stream, src, n, out);
    FM_CHECK_LAUNCH("fm_stream_probe");
    return FM_OK;
}

extern "C" int fm_stream_copy_probe(const double* src, double* dst, int64_t n, void* stream) {
    using namespace fm;
    FM_REQUIRE(src && dst, "fm_stream_copy_probe: null pointer");
    FM_REQUIRE((((uintptr_t)src | (uintptr_t)dst) & 15) == 0, "fm_stream_copy_probe: src and dst must be 16-byte aligned");
    FM_REQUIRE(n >= 0, "fm_stream_copy_probe: negative n");
    if (n == 0) return FM_OK;
    hipLaunchKernelGGL(copy_probe_kernel, dim3(256 * 8), dim3(ET), 0, (hipStream_t)stream, src, dst, n);
    FM_CHECK_LAUNCH("fm_stream_copy_probe");
    return FM_OK;
}

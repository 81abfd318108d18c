// Table 1: per-month cross-sectional moments and distinct firms.
//
// Replaces, in build_table_1 (reference src/calc_Lewellen_2014.py:577-670), the inf->NaN
// replacement and dropna (:625-627), groupby("mthcaldt")[var].agg(["mean","std"]) (:638,
// std with ddof=1) and df_clean["permno"].nunique() (:645), for every variable of one
// universe at once (universe = rows with level >= min_level).
#include <math.h>

#include "fm_common.h"

namespace fm {
namespace {

constexpr int MT = 256;
constexpr int MNW = MT / WAVE;

// One workgroup per (month, column): count, mean and ddof=1 std of the non-NaN values
// (finite_only: +-inf count as missing).  Two passes over the segment (L2-resident).
__global__ __launch_bounds__(MT) void moments_kernel(const double* __restrict__ cols, int64_t stride,
                                                     const int64_t* __restrict__ seg_off, int nseg,
                                                     const uint8_t* __restrict__ level, int min_level,
                                                     int finite_only, int32_t* __restrict__ count,
                                                     double* __restrict__ mean, double* __restrict__ sd) {
    __shared__ double dred[MNW];
    __shared__ int ired[MNW];
    const int s = blockIdx.x, c = blockIdx.y;
    const int64_t r0 = seg_off[s], r1 = seg_off[s + 1];
    const double* x = cols + (int64_t)c * stride;
    double sum = 0.0;
    int cnt = 0;
    for (int64_t r = r0 + threadIdx.x; r < r1; r += MT) {
        const double v = x[r];
        const bool lv = level == nullptr || (int)level[r] >= min_level;
        const bool ok = lv && !isnan(v) && (!finite_only || isfinite(v));
        sum += ok ? v : 0.0;
        cnt += ok ? 1 : 0;
    }
    sum = block_sum<MNW>(sum, dred);
    cnt = block_sum<MNW>(cnt, ired);
    const double mu = cnt > 0 ? sum / (double)cnt : NAN;
    double ss = 0.0;
    for (int64_t r = r0 + threadIdx.x; r < r1; r += MT) {
        const double v = x[r];
        const bool lv = level == nullptr || (int)level[r] >= min_level;
        const bool ok = lv && !isnan(v) && (!finite_only || isfinite(v));
        const double d = ok ? v - mu : 0.0;
        ss += d * d;
    }
    ss = block_sum<MNW>(ss, dred);
    if (threadIdx.x == 0) {
        const int64_t o = (int64_t)c * nseg + s;
        count[o] = cnt;
        mean[o] = mu;
        sd[o] = cnt > 1 ? sqrt(ss / (double)(cnt - 1)) : NAN;
    }
}

// Distinct ids among rows where column c is present: a bitmap per column over
// [id_lo, id_lo + id_range), then a popcount.
__global__ __launch_bounds__(MT) void distinct_mark_kernel(const int64_t* __restrict__ ids, int64_t n,
                                                           const double* __restrict__ cols, int64_t stride,
                                                           int ncols, const uint8_t* __restrict__ level,
                                                           int min_level, int finite_only, int64_t id_lo,
                                                           int64_t words, uint32_t* __restrict__ bitmap) {
    for (int64_t r = (int64_t)blockIdx.x * MT + threadIdx.x; r < n; r += (int64_t)gridDim.x * MT) {
        if (level != nullptr && (int)level[r] < min_level) continue;
        const int64_t b = ids[r] - id_lo;
        for (int c = 0; c < ncols; ++c) {
            const double v = cols[(int64_t)c * stride + r];
            if (isnan(v) || (finite_only && !isfinite(v))) continue;
            atomicOr(&bitmap[(int64_t)c * words + (b >> 5)], 1u << (b & 31));
        }
    }
}

__global__ __launch_bounds__(MT) void distinct_count_kernel(const uint32_t* __restrict__ bitmap,
                                                            int64_t words, int32_t* __restrict__ out) {
    __shared__ int red[MNW];
    const int c = blockIdx.x;
    int cnt = 0;
    for (int64_t i = threadIdx.x; i < words; i += MT) cnt += __popc(bitmap[(int64_t)c * words + i]);
    cnt = block_sum<MNW>(cnt, red);
    if (threadIdx.x == 0) out[c] = cnt;
}

}  // namespace
}  // namespace fm

extern "C" int fm_segment_moments(const double* cols, int64_t col_stride, int32_t ncols,
                                  const int64_t* seg_off, int32_t nseg, const uint8_t* level,
                                  int32_t min_level, int32_t finite_only, int32_t* count,
                                  double* mean, double* sd, void* stream) {
    using namespace fm;
    FM_REQUIRE(cols && seg_off && count && mean && sd, "fm_segment_moments: null pointer");
    FM_REQUIRE(ncols > 0 && ncols <= 65535, "fm_segment_moments: bad ncols");
    if (nseg == 0) return FM_OK;
    hipLaunchKernelGGL(moments_kernel, dim3(nseg, ncols), dim3(MT), 0, (hipStream_t)stream, cols,
                       col_stride, seg_off, nseg, level, min_level, finite_only, count, mean, sd);
    FM_CHECK_LAUNCH("fm_segment_moments");
    return FM_OK;
}

extern "C" int fm_distinct_count(const int64_t* ids, int64_t nrows, const double* cols,
                                 int64_t col_stride, int32_t ncols, const uint8_t* level,
                                 int32_t min_level, int32_t finite_only, int64_t id_lo,
                                 int64_t id_range, uint32_t* bitmap, int32_t* out, void* stream) {
    using namespace fm;
    FM_REQUIRE(ids && cols && bitmap && out, "fm_distinct_count: null pointer");
    FM_REQUIRE(id_range > 0 && id_range <= (1ll << 34), "fm_distinct_count: id range out of bounds");
    const int64_t words = (id_range + 31) / 32;
    hipStream_t st = (hipStream_t)stream;
    if (hipMemsetAsync(bitmap, 0, (size_t)words * 4 * ncols, st) != hipSuccess) {
        set_error("fm_distinct_count: hipMemsetAsync failed");
        return FM_EHIP;
    }
    if (nrows > 0) {
        int64_t blocks = (nrows + MT - 1) / MT;
        blocks = blocks > 4096 ? 4096 : blocks;
        hipLaunchKernelGGL(distinct_mark_kernel, dim3((unsigned)blocks), dim3(MT), 0, st, ids, nrows,
                           cols, col_stride, ncols, level, min_level, finite_only, id_lo, words, bitmap);
        FM_CHECK_LAUNCH("fm_distinct_count(mark)");
    }
    hipLaunchKernelGGL(distinct_count_kernel, dim3(ncols), dim3(MT), 0, st, bitmap, words, out);
    FM_CHECK_LAUNCH("fm_distinct_count(count)");
    return FM_OK;
}

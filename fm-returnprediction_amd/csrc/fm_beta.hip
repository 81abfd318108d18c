// fm_rolling_beta: the 156-week rolling market beta of calculate_rolling_beta (reference
// src/calc_Lewellen_2014.py:344-434, a polars group_by_dynamic), on firm-major daily rows.
//
// Reference semantics (restated in oracle/chars_oracle.py; parity UNPINNED: polars 1.22 is
// not installed here): per permno, windows [S, S + 156 weeks) for the Mondays S from the
// week of the firm's first date while S <= its last date, non-empty windows only; per
// window the sums of log(1+Ri), log(1+Rm), their product, log(1+Rm)^2 and the row count;
// beta = (sum_RiRm - sum_Ri sum_Rm / N) / (sum_Rm2 - sum_Rm^2 / N); per (permno, month)
// the LAST window starting in that month is kept.
//
//   beta_prefix_kernel  one workgroup per firm: inclusive prefix sums of the four products
//                       (finite rows) and of the count of non-finite rows, firm-relative
//   beta_query_kernel   one thread per (firm, month) query: the last Monday S of the month
//                       inside [week(first date), last date] whose window holds a row
//                       (binary searches on the firm's days), window sums as prefix
//                       differences; a window of <= 128 rows or with a non-finite log
//                       return is summed directly (IEEE NaN / inf propagation as in
//                       polars; a one-row window's 0/0 stays NaN)
#include <math.h>

#include "fm_common.h"

namespace fm {
namespace {

constexpr int BT = 256;

__device__ __forceinline__ int week_start_dev(int d) {   // Monday; 1970-01-01 was a Thursday
    int m = (d + 3) % 7;
    if (m < 0) m += 7;
    return d - m;
}

__global__ __launch_bounds__(BT) void beta_prefix_kernel(const double* __restrict__ ri,
                                                         const double* __restrict__ rm,
                                                         const int64_t* __restrict__ seg_off, int64_t n,
                                                         double* __restrict__ ws) {
    __shared__ double tot[5][BT];
    const int f = blockIdx.x, tid = threadIdx.x;
    const int64_t a = seg_off[f], b = seg_off[f + 1];
    const int64_t L = b - a;
    const int64_t per = (L + BT - 1) / BT;
    const int64_t c0 = a + tid * per, c1 = c0 + per < b ? c0 + per : b;
    double s[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
    for (int64_t i = c0; i < c1; ++i) {
        const double x = log(ri[i] + 1.0), y = log(rm[i] + 1.0);
        if (isfinite(x) && isfinite(y)) {
            s[0] += x;
            s[1] += y;
            s[2] += x * y;
            s[3] += y * y;
        } else {
            s[4] += 1.0;
        }
    }
#pragma unroll
    for (int k = 0; k < 5; ++k) tot[k][tid] = s[k];
    __syncthreads();
    if (tid < 5) {   // exclusive scan of the 256 chunk totals, one quantity per thread
        double run = 0.0;
        for (int t = 0; t < BT; ++t) {
            const double v = tot[tid][t];
            tot[tid][t] = run;
            run += v;
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 5; ++k) s[k] = tot[k][tid];
    for (int64_t i = c0; i < c1; ++i) {
        const double x = log(ri[i] + 1.0), y = log(rm[i] + 1.0);
        if (isfinite(x) && isfinite(y)) {
            s[0] += x;
            s[1] += y;
            s[2] += x * y;
            s[3] += y * y;
        } else {
            s[4] += 1.0;
        }
#pragma unroll
        for (int k = 0; k < 5; ++k) ws[(int64_t)k * n + i] = s[k];
    }
}

__device__ __forceinline__ int64_t lower_bound_days(const int32_t* day, int64_t lo, int64_t hi, int v) {
    while (lo < hi) {
        const int64_t mid = lo + ((hi - lo) >> 1);
        if (day[mid] < v) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// numpy's pairwise-sum leaf (a block of <= 128 values: eight running accumulators combined
// as ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)), then the n % 8 tail; < 8 values in order), so a
// short window's sums are the oracle's bit for bit.  Longer windows (non-finite ones only)
// are summed in row order: NaN / inf propagate the same either way.
constexpr int PW_BLOCK = 128;

__device__ __forceinline__ void window_sums(const double* ri, const double* rm, int64_t i0, int64_t i1,
                                            double s[5]) {
    const int64_t n = i1 - i0;
    auto at = [&](int64_t i, double v[4]) {
        const double x = log(ri[i] + 1.0), y = log(rm[i] + 1.0);
        v[0] = x;
        v[1] = y;
        v[2] = x * y;
        v[3] = y * y;
    };
    double v[4];
    if (n < 8 || n > PW_BLOCK) {
        s[0] = s[1] = s[2] = s[3] = 0.0;
        for (int64_t i = i0; i < i1; ++i) {
            at(i, v);
#pragma unroll
            for (int k = 0; k < 4; ++k) s[k] += v[k];
        }
        return;
    }
    double r[4][8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        at(i0 + j, v);
#pragma unroll
        for (int k = 0; k < 4; ++k) r[k][j] = v[k];
    }
    const int64_t m = n - n % 8;
    for (int64_t i = 8; i < m; i += 8) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            at(i0 + i + j, v);
#pragma unroll
            for (int k = 0; k < 4; ++k) r[k][j] += v[k];
        }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) s[k] = ((r[k][0] + r[k][1]) + (r[k][2] + r[k][3])) + ((r[k][4] + r[k][5]) + (r[k][6] + r[k][7]));
    for (int64_t i = m; i < n; ++i) {
        at(i0 + i, v);
#pragma unroll
        for (int k = 0; k < 4; ++k) s[k] += v[k];
    }
}

__global__ __launch_bounds__(BT) void beta_query_kernel(const int32_t* __restrict__ day,
                                                        const double* __restrict__ ri,
                                                        const double* __restrict__ rm,
                                                        const int64_t* __restrict__ seg_off, int64_t n,
                                                        int period_days, const int32_t* __restrict__ q_seg,
                                                        const int32_t* __restrict__ q_day0,
                                                        const int32_t* __restrict__ q_day1, int nq,
                                                        const double* __restrict__ ws, double* __restrict__ out) {
    const int q = blockIdx.x * BT + threadIdx.x;
    if (q >= nq) return;
    const int f = q_seg[q];
    const int64_t a = seg_off[f], b = seg_off[f + 1];
    double beta = NAN;
    if (b > a) {
        const int t0 = week_start_dev(day[a]), last = day[b - 1];
        for (int S = week_start_dev(q_day1[q]); S >= q_day0[q]; S -= 7) {
            if (S < t0 || S > last) continue;
            const int64_t i0 = lower_bound_days(day, a, b, S);
            const int64_t i1 = lower_bound_days(day, i0, b, S + period_days);
            if (i1 <= i0) continue;   // an empty window is not emitted
            double s[5];
#pragma unroll
            for (int k = 0; k < 5; ++k)
                s[k] = ws[(int64_t)k * n + i1 - 1] - (i0 > a ? ws[(int64_t)k * n + i0 - 1] : 0.0);
            if (s[4] > 0.0 || i1 - i0 <= PW_BLOCK) {
                // short windows (prefix differences lose digits there, and a one-row window
                // must give 0/0) and windows with a non-finite log return: summed directly
                window_sums(ri, rm, i0, i1, s);
            }
            const double N = (double)(i1 - i0);
            beta = (s[2] - s[0] * s[1] / N) / (s[3] - s[1] * s[1] / N);
            break;
        }
    }
    out[q] = beta;
}

}  // namespace
}  // namespace fm

extern "C" int fm_rolling_beta(const int32_t* day, const double* ri, const double* rm, int64_t n,
                               const int64_t* seg_off, int32_t nseg, int32_t period_days,
                               const int32_t* q_seg, const int32_t* q_day0, const int32_t* q_day1,
                               int32_t nq, double* ws, double* beta, void* stream) {
    using namespace fm;
    FM_REQUIRE(n >= 0 && nseg >= 0 && nq >= 0 && period_days >= 1, "fm_rolling_beta: bad sizes");
    if (nq == 0) return FM_OK;
    FM_REQUIRE(q_seg && q_day0 && q_day1 && beta && seg_off, "fm_rolling_beta: null pointer");
    hipStream_t st = (hipStream_t)stream;
    if (n > 0 && nseg > 0) {
        FM_REQUIRE(day && ri && rm && ws, "fm_rolling_beta: null pointer");
        hipLaunchKernelGGL(beta_prefix_kernel, dim3((unsigned)nseg), dim3(BT), 0, st, ri, rm, seg_off, n, ws);
        FM_CHECK_LAUNCH("fm_rolling_beta(prefix)");
    }
    hipLaunchKernelGGL(beta_query_kernel, dim3((unsigned)((nq + BT - 1) / BT)), dim3(BT), 0, st, day, ri, rm,
                       seg_off, n, period_days, q_seg, q_day0, q_day1, nq, ws, beta);
    FM_CHECK_LAUNCH("fm_rolling_beta(query)");
    return FM_OK;
}

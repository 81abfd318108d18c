// Time-series stage on device: Fama-MacBeth averages with Newey-West errors, the
// 120-month rolling coefficient means, and the lagged-rolling forecasts with their
// predictive-slope regressions.
//
//   fm_ts_compact   the month list of each problem (months with status FITTED, ascending)
//                   = the rows of the reference's results_df (src/regressions.py:75)
//   fm_ts_summary   per coefficient: slopes.dropna() (:113), mean (:120), NW s.e. with
//                   weights 1-k/T that stop at the first negative weight (:78-100),
//                   t = mean/se (:125); also used for mean_R2 / mean_N (:128-129)
//   fm_rolling_mean rolling(window, min_periods).mean() over the fitted-month rows, NaN
//                   values skipped and not counted (src/calc_Lewellen_2014.py:926)
//   fm_predictive   build-defined A7/A8: with c = the rolling coefficients `lag` rows
//                   earlier, F_i = c0 + c'x_i; the per-month OLS of y on [1, F] has
//                   slope = c'Sxy / c'Sxx c and R^2 = (c'Sxy)^2 / (c'Sxx c * Syy), both
//                   from the month's centered moments, so no second pass over the panel.
//
// Record addressing is strided so the same kernels serve the per-(month, problem)
// records of fm_solve and the per-(problem, month) predictive records.
#include <math.h>

#include "fm_common.h"

namespace fm {
namespace {

constexpr int TT = 256;
constexpr int TNW = TT / WAVE;

__global__ __launch_bounds__(TT) void compact_kernel(const uint32_t* status, int64_t s_seg,
                                                     int64_t s_prob, int nseg, int32_t* idx,
                                                     int32_t* count) {
    __shared__ int scr[TNW];
    const int p = blockIdx.x;
    int base = 0;
    for (int s0 = 0; s0 < nseg; s0 += TT) {
        const int s = s0 + threadIdx.x;
        const int f = (s < nseg && (status[s * s_seg + p * s_prob] & FM_ST_FITTED)) ? 1 : 0;
        int tot = 0;
        const int off = block_excl_scan<TNW>(f, scr, &tot);
        if (f) idx[(int64_t)p * nseg + base + off] = s;
        base += tot;
    }
    if (threadIdx.x == 0) count[p] = base;
}

struct SumArgs {
    const double* rec;
    int64_t r_seg, r_prob;
    const int32_t* idx;
    const int32_t* count;
    int nseg, kmax, nw_lags;
    double* mean;
    double* se;
    double* tstat;
    int32_t* nobs;
    double* work;
};

__global__ __launch_bounds__(TT) void summary_kernel(SumArgs a) {
    __shared__ double dred[TNW];
    __shared__ int ired[TNW];
    const int k = blockIdx.x, p = blockIdx.y;
    const int cnt = a.count[p];
    const int32_t* ix = a.idx + (int64_t)p * a.nseg;
    double* wk = a.work + ((int64_t)p * a.kmax + k) * a.nseg;
    // dropna-compaction, preserving month order
    int base = 0;
    for (int i0 = 0; i0 < cnt; i0 += TT) {
        const int i = i0 + threadIdx.x;
        double x = NAN;
        if (i < cnt) x = a.rec[(int64_t)ix[i] * a.r_seg + (int64_t)p * a.r_prob + k];
        const int f = (i < cnt && !isnan(x)) ? 1 : 0;
        int tot = 0;
        const int off = block_excl_scan<TNW>(f, ired, &tot);
        if (f) wk[base + off] = x;
        base += tot;
    }
    __syncthreads();
    const int n = base;
    double sum = 0.0;
    for (int i = threadIdx.x; i < n; i += TT) sum += wk[i];
    sum = block_sum<TNW>(sum, dred);
    const double mu = n > 0 ? sum / (double)n : NAN;
    // Newey-West: gamma_k = sum u[i] u[i-k], w_k = 1 - k/T, stop at the first w_k < 0
    double g0 = 0.0;
    for (int i = threadIdx.x; i < n; i += TT) {
        const double u = wk[i] - mu;
        g0 += u * u;
    }
    g0 = block_sum<TNW>(g0, dred);
    double acc = 0.0;
    for (int L = 1; L <= a.nw_lags; ++L) {
        const double wgt = 1.0 - ((double)L / (double)n);
        if (wgt < 0.0) break;
        double gk = 0.0;
        for (int i = L + threadIdx.x; i < n; i += TT) gk += (wk[i] - mu) * (wk[i - L] - mu);
        gk = block_sum<TNW>(gk, dred);
        acc += wgt * gk;
    }
    if (threadIdx.x == 0) {
        const int64_t o = (int64_t)p * a.kmax + k;
        double se = NAN;
        if (n >= 2) se = sqrt((g0 + 2.0 * acc) / ((double)n * (double)n));
        a.mean[o] = mu;
        a.se[o] = se;
        a.tstat[o] = mu / se;
        a.nobs[o] = n;
    }
}

// One workgroup per (problem, coefficient, chunk of RCH output rows): the chunk's window
// span is staged in LDS, each output is a direct sum over its window (no running-sum drift).
constexpr int RCH = 1024;
constexpr int RMAXW = 1024;

__global__ __launch_bounds__(TT) void rolling_kernel(const double* rec, int64_t r_seg,
                                                     int64_t r_prob, const int32_t* idx,
                                                     const int32_t* count, int nseg, int kmax,
                                                     int window, int minp, double* out) {
    __shared__ double xs[RCH + RMAXW];
    const int p = blockIdx.y / kmax, k = blockIdx.y - (blockIdx.y / kmax) * kmax;
    const int c0 = blockIdx.x * RCH;
    const int cnt = count[p];
    if (c0 >= cnt) return;
    const int32_t* ix = idx + (int64_t)p * nseg;
    const int lo = c0 - window + 1 < 0 ? 0 : c0 - window + 1;
    const int hi = c0 + RCH < cnt ? c0 + RCH : cnt;
    for (int j = lo + threadIdx.x; j < hi; j += TT)
        xs[j - lo] = rec[(int64_t)ix[j] * r_seg + (int64_t)p * r_prob + k];
    __syncthreads();
    for (int i = c0 + threadIdx.x; i < hi; i += TT) {
        const int j0 = i - window + 1 < 0 ? 0 : i - window + 1;
        double sm = 0.0;
        int c = 0;
        for (int j = j0; j <= i; ++j) {
            const double x = xs[j - lo];
            if (!isnan(x)) {
                sm += x;
                ++c;
            }
        }
        out[((int64_t)p * nseg + i) * kmax + k] = c >= minp ? sm / (double)c : NAN;
    }
}

// One wave per (problem, fitted-month row); lane a owns regressor a.
__global__ __launch_bounds__(WAVE) void predictive_kernel(const double* mom, int mom_stride,
                                                          int nseg, int nprob,
                                                          const int32_t* prob_k, const int32_t* idx,
                                                          const int32_t* count, const double* roll,
                                                          int pmax, int lag, int seg_lo, int seg_hi,
                                                          double* pred, uint32_t* pst) {
    const int p = blockIdx.y, i = blockIdx.x, lane = threadIdx.x;
    double* o = pred + ((int64_t)p * nseg + i) * 4;
    const int cnt = count[p];
    const int s = i < cnt ? idx[(int64_t)p * nseg + i] : -1;
    if (i < cnt && (s < seg_lo || s >= seg_hi)) {
        // another rank's month (sharded runs): zero record for the sum-combine
        if (lane < 4) o[lane] = 0.0;
        if (lane == 0) pst[(int64_t)p * nseg + i] = 0;
        return;
    }
    uint32_t st = 0;
    double slope = NAN, r2 = NAN, nn = NAN;
    if (i < cnt && i >= lag) {
        const int K = prob_k[p];
        const double* c = roll + ((int64_t)p * nseg + (i - lag)) * pmax;
        const bool bad = lane <= K && isnan(c[lane]);
        const double* mo = mom + ((int64_t)(s - seg_lo) * nprob + p) * mom_stride;
        const int K1 = K + 1;
        const double n = mo[0];
        if (__ballot(bad) == 0 && n >= 2.0) {
            const double* S = mo + 1 + K1;
            double tb = 0.0, ty = 0.0;
            if (lane < K) {
                double t = 0.0;
                for (int b = 0; b < K; ++b) t += S[lane * K1 + b] * c[1 + b];
                tb = c[1 + lane] * t;
                ty = c[1 + lane] * S[lane * K1 + K];
            }
            const double bsb = wave_sum(tb), bsy = wave_sum(ty);
            const double syy = S[K * K1 + K];
            slope = bsy / bsb;
            r2 = (bsy * bsy) / (bsb * syy);
            nn = n;
            st = FM_ST_FITTED;
            if (!(bsb > 0.0)) st |= FM_ST_CONST_COL;
        }
    }
    if (lane == 0) {
        o[0] = slope;
        o[1] = r2;
        o[2] = nn;
        o[3] = 0.0;
        pst[(int64_t)p * nseg + i] = st;
    }
}

// Per-row forecast F = c0 + sum_k c_k x_k with the segment's coefficient row (A7).
__global__ __launch_bounds__(TT) void forecast_kernel(const double* cols, int64_t stride, int K,
                                                      const int64_t* seg_off, const double* coef,
                                                      int cstride, double* out) {
    const int s = blockIdx.x;
    const int64_t r0 = seg_off[s], r1 = seg_off[s + 1];
    const double* c = coef + (int64_t)s * cstride;
    for (int64_t r = r0 + (int64_t)blockIdx.z * TT + threadIdx.x; r < r1; r += (int64_t)gridDim.z * TT) {
        double f = c[0];
        for (int k = 0; k < K; ++k) f += c[1 + k] * cols[(int64_t)k * stride + r];
        out[r] = f;
    }
}

}  // namespace
}  // namespace fm

extern "C" int fm_forecast(const double* cols, int64_t col_stride, int32_t K,
                           const int64_t* seg_off, int32_t nseg, int64_t nrows, const double* coef,
                           int32_t coef_stride, double* out, void* stream) {
    using namespace fm;
    FM_REQUIRE(cols && seg_off && coef && out, "fm_forecast: null pointer");
    FM_REQUIRE(K >= 0 && coef_stride >= K + 1, "fm_forecast: bad K / coef_stride");
    if (nseg == 0) return FM_OK;
    int64_t z = (nrows / nseg + 4 * TT - 1) / (4 * TT);
    z = z < 1 ? 1 : (z > 64 ? 64 : z);
    hipLaunchKernelGGL(forecast_kernel, dim3(nseg, 1, (unsigned)z), dim3(TT), 0, (hipStream_t)stream,
                       cols, col_stride, K, seg_off, coef, coef_stride, out);
    FM_CHECK_LAUNCH("fm_forecast");
    return FM_OK;
}

extern "C" int fm_ts_compact(const uint32_t* status, int64_t s_seg, int64_t s_prob, int32_t nseg,
                             int32_t nprob, int32_t* idx, int32_t* count, void* stream) {
    using namespace fm;
    FM_REQUIRE(status && idx && count, "fm_ts_compact: null pointer");
    if (nprob == 0) return FM_OK;
    hipLaunchKernelGGL(compact_kernel, dim3(nprob), dim3(TT), 0, (hipStream_t)stream, status, s_seg,
                       s_prob, nseg, idx, count);
    FM_CHECK_LAUNCH("fm_ts_compact");
    return FM_OK;
}

extern "C" int fm_ts_summary(const double* rec, int64_t r_seg, int64_t r_prob, const int32_t* idx,
                             const int32_t* count, int32_t nseg, int32_t nprob, int32_t kmax,
                             int32_t nw_lags, double* mean, double* se, double* tstat,
                             int32_t* nobs, double* work, void* stream) {
    using namespace fm;
    FM_REQUIRE(rec && idx && count && mean && se && tstat && nobs && work,
               "fm_ts_summary: null pointer");
    FM_REQUIRE(nw_lags >= 0, "fm_ts_summary: nw_lags < 0");
    if (nprob == 0 || kmax == 0) return FM_OK;
    SumArgs a{rec, r_seg, r_prob, idx, count, nseg, kmax, nw_lags, mean, se, tstat, nobs, work};
    hipLaunchKernelGGL(summary_kernel, dim3(kmax, nprob), dim3(TT), 0, (hipStream_t)stream, a);
    FM_CHECK_LAUNCH("fm_ts_summary");
    return FM_OK;
}

extern "C" int fm_rolling_mean(const double* rec, int64_t r_seg, int64_t r_prob,
                               const int32_t* idx, const int32_t* count, int32_t nseg,
                               int32_t nprob, int32_t kmax, int32_t window, int32_t min_periods,
                               double* out, void* stream) {
    using namespace fm;
    FM_REQUIRE(rec && idx && count && out, "fm_rolling_mean: null pointer");
    FM_REQUIRE(window >= 1 && window <= RMAXW && min_periods >= 0,
               "fm_rolling_mean: window must be 1..%d", RMAXW);
    if (nprob == 0 || nseg == 0 || kmax == 0) return FM_OK;
    dim3 grid((nseg + RCH - 1) / RCH, nprob * kmax);
    hipLaunchKernelGGL(rolling_kernel, grid, dim3(TT), 0, (hipStream_t)stream, rec, r_seg, r_prob,
                       idx, count, nseg, kmax, window, min_periods, out);
    FM_CHECK_LAUNCH("fm_rolling_mean");
    return FM_OK;
}

extern "C" int fm_predictive(const double* moments, int32_t mom_stride, int32_t nseg,
                             int32_t nprob, const int32_t* prob_k, const int32_t* idx,
                             const int32_t* count, const double* rolling, int32_t pmax,
                             int32_t lag, int32_t seg_lo, int32_t seg_hi, double* pred,
                             uint32_t* pred_status, void* stream) {
    using namespace fm;
    FM_REQUIRE(moments && prob_k && idx && count && rolling && pred && pred_status,
               "fm_predictive: null pointer");
    FM_REQUIRE(lag >= 1, "fm_predictive: lag must be >= 1");
    if (nprob == 0 || nseg == 0) return FM_OK;
    dim3 grid(nseg, nprob);
    hipLaunchKernelGGL(predictive_kernel, grid, dim3(WAVE), 0, (hipStream_t)stream, moments,
                       mom_stride, nseg, nprob, prob_k, idx, count, rolling, pmax, lag, seg_lo,
                       seg_hi, pred, pred_status);
    FM_CHECK_LAUNCH("fm_predictive");
    return FM_OK;
}

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
//                   and +-inf values skipped and not counted (pandas' rolling turns inf
//                   into NaN before its window sums; src/calc_Lewellen_2014.py:926)
//   fm_predictive   build-defined A7/A8: with c = the rolling coefficients `lag` rows
//                   earlier, F_i = c0 + c'x_i; the per-month OLS of y on [1, F] has
//                   slope = c'Sxy / c'Sxx c and R^2 = (c'Sxy)^2 / (c'Sxx c * Syy), both
//                   from the month's centered moments, so no second pass over the panel.
//
// Record addressing is strided so the same kernels serve the per-(month, problem)
// records of fm_solve and the per-(problem, month) predictive records.
#include <math.h>

#include "fm_common.h"

FM_PROBE_BUFFER(ts)

namespace fm {
namespace {

constexpr int TT = 256;
constexpr int TNW = TT / WAVE;

// Grid (chunks of CB months, problems): a workgroup counts the fitted months before its chunk
// (a strided pass over the earlier status words) and scans its own chunk (CPT contiguous
// months per thread), so a 100,000-month series takes one launch of independent workgroups
// instead of one workgroup scanning the whole series.
constexpr int CPT = 16;
constexpr int CB = TT * CPT;
__global__ __launch_bounds__(TT) void compact_kernel(const uint32_t* status, int64_t s_seg,
                                                     int64_t s_prob, int nseg, int32_t* idx,
                                                     int32_t* count) {
    __shared__ int scr[TNW];
    const int p = blockIdx.y;
    const int c0 = blockIdx.x * CB;
    const uint32_t* sp = status + (int64_t)p * s_prob;
    int before = 0;
    for (int s = threadIdx.x; s < c0; s += TT) before += (sp[(int64_t)s * s_seg] & FM_ST_FITTED) ? 1 : 0;
    before = block_sum<TNW>(before, scr);
    const int m0 = c0 + (int)threadIdx.x * CPT;
    uint32_t fm = 0;
    int loc = 0;
#pragma unroll
    for (int j = 0; j < CPT; ++j) {
        const int s = m0 + j;
        const bool f = s < nseg && (sp[(int64_t)(s < nseg ? s : 0) * s_seg] & FM_ST_FITTED);
        fm |= (f ? 1u : 0u) << j;
        loc += f ? 1 : 0;
    }
    int tot = 0;
    int pos = before + block_excl_scan<TNW>(loc, scr, &tot);
#pragma unroll
    for (int j = 0; j < CPT; ++j)
        if ((fm >> j) & 1u) idx[(int64_t)p * nseg + pos++] = m0 + j;
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) count[p] = before + tot;
}

struct SumArgs {
    const double* rec;
    int64_t r_seg, r_prob;
    const int32_t* idx;
    const int32_t* count;
    int nseg, kmax, nw_lags, nprob;
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

// Long series (>= SUM_CHUNKED months), three launches:
//   summary_gather_kernel  the fitted-month records of every (problem, coefficient) into
//                          contiguous series work[p][k][0..count) (one row's coefficients are
//                          adjacent in the records, so a workgroup reads rows x all k)
//   summary_part_kernel    per (chunk of SCH rows, coefficient, problem): NaN dropped in order,
//                          y' = x - K_c (K_c = the chunk's first value): m, S1', S2', the
//                          in-chunk lagged cross sums C'_L and the first / last SUM_MAXLAG y'
//   summary_combine_kernel per series, the chunks in order: each chunk's sums re-shifted to
//                          K0 = the series' first value (delta = K_c - K0), the lag pairs that
//                          straddle chunk boundaries from a ring of the last values so far;
//                          with d = S1 / n (= mean - K0),
//                          gamma_0 = S2 - n d^2, gamma_L = C_L - d (A_L + B_L) + (n - L) d^2,
//                          A_L / B_L = S1 minus the first / last L values -- the Newey-West
//                          sums of the two-pass formula in one pass over the series.
// work: [nprob][kmax][nseg] series, then [nprob][kmax][nchunk][SPART] partials.
constexpr int SCH = 2048;
constexpr int SPT = SCH / TT;
constexpr int SUM_MAXLAG = 8;
constexpr int SPART = 4 + SUM_MAXLAG + 2 * SUM_MAXLAG;   // m, K_c, S1', S2', C'_L, first, last
constexpr int SUM_CHUNKED = 4096;
constexpr int GROWS = 64;   // rows per gather workgroup (x kmax coefficients)

__global__ __launch_bounds__(TT) void summary_gather_kernel(SumArgs a) {
    const int p = blockIdx.y, r0 = blockIdx.x * GROWS;
    const int cnt = a.count[p];
    const int32_t* ix = a.idx + (int64_t)p * a.nseg;
    for (int e = threadIdx.x; e < GROWS * a.kmax; e += TT) {
        const int r = r0 + e / a.kmax, k = e - (e / a.kmax) * a.kmax;
        if (r < cnt)
            a.work[((int64_t)p * a.kmax + k) * a.nseg + r] = a.rec[(int64_t)ix[r] * a.r_seg + (int64_t)p * a.r_prob + k];
    }
}

__global__ __launch_bounds__(TT) void summary_part_kernel(SumArgs a) {
    __shared__ double ys[SCH];
    __shared__ int ired[TNW];
    __shared__ double dred[TNW];
    const int c = blockIdx.x, k = blockIdx.y, p = blockIdx.z;
    const int cnt = a.count[p];
    const int c0 = c * SCH;
    const double* ser = a.work + ((int64_t)p * a.kmax + k) * a.nseg;
    double* part = a.work + (int64_t)a.nprob * a.kmax * a.nseg +
                   (((int64_t)p * a.kmax + k) * gridDim.x + c) * SPART;
    // this chunk's values, SPT contiguous rows per thread, NaN dropped in order
    const int i0 = c0 + (int)threadIdx.x * SPT;
    double y[SPT];
    int loc = 0;
#pragma unroll
    for (int j = 0; j < SPT; ++j) {
        const int i = i0 + j;
        y[j] = i < cnt ? ser[i] : (double)NAN;
        loc += isnan(y[j]) ? 0 : 1;
    }
    int m = 0;
    int pos = block_excl_scan<TNW>(loc, ired, &m);
#pragma unroll
    for (int j = 0; j < SPT; ++j)
        if (!isnan(y[j])) ys[pos++] = y[j];
    __syncthreads();
    const double kc = m > 0 ? ys[0] : 0.0;
    double s1 = 0.0, s2 = 0.0, cl[SUM_MAXLAG];
#pragma unroll
    for (int l = 0; l < SUM_MAXLAG; ++l) cl[l] = 0.0;
    for (int j = threadIdx.x; j < m; j += TT) {
        const double v = ys[j] - kc;
        s1 += v;
        s2 += v * v;
#pragma unroll
        for (int l = 1; l <= SUM_MAXLAG; ++l)
            if (j - l >= 0) cl[l - 1] += v * (ys[j - l] - kc);
    }
    s1 = block_sum<TNW>(s1, dred);
    s2 = block_sum<TNW>(s2, dred);
#pragma unroll
    for (int l = 0; l < SUM_MAXLAG; ++l) {
        const double t = block_sum<TNW>(cl[l], dred);
        if (threadIdx.x == 0) part[4 + l] = t;
    }
    if (threadIdx.x == 0) {
        part[0] = (double)m;
        part[1] = kc;
        part[2] = s1;
        part[3] = s2;
    }
    if (threadIdx.x < SUM_MAXLAG) {
        const int t = threadIdx.x;
        part[4 + SUM_MAXLAG + t] = t < m ? ys[t] - kc : 0.0;                        // first
        part[4 + 2 * SUM_MAXLAG + t] = t < m ? ys[m - 1 - t] - kc : 0.0;            // last (reversed)
    }
}

// One wave per (coefficient, problem): the partials staged in LDS by all lanes, then the
// chunks in order (see above); mean, Newey-West s.e. and t (weights 1 - L/n, stop at the
// first negative weight; src/regressions.py:78-100).
constexpr int SCMAX = 64;   // chunks staged in LDS per pass of the combine
__global__ __launch_bounds__(WAVE) void summary_combine_kernel(SumArgs a, int nchunk) {
    __shared__ double stage[SCMAX * SPART];
    const int k = blockIdx.x, p = blockIdx.y;
    const int L = a.nw_lags < SUM_MAXLAG ? a.nw_lags : SUM_MAXLAG;
    const double* gpart = a.work + (int64_t)a.nprob * a.kmax * a.nseg + ((int64_t)p * a.kmax + k) * nchunk * SPART;
    const double* part = stage;
    int n = 0;
    double k0 = NAN, S1 = 0.0, S2 = 0.0, C[SUM_MAXLAG];
    double head[SUM_MAXLAG], ring[SUM_MAXLAG];   // first values; the last values so far (ring[0] newest)
    int nhead = 0;
#pragma unroll
    for (int l = 0; l < SUM_MAXLAG; ++l) C[l] = head[l] = ring[l] = 0.0;
    for (int c = 0; c < nchunk; ++c) {
        if (c % SCMAX == 0) {   // the next SCMAX chunks' partials, all lanes loading
            __syncthreads();
            const int nc = nchunk - c < SCMAX ? nchunk - c : SCMAX;
            for (int e = threadIdx.x; e < nc * SPART; e += WAVE) stage[e] = gpart[(int64_t)c * SPART + e];
            __syncthreads();
        }
        const double* q = part + (int64_t)(c % SCMAX) * SPART;
        const int m = (int)q[0];
        if (m == 0) continue;
        if (n == 0) k0 = q[1];
        const double dl = q[1] - k0;   // re-shift this chunk's sums from K_c to K0
        const double s1p = q[2], s2p = q[3];
        double fsum = 0.0, lsum = 0.0;
#pragma unroll
        for (int l = 1; l <= SUM_MAXLAG; ++l) {
            if (l > L) break;
            fsum += l - 1 < m ? q[4 + SUM_MAXLAG + l - 1] : 0.0;
            lsum += l - 1 < m ? q[4 + 2 * SUM_MAXLAG + l - 1] : 0.0;
            const int pc = m - l > 0 ? m - l : 0;   // in-chunk pairs at lag l
            double cc = q[4 + l - 1];
            if (pc > 0) cc += dl * ((s1p - fsum) + (s1p - lsum)) + (double)pc * dl * dl;
            // pairs (j, j - l) with j < l: partners before this chunk (the ring)
#pragma unroll
            for (int j = 0; j < SUM_MAXLAG; ++j)
                if (j < l && j < m && l - 1 - j < n && l - 1 - j < SUM_MAXLAG)
                    cc += (q[4 + SUM_MAXLAG + j] + dl) * ring[l - 1 - j];
            C[l - 1] += cc;
        }
        S1 += s1p + (double)m * dl;
        S2 += s2p + 2.0 * dl * s1p + (double)m * dl * dl;
        // the global first values; the ring of the last values (shifted to K0)
#pragma unroll
        for (int j = 0; j < SUM_MAXLAG; ++j)
            if (j < m && nhead < SUM_MAXLAG) head[nhead++] = q[4 + SUM_MAXLAG + j] + dl;
        const int push = m < SUM_MAXLAG ? m : SUM_MAXLAG;
#pragma unroll
        for (int j = SUM_MAXLAG - 1; j >= 0; --j)   // older values move back by `push`
            ring[j] = j - push >= 0 ? ring[j - push] : q[4 + 2 * SUM_MAXLAG + j] + dl;
        n += m;
    }
    double mu = NAN, se = NAN;
    if (n > 0) {
        const double d = S1 / (double)n;
        mu = k0 + d;
        const double g0 = S2 - (double)n * d * d;
        double accn = 0.0, hs = 0.0, ts = 0.0;
#pragma unroll
        for (int l = 1; l <= SUM_MAXLAG; ++l) {
            if (l > L) break;
            const double w = 1.0 - ((double)l / (double)n);
            if (w < 0.0) break;
            hs += head[l - 1];   // the first l values
            ts += ring[l - 1];   // the last l values
            accn += w * (C[l - 1] - d * ((S1 - hs) + (S1 - ts)) + (double)(n - l) * d * d);
        }
        if (n >= 2) se = sqrt((g0 + 2.0 * accn) / ((double)n * (double)n));
    }
    if (threadIdx.x == 0) {   // every lane walked the same (LDS-broadcast) partials
        const int64_t o = (int64_t)p * a.kmax + k;
        a.mean[o] = mu;
        a.se[o] = se;
        a.tstat[o] = mu / se;
        a.nobs[o] = n;
    }
}

// Grid (chunks of RCH output rows, problem): the chunk's window span of ALL coefficients is
// staged in LDS (a row's coefficients are adjacent in the records: one gather per row, not
// one per coefficient); thread (k, g) owns coefficient k on RPT consecutive rows: the first
// output is a direct sum over its window, the next RPT-1 slide it (add the entering row, drop
// the leaving one; finite values only -- pandas turns +-inf into NaN).
constexpr int RKMAX = 16;                 // coefficients per problem (pmax <= 16 here)
constexpr int RKS = RKMAX + 1;            // LDS row stride (odd: the row groups hit other banks)
constexpr int RPT = 16;                   // rows per thread
constexpr int RCH = TT / RKMAX * RPT;     // 256 output rows per workgroup
constexpr int RMAXW = 1024;
constexpr int RSPAN = RCH + 128;          // staged rows (windows up to 129 here): 52 KB of LDS

// First position of the ascending list ix[0..n) holding a value >= v (block-uniform).
__device__ __forceinline__ int lower_bound_i32(const int32_t* ix, int n, int v) {
    int lo = 0, hi = n;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (ix[mid] < v) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// own != 0 (fm_rolling_mean_own): only the rows [ra, rb) = [first fitted row of a month >=
// m_lo, minus lag; first fitted row of a month >= m_hi) are needed; workgroups and per-thread
// row blocks without such a row are skipped, the others compute exactly as in the full mode
// (same row-to-thread map, so the same bits), and no NaN fill is written.
__global__ __launch_bounds__(TT) void rolling_kernel(const double* rec, int64_t r_seg,
                                                     int64_t r_prob, const int32_t* idx,
                                                     const int32_t* count, int nseg, int kmax,
                                                     int window, int minp, double* out, int own,
                                                     int m_lo, int m_hi, int lag) {
    __shared__ double xs[RSPAN * RKS];
    const int p = blockIdx.y;
    const int c0 = blockIdx.x * RCH;
    const int cnt = count[p];
    const int32_t* ix = idx + (int64_t)p * nseg;
    int ra = 0, rb = cnt;
    if (own) {
        ra = lower_bound_i32(ix, cnt, m_lo) - lag;
        ra = ra < 0 ? 0 : ra;
        rb = lower_bound_i32(ix, cnt, m_hi);
        if (c0 + RCH <= ra || c0 >= rb) return;   // block-uniform
    } else {
        // rows past the fitted-month count have no month: NaN (never left uninitialised)
        const int cend = c0 + RCH < nseg ? c0 + RCH : nseg;
        for (int e = threadIdx.x; e < (cend - c0) * kmax; e += TT) {
            const int i = c0 + e / kmax;
            if (i >= cnt) out[((int64_t)p * nseg + i) * kmax + (e % kmax)] = NAN;
        }
    }
    if (c0 >= cnt) return;
    const int lo = c0 - window + 1 < 0 ? 0 : c0 - window + 1;
    const int hi = c0 + RCH < cnt ? c0 + RCH : cnt;
    for (int e = threadIdx.x; e < (hi - lo) * kmax; e += TT) {
        const int j = lo + e / kmax, k = e % kmax;
        xs[(j - lo) * RKS + k] = rec[(int64_t)ix[j] * r_seg + (int64_t)p * r_prob + k];
    }
    __syncthreads();
    const int k = threadIdx.x % RKMAX, g = threadIdx.x / RKMAX;
    const int ib = c0 + g * RPT;
    if (k >= kmax || ib >= hi) return;
    if (own && (ib + RPT <= ra || ib >= rb)) return;   // this thread's rows are not needed
    const int j0 = ib - window + 1 < 0 ? 0 : ib - window + 1;
    CSum sm;   // compensated: an outlier leaving the window leaves no ulp(outlier) behind
    int c = 0;
    for (int j = j0; j <= ib; ++j) {
        const double x = xs[(j - lo) * RKS + k];
        if (isfinite(x)) {   // pandas rolling: +-inf -> NaN (Window._prep_values)
            sm.add(x);
            ++c;
        }
    }
    out[((int64_t)p * nseg + ib) * kmax + k] = c >= minp ? sm.value() / (double)c : NAN;
    for (int i = ib + 1; i < ib + RPT && i < hi; ++i) {
        const double xi = xs[(i - lo) * RKS + k];
        if (isfinite(xi)) {
            sm.add(xi);
            ++c;
        }
        const int jo = i - window;   // leaves the window
        if (jo >= 0) {
            const double xo = xs[(jo - lo) * RKS + k];
            if (isfinite(xo)) {
                sm.add(-xo);
                --c;
            }
        }
        if (c == 0) sm.reset();
        out[((int64_t)p * nseg + i) * kmax + k] = c >= minp ? sm.value() / (double)c : NAN;
    }
}

// Sixteen lanes per (problem, fitted-month row), sixteen rows per workgroup: lane a owns
// regressor a (K <= 15), the quadratic forms c'Sxx c and c'Sxy are 16-lane sums.  Most rows
// of a gathered series belong to other ranks' months and only write the zero record.
//
// The zero record of another rank's month is -0.0, not +0.0: the SUM all-reduce that merges
// the ranks' records (fmcore.dist.combine_predictive) then returns the owner's value bit for
// bit, a signed zero included (v + (-0.0) == v for every v, -0.0 itself too; with +0.0
// fillers an owner's -0.0 would come back +0.0), in any summation order.
constexpr int PG = 16;
__global__ __launch_bounds__(TT) void predictive_kernel(const double* mom, int mom_stride,
                                                        int nseg, int nprob,
                                                        const int32_t* prob_k, const int32_t* idx,
                                                        const int32_t* count, const double* roll,
                                                        int pmax, int lag, int seg_lo, int seg_hi,
                                                        double* pred, uint32_t* pst) {
    const int p = blockIdx.y, lane = threadIdx.x % PG;
    const int i = blockIdx.x * (TT / PG) + threadIdx.x / PG;
    const bool row = i < nseg;
    const int ic = row ? i : 0;
    double* o = pred + ((int64_t)p * nseg + ic) * 4;
    const int cnt = count[p];
    const int s = ic < cnt ? idx[(int64_t)p * nseg + ic] : -1;
    const bool other = ic < cnt && (s < seg_lo || s >= seg_hi);   // another rank's month
    uint32_t st = 0;
    double slope = NAN, r2 = NAN, nn = NAN;
    const int K = prob_k[p];
    const bool own = row && !other && ic < cnt && ic >= lag;
    double tb = 0.0, ty = 0.0, syy = 0.0, n = 0.0;
    bool bad = false;
    if (own) {
        const double* c = roll + ((int64_t)p * nseg + (ic - lag)) * pmax;
        const double* mo = mom + ((int64_t)(s - seg_lo) * nprob + p) * mom_stride;
        const int K1 = K + 1;
        n = mo[0];
        bad = lane <= K && isnan(c[lane]);
        const double* S = mo + 1 + K1;
        if (lane < K) {
            double t = 0.0;
            for (int b = 0; b < K; ++b) t += S[lane * K1 + b] * c[1 + b];
            tb = c[1 + lane] * t;
            ty = c[1 + lane] * S[lane * K1 + K];
        }
        syy = S[K * K1 + K];
    }
    // 16-lane sums / any (every lane of the group takes part)
    int anybad = bad ? 1 : 0;
#pragma unroll
    for (int m = 8; m > 0; m >>= 1) {
        tb += __shfl_xor(tb, m, PG);
        ty += __shfl_xor(ty, m, PG);
        anybad |= __shfl_xor(anybad, m, PG);
    }
    if (own && !anybad && n >= 2.0) {
        slope = ty / tb;
        r2 = (ty * ty) / (tb * syy);
        nn = n;
        st = FM_ST_FITTED;
        if (!(tb > 0.0)) st |= FM_ST_CONST_COL;
    }
    if (row && lane == 0) {
        if (other) {   // -0.0 record for the sum-combine of sharded runs (exact, signs kept)
            o[0] = o[1] = o[2] = o[3] = -0.0;
            pst[(int64_t)p * nseg + ic] = 0;
        } else {
            o[0] = slope;
            o[1] = r2;
            o[2] = nn;
            o[3] = 0.0;
            pst[(int64_t)p * nseg + ic] = st;
        }
    }
}

// Wide problems (> 16 coefficients) or windows > 257 rows: one workgroup per (problem,
// coefficient, chunk of WRCH output rows), each output a direct sum over its window.
constexpr int WRCH = 1024;

__global__ __launch_bounds__(TT) void rolling_kernel_wide(const double* rec, int64_t r_seg,
                                                     int64_t r_prob, const int32_t* idx,
                                                     const int32_t* count, int nseg, int kmax,
                                                     int window, int minp, double* out) {
    __shared__ double xs[WRCH + RMAXW];
    const int p = blockIdx.y / kmax, k = blockIdx.y - (blockIdx.y / kmax) * kmax;
    const int c0 = blockIdx.x * WRCH;
    const int cnt = count[p];
    // rows past the fitted-month count have no month: NaN (never left uninitialised)
    const int cend = c0 + WRCH < nseg ? c0 + WRCH : nseg;
    for (int i = (c0 > cnt ? c0 : cnt) + threadIdx.x; i < cend; i += TT)
        out[((int64_t)p * nseg + i) * kmax + k] = NAN;
    if (c0 >= cnt) return;
    const int32_t* ix = idx + (int64_t)p * nseg;
    const int lo = c0 - window + 1 < 0 ? 0 : c0 - window + 1;
    const int hi = c0 + WRCH < cnt ? c0 + WRCH : cnt;
    for (int j = lo + threadIdx.x; j < hi; j += TT)
        xs[j - lo] = rec[(int64_t)ix[j] * r_seg + (int64_t)p * r_prob + k];
    __syncthreads();
    for (int i = c0 + threadIdx.x; i < hi; i += TT) {
        const int j0 = i - window + 1 < 0 ? 0 : i - window + 1;
        double sm = 0.0;
        int c = 0;
        for (int j = j0; j <= i; ++j) {
            const double x = xs[j - lo];
            if (isfinite(x)) {   // pandas rolling: +-inf -> NaN (Window._prep_values)
                sm += x;
                ++c;
            }
        }
        out[((int64_t)p * nseg + i) * kmax + k] = c >= minp ? sm / (double)c : NAN;
    }
}

// Wide problems (> 15 regressors): one wave per (problem, fitted-month row), lane a owns
// regressor a.
__global__ __launch_bounds__(WAVE) void predictive_kernel_wide(const double* mom, int mom_stride,
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
        // another rank's month (sharded runs): -0.0 record for the exact sum-combine
        if (lane < 4) o[lane] = -0.0;
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
    hipLaunchKernelGGL(compact_kernel, dim3((nseg + CB - 1) / CB > 0 ? (nseg + CB - 1) / CB : 1, nprob), dim3(TT), 0,
                       (hipStream_t)stream, status, s_seg, s_prob, nseg, idx, count);
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
    SumArgs a{rec, r_seg, r_prob, idx, count, nseg, kmax, nw_lags, nprob, mean, se, tstat, nobs, work};
    const int nchunk = (nseg + SCH - 1) / SCH;
    if (nseg >= SUM_CHUNKED && nw_lags <= SUM_MAXLAG) {
        hipStream_t st = (hipStream_t)stream;
        hipLaunchKernelGGL(summary_gather_kernel, dim3((nseg + GROWS - 1) / GROWS, nprob), dim3(TT), 0, st, a);
        hipLaunchKernelGGL(summary_part_kernel, dim3(nchunk, kmax, nprob), dim3(TT), 0, st, a);
        hipLaunchKernelGGL(summary_combine_kernel, dim3(kmax, nprob), dim3(WAVE), 0, st, a, nchunk);
    } else {
        hipLaunchKernelGGL(summary_kernel, dim3(kmax, nprob), dim3(TT), 0, (hipStream_t)stream, a);
    }
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
    if (kmax <= RKMAX && window <= RSPAN - RCH + 1) {
        dim3 grid((nseg + RCH - 1) / RCH, nprob);
        hipLaunchKernelGGL(rolling_kernel, grid, dim3(TT), 0, (hipStream_t)stream, rec, r_seg, r_prob,
                           idx, count, nseg, kmax, window, min_periods, out, 0, 0, 0, 0);
    } else {
        dim3 grid((nseg + WRCH - 1) / WRCH, nprob * kmax);
        hipLaunchKernelGGL(rolling_kernel_wide, grid, dim3(TT), 0, (hipStream_t)stream, rec, r_seg, r_prob,
                           idx, count, nseg, kmax, window, min_periods, out);
    }
    FM_CHECK_LAUNCH("fm_rolling_mean");
    return FM_OK;
}

extern "C" int fm_rolling_mean_own(const double* rec, int64_t r_seg, int64_t r_prob,
                                   const int32_t* idx, const int32_t* count, int32_t nseg,
                                   int32_t nprob, int32_t kmax, int32_t window, int32_t min_periods,
                                   int32_t seg_lo, int32_t seg_hi, int32_t lag, double* out,
                                   void* stream) {
    using namespace fm;
    FM_REQUIRE(rec && idx && count && out, "fm_rolling_mean_own: null pointer");
    FM_REQUIRE(window >= 1 && min_periods >= 0 && lag >= 0, "fm_rolling_mean_own: bad window / lag");
    FM_REQUIRE(kmax <= RKMAX && window <= RSPAN - RCH + 1,
               "fm_rolling_mean_own: kmax <= %d and window <= %d (the staged kernel)", RKMAX, RSPAN - RCH + 1);
    if (nprob == 0 || nseg == 0 || kmax == 0) return FM_OK;
    dim3 grid((nseg + RCH - 1) / RCH, nprob);
    hipLaunchKernelGGL(rolling_kernel, grid, dim3(TT), 0, (hipStream_t)stream, rec, r_seg, r_prob, idx, count,
                       nseg, kmax, window, min_periods, out, 1, seg_lo, seg_hi, lag);
    FM_CHECK_LAUNCH("fm_rolling_mean_own");
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
    if (pmax <= PG) {
        dim3 grid((nseg + TT / PG - 1) / (TT / PG), nprob);
        hipLaunchKernelGGL(predictive_kernel, grid, dim3(TT), 0, (hipStream_t)stream, moments,
                           mom_stride, nseg, nprob, prob_k, idx, count, rolling, pmax, lag, seg_lo,
                           seg_hi, pred, pred_status);
    } else {
        hipLaunchKernelGGL(predictive_kernel_wide, dim3(nseg, nprob), dim3(WAVE), 0, (hipStream_t)stream, moments,
                           mom_stride, nseg, nprob, prob_k, idx, count, rolling, pmax, lag, seg_lo,
                           seg_hi, pred, pred_status);
    }
    FM_CHECK_LAUNCH("fm_predictive");
    return FM_OK;
}

// ---------------------------------------------------------------------------------------
// fm_ts_fused: the whole time-series stage in one launch.  Grid (kmax + nchunk, nprob):
//   x <  kmax   summary workgroup of coefficient k: dropna, mean, Newey-West (fm_ts_summary)
//   x >= kmax   rolling workgroup of RROWS consecutive fitted-month rows: the rolling means
//               of every coefficient on those rows (fm_rolling_mean) and, from the rows'
//               `lag`-earlier rolling means, their predictive slopes (fm_predictive)
// Every workgroup first rebuilds its problem's fitted-month list (fm_ts_compact) in LDS --
// a few hundred status words, cheaper than a kernel boundary -- and works on LDS copies of
// the records it needs, so no phase waits on a dependent chain of L2 gathers.  Called on the
// predictive records (roll = pred = NULL) it gives their summary.
namespace fm {
namespace {

constexpr int FT = 256;
constexpr int FNW = FT / WAVE;
// rows per rolling workgroup (RROWS / 16 predictive rows per 16-lane group): the shortest
// chain per workgroup wins -- 16 rows 11.8 us, 32 rows 15.8 us, 64 rows 19.4 us for the bench's
// 600 x 11 series (profiles/r05/v9_kbench_ts_rrows.log): more workgroups each stage more window
// rows, but a workgroup's serial work (prefix sums, rolling means, predictive rows) shrinks
#ifndef FM_TS_RROWS
#define FM_TS_RROWS 16
#endif
constexpr int RROWS = FM_TS_RROWS;
static_assert(RROWS % 16 == 0, "fm_ts_fused: RROWS is a multiple of the 16 row groups");
constexpr int MAXL = 8;      // Newey-West lags accumulated in one sweep

__host__ __device__ __forceinline__ size_t ts_ix_bytes(int T) { return ((size_t)T * 4 + 15) & ~(size_t)15; }

// fitted months of problem p, ascending, into ixs; returns their count (block-uniform)
__device__ __forceinline__ int ts_compact_lds(const fm_ts_args& a, int p, int* ixs, int* wtot) {
    const int tid = threadIdx.x, lane = tid & (WAVE - 1), w = tid / WAVE;
    int base = 0;
    constexpr int PF = 8;   // status words per thread loaded before the first scan (in flight together)
    for (int sb = 0; sb < a.nseg; sb += PF * FT) {
    uint32_t sw[PF];
#pragma unroll
    for (int k = 0; k < PF; ++k) {   // clamped, unconditional loads
        const int s = sb + k * FT + tid;
        const int sc = s < a.nseg ? s : a.nseg - 1;
        sw[k] = a.status[(int64_t)sc * a.s_seg + (int64_t)p * a.s_prob];
    }
#pragma unroll
    for (int k = 0; k < PF; ++k) {
        const int s0 = sb + k * FT;
        if (s0 >= a.nseg) break;   // block-uniform
        const int s = s0 + tid;
        const bool f = s < a.nseg && (sw[k] & FM_ST_FITTED);
        const uint64_t bm = __ballot(f);
        if (lane == 0) wtot[w] = (int)__popcll(bm);
        __syncthreads();
        int off = 0, tot = 0;
#pragma unroll
        for (int q = 0; q < FNW; ++q) {
            const int c = wtot[q];
            off += q < w ? c : 0;
            tot += c;
        }
        if (f) ixs[base + off + mask_rank(bm)] = s;
        base += tot;
        __syncthreads();
    }
    }
    return base;
}

template <int ML>   // the lags accumulated in the one sweep (the run's NW lags, or MAXL)
__device__ __forceinline__ void ts_summary_wg_t(const fm_ts_args& a, int p, int k, const int* ixs, int cnt, double* xs,
                              int* wtot, double* dred) {
    const int tid = threadIdx.x, lane = tid & (WAVE - 1), w = tid / WAVE;
    const double* rk = a.rec + (int64_t)p * a.r_prob + k;
    for (int i0 = 0; i0 < cnt; i0 += 8 * FT) {   // 8 gathers per thread in flight together
        double v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int i = i0 + k * FT + tid;
            v[k] = rk[(int64_t)ixs[i < cnt ? i : cnt - 1] * a.r_seg];
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int i = i0 + k * FT + tid;
            if (i < cnt) xs[i] = v[k];
        }
    }
    __syncthreads();
    FM_PROBE_AT(ts, 2);
    // dropna in place, month order kept (each pass reads its span before any write lands)
    int n = 0;
    for (int i0 = 0; i0 < cnt; i0 += FT) {
        const int i = i0 + tid;
        const double x = i < cnt ? xs[i] : NAN;
        const bool v = !isnan(x);
        const uint64_t bm = __ballot(v);
        if (lane == 0) wtot[w] = (int)__popcll(bm);
        __syncthreads();
        int off = 0, tot = 0;
#pragma unroll
        for (int q = 0; q < FNW; ++q) {
            const int c = wtot[q];
            off += q < w ? c : 0;
            tot += c;
        }
        if (v) xs[n + off + mask_rank(bm)] = x;
        n += tot;
        __syncthreads();
    }
    FM_PROBE_AT(ts, 3);
    double sum = 0.0;
    for (int i = tid; i < n; i += FT) sum += xs[i];
    sum = block_sum<FNW>(sum, dred);
    const double mu = n > 0 ? sum / (double)n : NAN;
    // gamma_0 .. gamma_min(lags, ML) in one sweep, one reduction
    const int lags = a.nw_lags < ML ? a.nw_lags : ML;
    double gl[ML + 1];
#pragma unroll
    for (int L = 0; L <= ML; ++L) gl[L] = 0.0;
    for (int i = tid; i < n; i += FT) {
        const double ui = xs[i] - mu;
#pragma unroll
        for (int L = 0; L <= ML; ++L)
            if (L <= lags && i >= L) gl[L] += ui * (xs[i - L] - mu);
    }
    __syncthreads();   // block_sum's readers are done with dred
#pragma unroll
    for (int L = 0; L <= ML; ++L) {
        const double v = wave_sum(gl[L]);
        if (lane == 0) dred[L * FNW + w] = v;
    }
    __syncthreads();
#pragma unroll
    for (int L = 0; L <= ML; ++L) {
        double t = 0.0;
#pragma unroll
        for (int q = 0; q < FNW; ++q) t += dred[L * FNW + q];
        gl[L] = t;
    }
    __syncthreads();
    double acc = 0.0;
    for (int L = 1; L <= a.nw_lags; ++L) {
        const double wgt = 1.0 - ((double)L / (double)n);
        if (wgt < 0.0) break;
        double gk = 0.0;
        if (L <= ML) {
#pragma unroll
            for (int q = 1; q <= ML; ++q)
                if (q == L) gk = gl[q];
        } else {
            for (int i = L + tid; i < n; i += FT) gk += (xs[i] - mu) * (xs[i - L] - mu);
            gk = block_sum<FNW>(gk, dred);
        }
        acc += wgt * gk;
    }
    FM_PROBE_AT(ts, 4);
    if (tid == 0) {
        const int64_t o = (int64_t)p * a.kmax + k;
        double se = NAN;
        if (n >= 2) se = sqrt((gl[0] + 2.0 * acc) / ((double)n * (double)n));
        a.mean[o] = mu;
        a.se[o] = se;
        a.tstat[o] = mu / se;
        a.nobs[o] = n;
    }
}

// the summary, specialised for the reference's 4 Newey-West lags (the sweep and the reduction
// carry gamma_0..4 instead of 0..8; identical bits: the extra terms were never accumulated)
__device__ void ts_summary_wg(const fm_ts_args& a, int p, int k, const int* ixs, int cnt, double* xs,
                              int* wtot, double* dred) {
    if (a.nw_lags == 4) ts_summary_wg_t<4>(a, p, k, ixs, cnt, xs, wtot, dred);
    else ts_summary_wg_t<MAXL>(a, p, k, ixs, cnt, xs, wtot, dred);
}

__device__ void ts_rolling_wg(const fm_ts_args& a, int p, int chunk, const int* ixs, int cnt,
                              double* lds_d) {
    const int tid = threadIdx.x;
    const int r0 = chunk * RROWS;
    const int T = a.nseg, PM = a.pmax;
    const bool predictive = a.pred != nullptr;
    if (a.roll_own && r0 < cnt) {
        // a sharded rank rolls only the rows its predictive records read: [first fitted row of
        // its months - lag, first fitted row past them)
        auto lb = [&](int v) {
            int lo = 0, hi = cnt;
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (ixs[mid] < v) lo = mid + 1;
                else hi = mid;
            }
            return lo;
        };
        int ra = lb(a.seg_lo) - (predictive ? a.lag : 0);
        ra = ra < 0 ? 0 : ra;
        const int rb = lb(a.seg_hi);
        if (r0 + RROWS <= ra || r0 >= rb) {   // block-uniform: none of this chunk's rows needed
            if (predictive) {
                // the chunk's predictive records are still this rank's to write: -0.0 records of
                // other ranks' months, NaN past the fitted count (status 0), as below
                const int e1 = r0 + RROWS < T ? r0 + RROWS : T;
                for (int i = r0 + tid; i < e1; i += FT) {
                    double* o = a.pred + ((int64_t)p * T + i) * 4;
                    const bool row = i < cnt;
                    o[0] = o[1] = o[2] = row ? -0.0 : NAN;
                    o[3] = row ? -0.0 : 0.0;
                    a.pred_status[(int64_t)p * T + i] = 0;
                }
            }
            return;
        }
    }
    {
        // rows of this chunk past the fitted-month count hold no month: NaN rolling means,
        // NaN predictive record, status 0 (the buffers are never left uninitialised)
        const int e0 = r0 > cnt ? r0 : cnt, e1 = r0 + RROWS < T ? r0 + RROWS : T;
        for (int e = tid; e < (e1 - e0) * PM; e += FT) a.roll[((int64_t)p * T + e0) * PM + e] = NAN;
        if (predictive)
            for (int i = e0 + tid; i < e1; i += FT) {
                double* o = a.pred + ((int64_t)p * T + i) * 4;
                o[0] = o[1] = o[2] = NAN;
                o[3] = 0.0;
                a.pred_status[(int64_t)p * T + i] = 0;
            }
    }
    if (r0 >= cnt) return;                               // block-uniform
    const int r1 = r0 + RROWS < cnt ? r0 + RROWS : cnt;
    // Predictive slopes, K < 16 (block-uniform): the month moments of ALL of a 16-lane group's
    // rows (n, Syy and this lane's S column, clamped to a valid row) are loaded here, before
    // the window rows are staged, so the round trip overlaps the staging and the rolling
    // sums (the registers cost no occupancy: the workgroup's LDS holds it to 2 per CU).  A
    // shard with no months of its own has no moments rows at all: nothing to preload.
    const int K = predictive ? a.prob_k[p] : 0, K1 = K + 1;
    const int g = tid >> 4, b = tid & 15;
    constexpr int NIT = RROWS / (FT / 16);   // rows per 16-lane group
    double scq[NIT][15], n0q[NIT], syq[NIT];
    if (predictive && K < 16 && a.seg_hi > a.seg_lo) {
        const int bc = b <= K ? b : 0;
#pragma unroll
        for (int it = 0; it < NIT; ++it) {
            const int i = r0 + g + it * (FT / 16);
            const int s = i < r1 ? ixs[i] : -1;
            const bool have = i < r1 && s >= a.seg_lo && s < a.seg_hi && i >= a.lag;
            const int sr = have ? s - a.seg_lo : 0;
            const double* mo = a.moments + ((int64_t)sr * a.nprob + p) * a.mom_stride;
            const double* S = mo + 1 + K1;
#pragma unroll
            for (int r = 0; r < 15; ++r) scq[it][r] = S[(r < K ? r : 0) * K1 + bc];
            n0q[it] = mo[0];
            syq[it] = S[K * K1 + K];
        }
    }
    const int q0 = predictive ? (r0 - a.lag > 0 ? r0 - a.lag : 0) : r0;   // rows rolled here
    const int j0 = q0 - a.window + 1 > 0 ? q0 - a.window + 1 : 0;          // rows read
    const int nsrc = r1 - j0, nq = r1 - q0;
    double* xs = lds_d;                  // [nsrc][PM]
    double* rl = lds_d + nsrc * PM;      // [nq][PM]
    const double* rp = a.rec + (int64_t)p * a.r_prob;
    {
        // SB gathers per thread in flight together (clamped, unconditional loads; stores
        // after): a load -> wait -> store loop pays one L2 round trip per element
        constexpr int SB = 8;
        const int ne = nsrc * PM;
        for (int e0 = 0; e0 < ne; e0 += SB * FT) {
            double v[SB];
#pragma unroll
            for (int q = 0; q < SB; ++q) {
                const int e = e0 + q * FT + tid;
                const int ec = e < ne ? e : ne - 1;
                const int j = ec / PM, k = ec - j * PM;
                v[q] = rp[(int64_t)ixs[j0 + j] * a.r_seg + k];
            }
#pragma unroll
            for (int q = 0; q < SB; ++q) {
                const int e = e0 + q * FT + tid;
                if (e < ne) xs[e] = v[q];
            }
        }
    }
    __syncthreads();
    FM_PROBE_AT(ts, 2);
    // per-column inclusive prefix sums of the finite values and their counts over the staged
    // rows (each output is then a difference of two prefixes: no serial window sums).  A
    // column's rows are split over 16 threads: local scans, then the 16 block totals.  The
    // prefixes are double-double (high part in ps, low part in place of the staged value):
    // a prefix difference then loses nothing to an outlier that entered before both ends,
    // where a plain prefix would leave ulp(outlier) in every later window.
    double* ps = rl + nq * PM;                        // [nsrc][PM] prefix sums (high part)
    double* pl = xs;                                  // [nsrc][PM] low part (overwrites xs)
    int* pc = reinterpret_cast<int*>(ps + nsrc * PM);  // [nsrc][PM] prefix counts
    for (int kb = 0; kb < PM; kb += 16) {
        const int k = kb + (tid >> 4), part = tid & 15;   // 16 columns x 16 parts at a time
        const int per = (nsrc + 15) / 16;
        const int a0 = part * per, a1 = a0 + per < nsrc ? a0 + per : nsrc;
        CSum sm;
        int cn = 0;
        if (k < PM) {
            for (int j = a0; j < a1; ++j) {
                const double x = xs[j * PM + k];
                if (isfinite(x)) {   // pandas rolling: +-inf -> NaN (Window._prep_values)
                    sm.add(x);
                    ++cn;
                }
                ps[j * PM + k] = sm.s;
                pl[j * PM + k] = sm.c;
                pc[j * PM + k] = cn;
            }
        }
        // exclusive prefix of the 16 part totals (lanes of one 16-lane row group)
        CSum bs = sm;
        int bc = cn;
        static_for<0, 4>([&](auto oc) {
            constexpr int o = 1 << decltype(oc)::value;
            const double yh = row_shr<o>(bs.s);
            const double yl = row_shr<o>(bs.c);
            const int yc = row_shr<o>(bc);
            if (part >= o) {
                bs.add(yh);
                bs.c += yl;
                bc += yc;
            }
        });
        bs.add(-sm.s);
        bs.c -= sm.c;
        bc -= cn;
        if (k < PM)
            for (int j = a0; j < a1; ++j) {
                double e;
                const double h = two_sum(ps[j * PM + k], bs.s, &e);
                ps[j * PM + k] = h;
                pl[j * PM + k] += bs.c + e;
                pc[j * PM + k] += bc;
            }
    }
    __syncthreads();
    FM_PROBE_AT(ts, 3);
    for (int e = tid; e < nq * PM; e += FT) {
        const int q = e / PM, k = e - q * PM, i = q0 + q;
        const int jlo = i - a.window;                 // prefix just before the window
        double sm = ps[(i - j0) * PM + k];
        double sl = pl[(i - j0) * PM + k];
        int cn = pc[(i - j0) * PM + k];
        if (jlo >= j0) {
            sm -= ps[(jlo - j0) * PM + k];
            sl -= pl[(jlo - j0) * PM + k];
            cn -= pc[(jlo - j0) * PM + k];
        }
        sm += sl;
        const double m = cn >= a.min_periods && cn > 0 ? sm / (double)cn : NAN;
        rl[q * PM + k] = m;
        if (i >= r0) a.roll[((int64_t)p * T + i) * PM + k] = m;
    }
    if (!predictive) return;
    __syncthreads();
    FM_PROBE_AT(ts, 4);
    // predictive slopes: a 16-lane group per row, lane b owns column b of each S row
    FM_PROBE_AT(ts, 5);
#pragma unroll
    for (int it = 0; it < NIT; ++it) {     // uniform trip count (shuffles)
        const int i = r0 + g + it * (FT / 16);
        const bool row = i < r1;
        const int s = row ? ixs[i] : -1;
        const bool mine = row && s >= a.seg_lo && s < a.seg_hi;
        bool ok = false;
        double n = NAN, tb = 0.0, ty = 0.0, syy = NAN;
        if (K < 16) {
            if (mine && i >= a.lag) {
                const double* c = rl + (i - a.lag - q0) * PM;
                bool bad = false;
#pragma unroll
                for (int q = 0; q < 16; ++q)   // a fixed trip count: the LDS reads issue together
                    if (q <= K) bad |= isnan(c[q]);
                n = n0q[it];
                ok = !bad && n >= 2.0;
                if (ok) {
                    syy = syq[it];
                    const double cb = b < K ? c[1 + b] : 0.0;
#pragma unroll
                    for (int r = 0; r < 15; ++r) {
                        if (r < K) {
                            const double v = scq[it][r] * c[1 + r];
                            if (b < K) tb += v * cb;
                            else if (b == K) ty += v;
                        }
                    }
                }
            }
        } else if (mine && i >= a.lag) {
            const double* c = rl + (i - a.lag - q0) * PM;
            bool bad = false;
            for (int q = 0; q <= K; ++q) bad |= isnan(c[q]);
            const double* mo = a.moments + ((int64_t)(s - a.seg_lo) * a.nprob + p) * a.mom_stride;
            n = mo[0];
            ok = !bad && n >= 2.0;
            if (ok) {
                const double* S = mo + 1 + K1;
                syy = S[K * K1 + K];
                for (int bb = b; bb <= K; bb += 16) {
                    const double cb = bb < K ? c[1 + bb] : 0.0;
#pragma unroll 4
                    for (int r = 0; r < K; ++r) {
                        const double v = S[r * K1 + bb] * c[1 + r];
                        if (bb < K) tb += v * cb;
                        else ty += v;
                    }
                }
            }
        }
        tb = row16_sum(tb);
        ty = row16_sum(ty);
        if (row && b == 0) {
            double* o = a.pred + ((int64_t)p * T + i) * 4;
            uint32_t st = 0;
            double slope = NAN, r2 = NAN, nn = NAN;
            if (!mine) {
                // another rank's month (sharded runs): -0.0 record for the exact sum-combine
                slope = r2 = nn = -0.0;
            } else if (ok) {
                slope = ty / tb;
                r2 = (ty * ty) / (tb * syy);
                nn = n;
                st = FM_ST_FITTED;
                if (!(tb > 0.0)) st |= FM_ST_CONST_COL;
            }
            o[0] = slope;
            o[1] = r2;
            o[2] = nn;
            o[3] = mine ? 0.0 : -0.0;
            a.pred_status[(int64_t)p * T + i] = st;
        }
    }
}

__global__ __launch_bounds__(FT) void ts_fused_kernel(fm_ts_args a) {
    extern __shared__ double lds[];
    __shared__ int wtot[FNW];
    __shared__ double dred[(MAXL + 1) * FNW];
    const int p = blockIdx.y, bx = blockIdx.x;
    int* ixs = reinterpret_cast<int*>(lds);
    double* lds_d = lds + ts_ix_bytes(a.nseg) / 8;
    FM_PROBE_AT(ts, 0);
    const int cnt = ts_compact_lds(a, p, ixs, wtot);
    FM_PROBE_AT(ts, 1);
    if (bx == 0) {
        for (int i = threadIdx.x; i < cnt; i += FT) a.idx[(int64_t)p * a.nseg + i] = ixs[i];
        if (threadIdx.x == 0) a.count[p] = cnt;
    }
    if (bx < a.kmax) {
        if (a.sum_p_hi > 0 && (p < a.sum_p_lo || p >= a.sum_p_hi)) {   // block-uniform
            // another rank's problem (sharded runs): -0.0 / 0 for the exact SUM-combine
            if (threadIdx.x == 0) {
                const int64_t o = (int64_t)p * a.kmax + bx;
                a.mean[o] = a.se[o] = a.tstat[o] = -0.0;
                a.nobs[o] = 0;
            }
        } else {
            ts_summary_wg(a, p, bx, ixs, cnt, lds_d, wtot, dred);
        }
    } else {
        ts_rolling_wg(a, p, bx - a.kmax, ixs, cnt, lds_d);
        FM_PROBE_AT(ts, 6);
    }
    FM_PROBE_AT(ts, 7);
}

}  // namespace
}  // namespace fm

extern "C" size_t fm_ts_fused_lds_bytes(int32_t nseg, int32_t pmax, int32_t window, int32_t lag,
                                         int32_t rolling, int32_t predictive) {
    using namespace fm;
    size_t d = (size_t)nseg * 8;
    if (rolling) {
        const size_t l = predictive ? (size_t)lag : 0;
        const size_t nsrc = RROWS + l + (size_t)window - 1;
        // staged rows, rolling means, prefix sums (8 B) and prefix counts (4 B)
        const size_t r = (size_t)pmax * (8 * nsrc + 8 * (RROWS + l) + 12 * nsrc);
        d = d > r ? d : r;
    }
    return ts_ix_bytes(nseg) + d;
}

extern "C" int fm_ts_fused(const fm_ts_args* args, void* stream) {
    using namespace fm;
    FM_REQUIRE(args != nullptr, "fm_ts_fused: null args");
    const fm_ts_args& a = *args;
    FM_REQUIRE(a.rec && a.status && a.idx && a.count && a.mean && a.se && a.tstat && a.nobs,
               "fm_ts_fused: null pointer");
    FM_REQUIRE(a.nw_lags >= 0, "fm_ts_fused: nw_lags < 0");
    FM_REQUIRE(a.roll == nullptr || (a.window >= 1 && a.min_periods >= 0 && a.pmax >= 1),
               "fm_ts_fused: bad rolling window");
    FM_REQUIRE(a.pred == nullptr || (a.roll && a.moments && a.prob_k && a.pred_status && a.lag >= 1),
               "fm_ts_fused: the predictive stage needs roll, moments, prob_k, pst and lag >= 1");
    if (a.nprob == 0 || a.nseg == 0) return FM_OK;
    const size_t lds = fm_ts_fused_lds_bytes(a.nseg, a.pmax, a.window, a.lag, a.roll != nullptr,
                                             a.pred != nullptr);
    FM_REQUIRE(lds <= FM_TS_FUSED_MAX_LDS,
               "fm_ts_fused: series too long for LDS staging (use the per-stage entry points)");
    if (lds > 64 * 1024) {   // beyond the default dynamic-LDS limit: opt in (once)
        static bool attr_set = false;
        if (!attr_set) {
            FM_REQUIRE(hipFuncSetAttribute((const void*)ts_fused_kernel,
                                           hipFuncAttributeMaxDynamicSharedMemorySize,
                                           FM_TS_FUSED_MAX_LDS) == hipSuccess,
                       "fm_ts_fused: cannot raise the dynamic LDS limit");
            attr_set = true;
        }
    }
    const int nchunk = a.roll ? (a.nseg + RROWS - 1) / RROWS : 0;
    hipLaunchKernelGGL(ts_fused_kernel, dim3(a.kmax + nchunk, a.nprob), dim3(FT), lds, (hipStream_t)stream, a);
    FM_CHECK_LAUNCH("fm_ts_fused");
    return FM_OK;
}

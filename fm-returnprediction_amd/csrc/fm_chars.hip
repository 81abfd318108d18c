// Firm-axis characteristic construction: the per-firm lags,
// rolling windows and log / ratio arithmetic that get_factors runs before winsorize
// (reference src/calc_Lewellen_2014.py:531-575), as two HBM-streaming kernels over a
// FIRM-major panel (rows grouped by permno, each group in frame order).
//
//   firm_chars_kernel  <- calc_log_size .. calc_sales_price (:137-341): one workgroup per
//                         256-row tile, one row per thread.  The 36-row halo of firm ids and
//                         the return-derived window inputs (1 + retx, log(1 + retx), dvc)
//                         are staged in LDS once per tile; lag-k reads of the other fields
//                         are coalesced global loads that hit L2 (the previous tile's rows).
//                         Because groups are contiguous, "row i-k belongs to row i's firm" is
//                         one compare: ids[i-k] == ids[i].
//   rolling_std_kernel <- calc_std_12's 252-day rolling std (:448-456): each thread owns 8
//                         consecutive rows of a 2,048-row tile; firm starts are a ballot
//                         bitmask; the first window sums per-8-row block states (count, mean,
//                         M2) precomputed in LDS for the tile and its halo, as shifted sums
//                         about a block mean near the window end; the next 7 rows slide those
//                         sums (adds only, one division per output).  pandas slides
//                         one Welford/Kahan state along the whole group; both agree to
//                         rounding (tests: 1e-9 series-RMS tolerance).
#include <math.h>

#include "fm_common.h"

namespace fm {
namespace {

constexpr int CT = 256;   // rows per firm_chars tile (= threads)
constexpr int CH = 36;    // longest lag (calc_log_issues_36 / calc_log_return_13_36)

__device__ __forceinline__ double nan_if_inf(double x) { return isinf(x) ? (double)NAN : x; }

__global__ __launch_bounds__(CT) void firm_chars_kernel(fm_chars_args a, int need_ret, int need_dvc) {
    __shared__ int64_t sid[CT + CH];
    __shared__ double opr[CT + CH];   // 1 + retx, +-inf -> NaN (rolling input, :178-186)
    __shared__ double lr[CT + CH];    // log(1 + retx), +-inf -> NaN (:298, :302-306)
    __shared__ double dv[CT + CH];    // dvc, +-inf -> NaN (:273-278)
    const int64_t n = a.n;
    const int64_t b = (int64_t)blockIdx.x * CT;
    const int64_t i = b + threadIdx.x;
    const bool live = i < n;
    const int64_t ic = live ? i : n - 1;   // clamped row: every load below is unconditional
    double* const* o = a.out;
    // ---- this row's global loads, issued before the tile barrier so they fly while the
    // halo is staged (each a coalesced read; lags hit L2: the previous rows of this tile or
    // the previous tile).  Pointer tests are kernel-argument (scalar) branches.
    auto ld = [&](int f, int k) {
        const double* p = a.field[f];
        return p[ic - k >= 0 ? ic - k : 0];
    };
    const bool need_me1 = o[FM_CHAR_LOG_SIZE] || o[FM_CHAR_LOG_BM] || o[FM_CHAR_DEBT_PRICE] ||
                          o[FM_CHAR_SALES_PRICE];
    const bool need_sh = o[FM_CHAR_LOG_ISSUES_12] || o[FM_CHAR_LOG_ISSUES_36];
    const double me1 = need_me1 ? ld(FM_FIELD_ME, 1) : 0.0;
    const double be1 = o[FM_CHAR_LOG_BM] ? ld(FM_FIELD_BE, 1) : 0.0;
    const double acc = o[FM_CHAR_ACCRUALS_FINAL] ? ld(FM_FIELD_ACCRUALS, 0) : 0.0;
    const double dep = o[FM_CHAR_ACCRUALS_FINAL] ? ld(FM_FIELD_DEPRECIATION, 0) : 0.0;
    const double ern = o[FM_CHAR_ROA] ? ld(FM_FIELD_EARNINGS, 0) : 0.0;
    const bool need_as = o[FM_CHAR_ROA] || o[FM_CHAR_LOG_ASSETS_GROWTH];
    const double as0 = need_as ? ld(FM_FIELD_ASSETS, 0) : 0.0;
    const double as12 = o[FM_CHAR_LOG_ASSETS_GROWTH] ? ld(FM_FIELD_ASSETS, 12) : 0.0;
    const double prc1 = o[FM_CHAR_DY] ? ld(FM_FIELD_PRC, 1) : 0.0;
    const double sh1 = need_sh ? ld(FM_FIELD_SHROUT, 1) : 0.0;
    const double sh12 = o[FM_CHAR_LOG_ISSUES_12] ? ld(FM_FIELD_SHROUT, 12) : 0.0;
    const double sh36 = o[FM_CHAR_LOG_ISSUES_36] ? ld(FM_FIELD_SHROUT, 36) : 0.0;
    const double td = o[FM_CHAR_DEBT_PRICE] ? ld(FM_FIELD_TOTAL_DEBT, 0) : 0.0;
    const double sl = o[FM_CHAR_SALES_PRICE] ? ld(FM_FIELD_SALES, 0) : 0.0;
    const double* retx = a.field[FM_FIELD_RETX];
    const double* dvc = a.field[FM_FIELD_DVC];
    for (int j = threadIdx.x; j < CT + CH; j += CT) {
        const int64_t r = b - CH + j;
        const bool in = r >= 0 && r < n;
        const int64_t rc = r < 0 ? 0 : (r < n ? r : n - 1);
        sid[j] = in ? a.ids[rc] : 0;
        if (need_ret) {
            const double x = retx[rc];
            const double op = 1.0 + (in ? x : (double)NAN);
            opr[j] = nan_if_inf(op);
            lr[j] = nan_if_inf(log(op));
        }
        if (need_dvc) {
            const double v = dvc[rc];
            dv[j] = in ? nan_if_inf(v) : (double)NAN;
        }
    }
    __syncthreads();
    if (!live) return;
    const int li = threadIdx.x + CH;
    const int64_t id = sid[li];
    auto same = [&](int k) { return i - k >= 0 && sid[li - k] == id; };
    const double nan = NAN;
    const double m1 = same(1) ? me1 : nan;
    if (o[FM_CHAR_LOG_SIZE]) o[FM_CHAR_LOG_SIZE][i] = log(m1);
    if (o[FM_CHAR_LOG_BM]) o[FM_CHAR_LOG_BM][i] = log(same(1) ? be1 : nan) - log(m1);
    if (o[FM_CHAR_RETURN_12_2]) {
        // rolling(11, min_periods=11).apply(np.prod) of the shift(2) column: rows t-12..t-2,
        // oldest first; any NaN in the window -> NaN (the product propagates it)
        double p = opr[li - 12];
#pragma unroll
        for (int k = 11; k >= 2; --k) p *= opr[li - k];
        o[FM_CHAR_RETURN_12_2][i] = same(12) ? p - 1.0 : nan;
    }
    if (o[FM_CHAR_ACCRUALS_FINAL]) o[FM_CHAR_ACCRUALS_FINAL][i] = acc - dep;
    if (o[FM_CHAR_ROA]) o[FM_CHAR_ROA][i] = ern / as0;
    if (o[FM_CHAR_LOG_ASSETS_GROWTH]) o[FM_CHAR_LOG_ASSETS_GROWTH][i] = log(as0 / (same(12) ? as12 : nan));
    if (o[FM_CHAR_DY]) {
        // rolling(12, min_periods=1).sum(): the observations among the firm's last 12 rows
        double sum = 0.0;
        int cnt = 0;
#pragma unroll
        for (int k = 11; k >= 0; --k) {
            const double v = dv[li - k];
            const bool ok = same(k) && !isnan(v);
            sum += ok ? v : 0.0;
            cnt += ok ? 1 : 0;
        }
        o[FM_CHAR_DY][i] = (cnt > 0 ? sum : nan) / (same(1) ? prc1 : nan);
    }
    if (o[FM_CHAR_LOG_RETURN_13_36]) {
        // rolling(24, min_periods=24).sum() of the shift(13) column: all 24 rows t-36..t-13
        double sum = 0.0;
#pragma unroll
        for (int k = 36; k >= 13; --k) sum += lr[li - k];
        o[FM_CHAR_LOG_RETURN_13_36][i] = same(36) ? sum : nan;
    }
    if (need_sh) {
        const double l1 = log(same(1) ? sh1 : nan);
        if (o[FM_CHAR_LOG_ISSUES_12]) o[FM_CHAR_LOG_ISSUES_12][i] = l1 - log(same(12) ? sh12 : nan);
        if (o[FM_CHAR_LOG_ISSUES_36]) o[FM_CHAR_LOG_ISSUES_36][i] = l1 - log(same(36) ? sh36 : nan);
    }
    if (o[FM_CHAR_DEBT_PRICE]) o[FM_CHAR_DEBT_PRICE][i] = td / m1;
    if (o[FM_CHAR_SALES_PRICE]) o[FM_CHAR_SALES_PRICE][i] = sl / m1;
}

// ---- rolling std --------------------------------------------------------------------------
// tile shape (timing builds may override): 256 x 8 measured best -- 512 x 8 0.116, 256 x 16
// 0.119, 512 x 4 0.179, 1024 x 4 0.205 vs 0.111 ms (profiles/r04/v11_stdbench_tile_sweep.log)
#ifndef FM_STD_ABL
#define FM_STD_ABL 0   // timing ablations only (wrong output): 1 no division / sqrt, 2 no first-window block sum, 3 staging + block stats only
#endif
#ifndef FM_STD_T
#define FM_STD_T 256
#endif
#ifndef FM_STD_R
#define FM_STD_R 8
#endif
constexpr int ST_T = FM_STD_T;       // threads
constexpr int ST_R = FM_STD_R;       // consecutive rows per thread
constexpr int ST_ROWS = ST_T * ST_R; // rows per tile
constexpr int ST_HA = 128;           // halo rows are loaded from a 128-row aligned start
#ifndef FM_STD_LP
#define FM_STD_LP 2                  // load batches per thread in flight: 2 -> 74 VGPRs, 0.1034 ms;
#endif                               // 3 -> 74, 0.1064; 4 -> 88, 0.1116 (profiles/r05/v4_stdbench_lp.log)

// LDS slot of halo element e: one pad slot per ST_R (the lanes of a wave read elements
// ST_R apart; stride ST_R + 1 doubles puts 32 lanes on distinct bank pairs)
__host__ __device__ __forceinline__ int spad(int e) { return e + e / ST_R; }
// halo rows staged before the tile: the window's W - 1 rows rounded up to ST_HA, so every
// wave loads 128 consecutive rows as 64 aligned 16-byte pairs
__host__ __device__ __forceinline__ int st_halo(int W) { return ((W - 1 + ST_HA - 1) / ST_HA) * ST_HA; }

// count / mean / M2 of the non-NaN observations of halo rows [a, b): two passes, no division
// per observation
struct RunStats {
    int n;
    double mean;
    double m2;
};

__device__ __forceinline__ RunStats range_stats(const double* xs, int a, int b) {
    // b - a <= ST_R always (a block, a head range or one row): a fixed, unrolled trip count
    // with masked lanes lets the LDS reads issue together
    double v[ST_R];
    int c = 0;
    double s1 = 0.0;
#pragma unroll
    for (int k = 0; k < ST_R; ++k) {
        const bool in = a + k < b;
        v[k] = in ? xs[spad(in ? a + k : a)] : (double)NAN;
        const bool ok = !isnan(v[k]);
        s1 += ok ? v[k] : 0.0;
        c += ok ? 1 : 0;
    }
    const double mean = c > 0 ? s1 / (double)c : 0.0;
    double m2 = 0.0;
#pragma unroll
    for (int k = 0; k < ST_R; ++k) {
        const double d = isnan(v[k]) ? 0.0 : v[k] - mean;
        m2 += d * d;
    }
    return RunStats{c, mean, m2};
}

// bits 0..31 of x spread to the even bit positions of a 64-bit word (Morton interleave)
__device__ __forceinline__ uint64_t spread_bits(uint32_t x32) {
    uint64_t x = x32;
    x = (x | (x << 16)) & 0x0000FFFF0000FFFFull;
    x = (x | (x << 8)) & 0x00FF00FF00FF00FFull;
    x = (x | (x << 4)) & 0x0F0F0F0F0F0F0F0Full;
    x = (x | (x << 2)) & 0x3333333333333333ull;
    x = (x | (x << 1)) & 0x5555555555555555ull;
    return x;
}

// 64-bit lane value of lane - 1 (DPP wave_shr:1); lane 0 gets `first`
__device__ __forceinline__ int64_t lane_prev_i64(int64_t v, int64_t first) {
    const uint64_t u = (uint64_t)v, f = (uint64_t)first;
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)f, (int)(uint32_t)u, 0x138, 0xF, 0xF, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)(f >> 32), (int)(uint32_t)(u >> 32), 0x138,
                                                               0xF, 0xF, false);
    return (int64_t)(((uint64_t)hi << 32) | lo);
}

__global__ __launch_bounds__(ST_T) void rolling_std_kernel(const int64_t* __restrict__ ids,
                                                           const double* __restrict__ x, int64_t n,
                                                           int W, int minp, double scale,
                                                           double* __restrict__ out) {
    extern __shared__ double sm[];
    const int H = W - 1;          // rows before a row that its window holds
    const int HP = st_halo(W);    // halo rows staged (>= H, 128-aligned)
    const int E = ST_ROWS + HP;   // staged rows (a multiple of 128)
    double* xs = sm;
    // firm starts as a bit per staged row (one wave ballot pair per 128 rows) instead of an
    // int64 id per row: 1 KB instead of 37 KB of LDS, so several workgroups share a CU
    uint64_t* fb = (uint64_t*)(sm + spad(E) + 1);
    const int nw = E / 64;
    const int64_t b = (int64_t)blockIdx.x * ST_ROWS;
    const int lane = (int)threadIdx.x & 63;
    // Loads: lane l of a wave takes staged rows 2q, 2q + 1 (q = wave pair index) as ONE
    // 16-byte load of x and one of ids (the rows' start is 128-aligned, hence even); the id
    // of the row before the pair is the previous lane's second id (DPP wave shift), for
    // lane 0 one scalar read -- no second pass over ids.  All batches are issued (clamped,
    // in bounds) before the first LDS store waits on them.
    constexpr int ST_LP = FM_STD_LP;   // pair batches per thread in flight (2,048 + 256 staged rows)
    const int NP = E / 2;
    for (int q1 = threadIdx.x; q1 < NP; q1 += ST_T * ST_LP) {
        double2 v[ST_LP];
        longlong2 id[ST_LP];
        int64_t pid0[ST_LP];
#pragma unroll
        for (int k = 0; k < ST_LP; ++k) {
            const int q = q1 + k * ST_T;
            const int64_t r = b - HP + 2 * (int64_t)q;   // even
            if (r >= 0 && r + 1 < n) {
                v[k] = *reinterpret_cast<const double2*>(x + r);
                id[k] = *reinterpret_cast<const longlong2*>(ids + r);
            } else {   // the array's edges (one wave per tile at most): two clamped reads
                const int64_t r0 = r < 0 ? 0 : (r < n ? r : n - 1);
                const int64_t r1 = r + 1 < 0 ? 0 : (r + 1 < n ? r + 1 : n - 1);
                v[k] = make_double2(x[r0], x[r1]);
                id[k] = make_longlong2(ids[r0], ids[r1]);
            }
            // the row before lane 0's pair (wave-uniform address: a scalar read)
            const int64_t rl0 = b - HP + 2 * (int64_t)(q - lane);
            pid0[k] = ids[rl0 >= 1 && rl0 - 1 < n ? rl0 - 1 : 0];
        }
#pragma unroll
        for (int k = 0; k < ST_LP; ++k) {
            const int q = q1 + k * ST_T;
            if (q - lane >= NP) break;   // wave-uniform
            const int e = 2 * q;
            const int64_t r = b - HP + e;
            const bool in0 = r >= 0 && r < n, in1 = r + 1 >= 0 && r + 1 < n;
            const int64_t prev = lane_prev_i64(id[k].y, pid0[k]);
            const uint64_t ev = __ballot(in0 && (r == 0 || id[k].x != prev));
            const uint64_t od = __ballot(in1 && (r + 1 == 0 || id[k].y != id[k].x));
            if (q < NP) {
                xs[spad(e)] = in0 ? nan_if_inf(v[k].x) : (double)NAN;
                xs[spad(e + 1)] = in1 ? nan_if_inf(v[k].y) : (double)NAN;
            }
            if (lane == 0) {   // rows 2q .. 2q + 127: fb words e / 64, e / 64 + 1
                fb[e >> 6] = spread_bits((uint32_t)ev) | (spread_bits((uint32_t)od) << 1);
                fb[(e >> 6) + 1] = spread_bits((uint32_t)(ev >> 32)) | (spread_bits((uint32_t)(od >> 32)) << 1);
            }
        }
    }
    __syncthreads();
    // per-ST_R-row block statistics (count, mean, M2 about the block mean; two-pass) for this
    // tile's own blocks and the nh whole blocks of the halo, so a first window adds ~W/8
    // block states instead of W observations
    const int nh = HP / ST_R;
    const int NB = ST_T + nh;
    double* bmean = (double*)(fb + nw);
    double* bm2 = bmean + NB;
    int* bcnt = (int*)(bm2 + NB);
    // 4-block superblock states (NB is a multiple of 16) and 1 / (c (c - 1)) for c <= W
    const int NS = NB / 4;
    double* smean = (double*)(bcnt + NB);
    double* sm2 = smean + NS;
    int* scnt = (int*)(sm2 + NS);
    double* ivar = (double*)(scnt + NS);
    for (int s = threadIdx.x; s < NB; s += ST_T) {
        const RunStats st = range_stats(xs, HP + (s - nh) * ST_R, HP + (s - nh + 1) * ST_R);
        bmean[s] = st.mean;
        bm2[s] = st.m2;
        bcnt[s] = st.n;
    }
    for (int c = threadIdx.x; c <= W; c += ST_T) ivar[c] = c >= 2 ? 1.0 / ((double)c * ((double)c - 1.0)) : 0.0;
    __syncthreads();
    // superblock = four block states merged (Chan et al.: M2 = sum M2_i + n_i (mean_i - mean)^2)
    for (int S = threadIdx.x; S < NS; S += ST_T) {
        int c = 0;
        double sx = 0.0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            c += bcnt[4 * S + i];
            sx += (double)bcnt[4 * S + i] * bmean[4 * S + i];
        }
        const double mean = c > 0 ? sx / (double)c : 0.0;
        double m2 = 0.0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const double d = bmean[4 * S + i] - mean;
            m2 += bm2[4 * S + i] + (double)bcnt[4 * S + i] * d * d;
        }
        smean[S] = mean;
        sm2[S] = m2;
        scnt[S] = c;
    }
    __syncthreads();
    const int t = threadIdx.x;
    const int e0 = HP + t * ST_R;   // staged index of this thread's first row
    const int64_t i0 = b + t * ST_R;
    if (i0 >= n) return;
#if FM_STD_ABL == 3
    if (i0 + ST_R <= n) {
#pragma unroll
        for (int r = 0; r < ST_R; r += 2)
            *reinterpret_cast<double2*>(out + i0 + r) = make_double2(xs[spad(e0 + r)] + bm2[t], xs[spad(e0 + r + 1)]);
    }
    return;
#endif
    // first window: staged rows [lo, e0], lo = max(e0 - H, the firm's first row): the highest
    // firm-start bit at or below e0 (fs = -1 when the firm starts before the window)
    const int lo0 = e0 - H;
    int fs = -1;
    {
        int w = e0 >> 6;
        uint64_t m = fb[w] & ((e0 & 63) == 63 ? ~0ull : ((2ull << (e0 & 63)) - 1));
        while (m == 0 && w > (lo0 >> 6)) m = fb[--w];
        if (m != 0) fs = w * 64 + 63 - __clzll((long long)m);
    }
    const int lo = fs > lo0 ? fs : lo0;
    // [lo, e0] = a head range, whole blocks jlo..t-1 (all rows inside the firm), row e0
    const int jlo = lo >= HP ? (lo - HP + ST_R - 1) / ST_R : -((HP - lo) / ST_R);
    // window state as count and sums of (x - K), (x - K)^2 about K = a block mean next to
    // the window end: each block / range state (n, mean, M2) adds n*d and M2 + n*d^2 with
    // d = mean - K (exact algebra, no division, four independent chains)
    double K = 0.0;
    {
        const int sk = t - 1 + nh;   // block t-1 (inside the window when jlo < t)
        const double xe = xs[spad(e0)];
        K = (jlo < t && bcnt[sk] > 0) ? bmean[sk] : (isnan(xe) ? 0.0 : xe);
    }
    int cnt = 0;
    double s1 = 0.0, s2 = 0.0;
    auto add_state = [&](const RunStats& st) {
        const double d = st.mean - K;
        const double nd = (double)st.n * d;
        cnt += st.n;
        s1 += nd;
        s2 += st.m2 + nd * d;
    };
    if (jlo >= t) {
        add_state(range_stats(xs, lo, e0 + 1));
    } else {
        add_state(range_stats(xs, lo, HP + jlo * ST_R));
        int c4[4] = {0, 0, 0, 0};
        double a4[4] = {0.0, 0.0, 0.0, 0.0}, q4[4] = {0.0, 0.0, 0.0, 0.0};
        auto acc4 = [&](int u, int c, double mean, double m2) {
            const double d = mean - K;
            const double nd = (double)c * d;
            c4[u] += c;
            a4[u] += nd;
            q4[u] += m2 + nd * d;
        };
        // blocks jlo .. t-1 as single blocks up to a superblock boundary, whole superblocks
        // (two chains), then single blocks: ~W / 32 + 6 states instead of ~W / 8
        int s = jlo + nh;
        const int se = t + nh;
#if FM_STD_ABL == 2
        s = se;
#endif
        for (; s < se && (s & 3) != 0; ++s) acc4(2, bcnt[s], bmean[s], bm2[s]);
        for (; s + 8 <= se; s += 8) {
            acc4(0, scnt[s >> 2], smean[s >> 2], sm2[s >> 2]);
            acc4(1, scnt[(s >> 2) + 1], smean[(s >> 2) + 1], sm2[(s >> 2) + 1]);
        }
        if (s + 4 <= se) {
            acc4(0, scnt[s >> 2], smean[s >> 2], sm2[s >> 2]);
            s += 4;
        }
        for (; s < se; ++s) acc4(3, bcnt[s], bmean[s], bm2[s]);
        cnt += (c4[0] + c4[1]) + (c4[2] + c4[3]);
        s1 += (a4[0] + a4[1]) + (a4[2] + a4[3]);
        s2 += (q4[0] + q4[1]) + (q4[2] + q4[3]);
        const double xe = xs[spad(e0)];
        if (!isnan(xe)) add_state(RunStats{1, xe, 0.0});
    }
    if (cnt == 0) {
        s1 = 0.0;
        s2 = 0.0;
    }
    // trailing run of equal observations (pandas' consecutive-same-value rule; sliding below
    // keeps it): counted back from the window end to the first different observation
    int run = 0;
    double last = NAN;
    for (int f = e0; f >= lo; --f) {
        const double v = xs[spad(f)];
        if (isnan(v)) continue;
        if (run > 0 && v != last) break;
        last = v;
        ++run;
    }
    const int need = minp > 2 ? minp : 2;
    double res[ST_R];
#pragma unroll
    for (int r = 0; r < ST_R; ++r) {
        const int e = e0 + r;
        if (r > 0) {
            if ((fb[e >> 6] >> (e & 63)) & 1ull) {   // a new firm starts here
                fs = e;
                cnt = 0;
                run = 0;
                s1 = 0.0;
                s2 = 0.0;
                last = NAN;
            } else if (fs <= e - W) {   // row e - W (same firm; NaN if before row 0) leaves
                const double v = xs[spad(e - W)];
                if (!isnan(v)) {
                    --cnt;
                    const double d = v - K;
                    s1 -= d;
                    s2 -= d * d;
                    if (cnt == 0) {
                        s1 = 0.0;
                        s2 = 0.0;
                    }
                }
            }
            const double v = xs[spad(e)];
            if (!isnan(v)) {
                if (cnt == 0) K = v;
                ++cnt;
                const double d = v - K;
                s1 += d;
                s2 += d * d;
                run = v == last ? run + 1 : 1;
                last = v;
            }
        }
        double rv = NAN;
        if (cnt >= need) {
            if (run >= cnt) {
                rv = 0.0;   // pandas: every observation in the window is the same value
            } else {
                const double c = (double)cnt;
#if FM_STD_ABL == 1
                rv = (s2 * c - s1 * s1) * scale;
#else
                // the division by c (c - 1) as a product with its tabled reciprocal (within an
                // ulp of the quotient)
                const double var = (s2 * c - s1 * s1) * ivar[cnt];
                rv = sqrt(var > 0.0 ? var : 0.0) * scale;
#endif
            }
        }
        res[r] = rv;
    }
    // 16-byte stores of row pairs (i0 is even); the array's last odd row alone
    if (i0 + ST_R <= n) {
#pragma unroll
        for (int r = 0; r < ST_R; r += 2)
            *reinterpret_cast<double2*>(out + i0 + r) = make_double2(res[r], res[r + 1]);
    } else {
#pragma unroll
        for (int r = 0; r < ST_R; ++r)
            if (i0 + r < n) out[i0 + r] = res[r];
    }
}

}  // namespace
}  // namespace fm

extern "C" int fm_firm_chars(const fm_chars_args* args, void* stream) {
    using namespace fm;
    FM_REQUIRE(args != nullptr, "fm_firm_chars: null args");
    const fm_chars_args& a = *args;
    FM_REQUIRE(a.n >= 0, "fm_firm_chars: negative n");
    if (a.n == 0) return FM_OK;
    FM_REQUIRE(a.ids != nullptr, "fm_firm_chars: null ids");
    // fields each characteristic reads (FM_CHAR_* order)
    static const uint32_t need[FM_NCHARS] = {
        1u << FM_FIELD_ME,
        (1u << FM_FIELD_ME) | (1u << FM_FIELD_BE),
        1u << FM_FIELD_RETX,
        (1u << FM_FIELD_ACCRUALS) | (1u << FM_FIELD_DEPRECIATION),
        (1u << FM_FIELD_EARNINGS) | (1u << FM_FIELD_ASSETS),
        1u << FM_FIELD_ASSETS,
        (1u << FM_FIELD_DVC) | (1u << FM_FIELD_PRC),
        1u << FM_FIELD_RETX,
        1u << FM_FIELD_SHROUT,
        1u << FM_FIELD_SHROUT,
        (1u << FM_FIELD_ME) | (1u << FM_FIELD_TOTAL_DEBT),
        (1u << FM_FIELD_ME) | (1u << FM_FIELD_SALES),
    };
    uint32_t req = 0;
    for (int c = 0; c < FM_NCHARS; ++c)
        if (a.out[c]) req |= need[c];
    if (req == 0) return FM_OK;
    for (int f = 0; f < FM_NFIELDS; ++f)
        FM_REQUIRE(!((req >> f) & 1u) || a.field[f] != nullptr, "fm_firm_chars: field %d required but NULL", f);
    const int need_ret = (a.out[FM_CHAR_RETURN_12_2] || a.out[FM_CHAR_LOG_RETURN_13_36]) ? 1 : 0;
    const int need_dvc = a.out[FM_CHAR_DY] ? 1 : 0;
    const int64_t blocks = (a.n + CT - 1) / CT;
    FM_REQUIRE(blocks < (1ll << 31), "fm_firm_chars: too many rows");
    hipLaunchKernelGGL(firm_chars_kernel, dim3((unsigned)blocks), dim3(CT), 0, (hipStream_t)stream, a,
                       need_ret, need_dvc);
    FM_CHECK_LAUNCH("fm_firm_chars");
    return FM_OK;
}

extern "C" int fm_rolling_std(const int64_t* ids, const double* x, int64_t n, int32_t window,
                              int32_t min_periods, double scale, double* out, void* stream) {
    using namespace fm;
    FM_REQUIRE(n >= 0, "fm_rolling_std: negative n");
    if (n == 0) return FM_OK;
    FM_REQUIRE(ids && x && out, "fm_rolling_std: null pointer");
    // the kernel moves row pairs with 16-byte loads / stores from the bases
    FM_REQUIRE((((uintptr_t)ids | (uintptr_t)x | (uintptr_t)out) & 15) == 0,
               "fm_rolling_std: ids, x and out must be 16-byte aligned");
    FM_REQUIRE(window >= 1 && window <= 4096, "fm_rolling_std: window must be 1..4096");
    FM_REQUIRE(min_periods >= 1 && min_periods <= window, "fm_rolling_std: min_periods must be 1..window");
    const int E = ST_ROWS + st_halo(window);
    const int nb = ST_T + st_halo(window) / ST_R;
    const size_t lds = (size_t)(spad(E) + 1) * 8 + (size_t)((E + 63) / 64) * 8 + (size_t)nb * (8 * 2 + 4) +
                       (size_t)(nb / 4) * (8 * 2 + 4) + (size_t)(window + 1) * 8;
    FM_REQUIRE(lds <= 160 * 1024, "fm_rolling_std: window too large for LDS");
    const int64_t blocks = (n + ST_ROWS - 1) / ST_ROWS;
    FM_REQUIRE(blocks < (1ll << 31), "fm_rolling_std: too many rows");
    if (lds > 64 * 1024 &&
        hipFuncSetAttribute((const void*)rolling_std_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds) != hipSuccess) {
        set_error("fm_rolling_std: cannot raise the dynamic LDS limit to %zu bytes", lds);
        return FM_EHIP;
    }
    hipLaunchKernelGGL(rolling_std_kernel, dim3((unsigned)blocks), dim3(ST_T), lds, (hipStream_t)stream, ids,
                       x, n, (int)window, (int)min_periods, scale, out);
    FM_CHECK_LAUNCH("fm_rolling_std");
    return FM_OK;
}

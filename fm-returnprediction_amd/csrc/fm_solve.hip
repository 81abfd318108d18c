// fm_solve: per (month, model, universe) OLS from the bucketed shifted Grams.
//
// Replaces sm.OLS(Y, X).fit() -> params / rsquared / N and the N < K+1 month skip of
// run_monthly_cs_regressions (reference src/regressions.py:52-72) and the create_figure_1
// OLS (src/calc_Lewellen_2014.py:913-921).  statsmodels solves with an SVD pseudo-inverse
// of X; here the slopes come from the centered normal equations
//     Sxx b = Sxy,  Sxx = sum (x-xbar)(x-xbar)', Sxy = sum (x-xbar)(y-ybar)
// by a Cholesky factorization (one wavefront per problem, lanes over matrix entries).
// When a pivot collapses (1 - R^2 of a regressor on the previous ones <= 1e-9, e.g. an
// all-zero column or an exactly collinear pair) the wave falls back to a Jacobi
// eigen-decomposition of Sxx and the minimum-norm (pseudo-inverse) solution of the
// uncentered design [1, X] (what statsmodels' pinv returns, see jacobi_pinv).
// R^2 = 1 - (Syy - b'Sxy)/Syy (centered TSS: the model has a constant).
//
// One workgroup (4 waves) per month: the month's bucket Grams are first summed over its
// chunks into LDS, then the waves take the month's problems round-robin.
#include <math.h>

#include <type_traits>

#include "fm_common.h"

FM_PROBE_BUFFER(solve)

namespace fm {
namespace {

constexpr int VT = 256;
constexpr int VNW = VT / WAVE;
constexpr int MAXB_LDS = 8192;   // doubles of bucket sums held in LDS (64 KB max)
constexpr int64_t SCAN_GRID = 1024;   // workgroups of the status-scanning fix-up launches
constexpr double CHOL_REL = 1e-9;
constexpr double EIG_REL = 1e-12;
// A pivot below REFIT_REL of its original diagonal (1 - R^2 of a regressor on the previous
// ones) means cond(Sxx) >~ 1e6: the normal-equation error (~eps * cond(Sxx)) could exceed
// the 1e-9 contract, so the problem is flagged FM_ST_REFIT and re-solved from its rows by
// fm_solve_fixup (Householder QR + SVD of R: error ~eps * cond(X), as statsmodels' SVD).
constexpr double REFIT_REL = 1e-6;
#ifndef FM_AB_SOLVE_STOP
#define FM_AB_SOLVE_STOP 0    // timing builds only: 1 stop after the bucket sums, 2 after the centering
#endif
#ifndef FM_AB_SOLVE_MOMROW
#define FM_AB_SOLVE_MOMROW 0  // timing builds only: the moments stored one S row per lane
#endif
#ifndef FM_AB_SOLVE_NOMOM
#define FM_AB_SOLVE_NOMOM 0   // timing builds only (tools/build_variant.sh): skip the moments store
#endif

template <int MD>
struct WaveScratch {
    double A[MD * MD];   // G, then L (Cholesky) or the Jacobi matrix
    double V[MD * MD];   // centered S, then Jacobi eigenvectors
    double sxy[MD], sdiag[MD], mu[MD], b[MD];
};

// Cyclic Jacobi + pseudo-inverse solve by lane 0 (rare fallback path).  A = Sxx (centered),
// mur[0..K-1] = the regressors' raw means and mur[K] = y's.  The range part is the centered
// minimum-norm slope vector b_c; statsmodels' pinv minimizes over the UNCENTERED design
// [1, X] instead, whose null space also holds every affine dependence (a regressor constant
// within the month, x2 = a x1 + c): with N = the null eigenvectors of Sxx, w = N' mur and
// beta0_c = ybar - b_c' mur, the min-norm LS solution is
//     b = b_c + N w beta0_c / (1 + |w|^2),  beta0 = beta0_c / (1 + |w|^2)
// (minimize beta0^2 + |b|^2 over b = b_c + N t, beta0 = beta0_c - w' t).  The intercept is
// then ybar - b' mur as on the regular path, which equals the beta0 above.
template <int MD>
__device__ void jacobi_pinv(double* A, double* V, int K, const double* sxy, const double* mur, double* b) {
    for (int i = 0; i < K; ++i)
        for (int j = 0; j < K; ++j) V[i * MD + j] = i == j ? 1.0 : 0.0;
    double frob = 0.0;
    for (int i = 0; i < K; ++i)
        for (int j = 0; j < K; ++j) frob += A[i * MD + j] * A[i * MD + j];
    for (int sweep = 0; sweep < 80; ++sweep) {
        double off = 0.0;
        for (int p = 0; p < K; ++p)
            for (int q = p + 1; q < K; ++q) off += A[p * MD + q] * A[p * MD + q];
        if (off <= 1e-34 * frob) break;
        for (int p = 0; p < K; ++p) {
            for (int q = p + 1; q < K; ++q) {
                const double apq = A[p * MD + q];
                if (apq == 0.0) continue;
                const double theta = (A[q * MD + q] - A[p * MD + p]) / (2.0 * apq);
                const double t = (theta >= 0.0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
                const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
                for (int k = 0; k < K; ++k) {
                    const double akp = A[k * MD + p], akq = A[k * MD + q];
                    A[k * MD + p] = c * akp - s * akq;
                    A[k * MD + q] = s * akp + c * akq;
                }
                for (int k = 0; k < K; ++k) {
                    const double apk = A[p * MD + k], aqk = A[q * MD + k];
                    A[p * MD + k] = c * apk - s * aqk;
                    A[q * MD + k] = s * apk + c * aqk;
                }
                A[p * MD + q] = 0.0;
                A[q * MD + p] = 0.0;
                for (int k = 0; k < K; ++k) {
                    const double vkp = V[k * MD + p], vkq = V[k * MD + q];
                    V[k * MD + p] = c * vkp - s * vkq;
                    V[k * MD + q] = s * vkp + c * vkq;
                }
            }
        }
    }
    double lmax = 0.0;
    for (int i = 0; i < K; ++i) lmax = fmax(lmax, fabs(A[i * MD + i]));
    for (int j = 0; j < K; ++j) b[j] = 0.0;
    for (int i = 0; i < K; ++i) {
        const double l = A[i * MD + i];
        if (!(l > EIG_REL * lmax)) continue;
        double proj = 0.0;
        for (int k = 0; k < K; ++k) proj += V[k * MD + i] * sxy[k];
        proj /= l;
        for (int j = 0; j < K; ++j) b[j] += proj * V[j * MD + i];
    }
    double b0 = mur[K], den = 1.0;
    for (int j = 0; j < K; ++j) b0 -= b[j] * mur[j];
    for (int i = 0; i < K; ++i) {
        if (A[i * MD + i] > EIG_REL * lmax) continue;
        double wi = 0.0;
        for (int k = 0; k < K; ++k) wi += V[k * MD + i] * mur[k];
        den += wi * wi;
    }
    if (!(den > 1.0) || !isfinite(b0)) return;   // the null space misses the intercept
    for (int i = 0; i < K; ++i) {
        if (A[i * MD + i] > EIG_REL * lmax) continue;
        double wi = 0.0;
        for (int k = 0; k < K; ++k) wi += V[k * MD + i] * mur[k];
        const double t = b0 * wi / den;
        for (int j = 0; j < K; ++j) b[j] += t * V[j * MD + i];
    }
}

__device__ __forceinline__ double readlane_f64(double v, int l) {
    return __longlong_as_double((long long)readlane_u64((uint64_t)__double_as_longlong(v), l));
}

// Sum the month's chunk partials into LDS: BCH loads per thread in flight per chunk (a
// one-load-per-iteration loop waits out one HBM round trip per element).
template <int NT>
__device__ __forceinline__ void sum_partials(const double* partial, int c0, int c1, int n, double* bs) {
    constexpr int BCH = 8;
    const int tid = threadIdx.x;
    for (int e0 = tid; e0 < n; e0 += NT * BCH) {
        double acc[BCH];
#pragma unroll
        for (int k = 0; k < BCH; ++k) acc[k] = 0.0;
        for (int c = c0; c < c1; ++c) {
            const double* pc = partial + (int64_t)c * n;
#pragma unroll
            for (int k = 0; k < BCH; ++k) {
                const int e = e0 + k * NT;
                acc[k] += pc[e < n ? e : n - 1];   // clamped: unconditional loads
            }
        }
#pragma unroll
        for (int k = 0; k < BCH; ++k) {
            const int e = e0 + k * NT;
            if (e < n) bs[e] = acc[k];
        }
    }
}

// Per month: bucket sums -> level-cumulative sums (bucket (pattern, u) becomes the sum over
// levels >= u, so a problem adds one bucket per pattern that contains its model) -> one
// wave per problem.  The wave keeps the centered moment matrix S over (x_1..x_K, y) in
// registers, lane i = row i (MD doubles), and factors it by a right-looking Cholesky whose
// pivot-row broadcasts are readlanes (no LDS round trip per column).  Factoring the
// augmented matrix [Sxx Sxy; Sxy' Syy] leaves l = L^-1 Sxy in the y row, so the forward
// substitution comes free; the back substitution L' b = l runs on the transposed factor
// (one LDS transpose), lane i owning b_i.
template <int MD>
__global__ __launch_bounds__(VT) void solve_kernel(fm_solve_args a) {
    extern __shared__ double bs[];   // [nb][zw(zw+1)/2] packed bucket sums of this month
    __shared__ WaveScratch<MD> ws_all[VNW];
    const int s = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & (WAVE - 1);
    const int w = __builtin_amdgcn_readfirstlane(tid / WAVE);
    const int zw = a.zw, zz = zw * (zw + 1) / 2;   // packed upper triangle per bucket
    const int nl = a.nlevels, npat = a.npatterns, nb = npat * nl;
    const int c0 = a.seg_chunk_off[s], c1 = a.seg_chunk_off[s + 1];
    sum_partials<VT>(a.partial, c0, c1, nb * zz, bs);
    __syncthreads();
    for (int e = tid; e < npat * zz; e += VT) {
        const int pid = e / zz, f = e - pid * zz;
        double* b0 = bs + (int64_t)pid * nl * zz + f;
        double run = b0[(nl - 1) * zz];
        for (int l = nl - 2; l >= 0; --l) {
            run += b0[l * zz];
            b0[l * zz] = run;
        }
    }
    __syncthreads();
    WaveScratch<MD>& ws = ws_all[w];
    const int rs = a.pmax + 2;
    constexpr int PKW = MD * (MD + 1) / 2;   // packed entries of one problem Gram
    constexpr int EPL = (PKW + WAVE - 1) / WAVE;
    for (int p = w; p < a.nprob; p += VNW) {
        const int m = a.prob_model[p], u = a.prob_level[p], nz = a.prob_nz[p];
        const int* zi = a.prob_z + p * 32;
        const int K = nz - 2, K1 = K + 1;
        // ---- the problem's Gram G[i][j] (i, j < nz over its z indices) into the wave's V:
        // lanes over packed (i <= j) entries, patterns in the outer loop, so each pattern
        // costs one batch of independent LDS reads; G is written in both triangles
        int off[EPL], dst[EPL], dsw[EPL];
        double acc[EPL];
#pragma unroll
        for (int t = 0; t < EPL; ++t) {
            const int e = lane + WAVE * t;
            int i = 0, rem = e;   // packed index e -> (i, j), rows of length nz - i
            while (i < nz && rem >= nz - i) {
                rem -= nz - i;
                ++i;
            }
            const bool in = i < nz;
            const int j = in ? i + rem : 0;
            const int zr = in ? zi[i] : 0, zc = in ? zi[j] : 0;
            const int r = zr < zc ? zr : zc, c = zr < zc ? zc : zr;
            off[t] = in ? r * zw - (r * (r - 1)) / 2 + (c - r) : 0;
            dst[t] = in ? i * MD + j : -1;
            dsw[t] = in ? j * MD + i : -1;
            acc[t] = 0.0;
        }
        for (int q = 0; q < npat; ++q) {
            if (!((a.pattern_models[q] >> m) & 1u)) continue;   // wave-uniform
            const double* bq = bs + (q * nl + u) * zz;
#pragma unroll
            for (int t = 0; t < EPL; ++t) acc[t] += bq[off[t]];
        }
#pragma unroll
        for (int t = 0; t < EPL; ++t)
            if (dst[t] >= 0) {
                ws.V[dst[t]] = acc[t];
                ws.V[dsw[t]] = acc[t];
            }
        wave_sync();
        const double* Gp = ws.V;   // G[i][j], row stride MD; z index 0 is the intercept
        const int zl = lane < K1 ? zi[1 + lane] : 0;   // panel z index of this lane's row
        const int li = lane < K1 ? 1 + lane : 0;       // this lane's row in Gp
        const double n = Gp[0];
        const double g0 = lane < K1 ? Gp[li] : 0.0;    // first moment of this lane's variable
        const double gdiag = lane < K1 ? Gp[li * MD + li] : 0.0;
        const int64_t ro = ((int64_t)s * a.nprob + p) * rs;
        uint32_t st = 0;
        // inf in the problem's rows: a regressor or y value of +-inf makes its Gram diagonal
        // sum(z^2) = +inf (columns the problem does not use are never read)
        if (__ballot(lane < K && isinf(gdiag)) != 0) st |= FM_ST_INF_IN_X;
        if (__ballot(lane == K && isinf(gdiag)) != 0) st |= FM_ST_INF_IN_Y;
        if (a.gram_flags) st |= a.gram_flags[(int64_t)s * a.nmodels + m] & (FM_ST_INF_IN_X | FM_ST_INF_IN_Y);
        if (!(n >= (double)(K + 1))) {
            for (int k = lane; k < rs; k += WAVE) a.rec[ro + k] = k == a.pmax + 1 ? n : NAN;
            if (lane == 0) a.status[(int64_t)s * a.nprob + p] = FM_ST_SKIPPED;
            continue;
        }
        // ---- centered moments: row i of S, S[i][j] = G(z_i, z_j) - G(0, z_i) G(0, z_j) / n
        double row[MD];
        double sii = 0.0, sxy = 0.0;   // S[i][i], S[i][K] of this lane
#pragma unroll
        for (int j = 0; j < MD; ++j) {
            row[j] = 0.0;
            if (j < K1) {
                const double v = lane < K1 ? Gp[li * MD + 1 + j] - g0 * Gp[1 + j] / n : 0.0;
                row[j] = v;
                if (j == lane) sii = v;
                if (j == K) sxy = v;
            }
        }
        const double mu = g0 / n;
        if (a.moments) {
            double* mo = a.moments + ((int64_t)s * a.nprob + p) * a.mom_stride;
            if (lane == 0) mo[0] = n;
            if (lane < K1) {
                mo[1 + lane] = mu;
#pragma unroll
                for (int j = 0; j < MD; ++j)
                    if (j < K1) mo[1 + K1 + lane * K1 + j] = row[j];
            }
        }
        if ((a.prob_flags[p] & 1) != 0) {
            if (__ballot(lane < K && !(sii > 1e-10 * gdiag)) != 0) st |= FM_ST_CONST_SUSPECT;
        }
        const double syy = readlane_f64(sii, K);
        // ---- augmented Cholesky, lane i = row i; rows >= K1 are zero
        bool ok = true;
#pragma unroll
        for (int k = 0; k < MD - 1; ++k) {
            if (ok && k < K) {   // wave-uniform
                const double orig = readlane_f64(sii, k);
                const double piv = readlane_f64(row[k], k);
                if (!(piv > REFIT_REL * orig)) st |= FM_ST_REFIT;
                if (!(orig > 0.0) || !(piv > CHOL_REL * orig)) {
                    ok = false;
                } else {
                    const double lkk = sqrt(piv);
                    const double rinv = 1.0 / lkk;
                    const double lik = row[k] * rinv;
#pragma unroll
                    for (int j = k + 1; j < MD; ++j) {
                        if (j <= K) {
                            const double sj = readlane_f64(row[j], k) * rinv;   // L[j][k]
                            row[j] -= lik * sj;
                        }
                    }
                    row[k] = lane == k ? lkk : lik;
                }
            }
        }
        double bi = 0.0;
        if (ok) {
            // transpose through LDS: lane i then holds column i of L (and l_i)
            double* T = ws.A;
#pragma unroll
            for (int j = 0; j < MD; ++j)
                if (lane < K1) T[lane * MD + j] = row[j];
            wave_sync();
            double col[MD];
#pragma unroll
            for (int r = 0; r < MD; ++r) col[r] = lane < MD ? T[r * MD + (lane & (MD - 1))] : 0.0;
            double t = lane < K ? T[K * MD + lane] : 0.0;   // l_i
#pragma unroll
            for (int j = MD - 2; j >= 0; --j) {
                if (j < K) {
                    const double bj = readlane_f64(t, j) / readlane_f64(col[j], j);
                    if (lane == j) t = bj;
                    else if (lane < j) t -= col[j] * bj;
                }
            }
            bi = lane < K ? t : 0.0;
            wave_sync();
        } else {
            st |= FM_ST_RANK_DEF | FM_ST_REFIT;
            // rebuild Sxx (rows were overwritten) for the pseudo-inverse fallback
#pragma unroll
            for (int j = 0; j < MD; ++j)
                if (j < K && lane < K) ws.A[lane * MD + j] = Gp[li * MD + 1 + j] - g0 * Gp[1 + j] / n;
            if (lane < K) ws.sxy[lane] = sxy;
            if (lane < K1) ws.mu[lane] = mu + (a.add_back ? a.add_back[(int64_t)(zl - 1) * a.nseg + s] : 0.0);
            wave_sync();
            if (lane == 0) jacobi_pinv<MD>(ws.A, ws.V, K, ws.sxy, ws.mu, ws.b);
            wave_sync();
            bi = lane < K ? ws.b[lane] : 0.0;
            wave_sync();
        }
        // R^2 = 1 - SSR/SST (centered), raw-coordinate intercept
        double t_sxy = lane < K ? bi * sxy : 0.0;
        double t_mu = lane < K ? bi * mu : 0.0;
        double t_ab = 0.0;
        if (a.add_back && lane < K) t_ab = bi * a.add_back[(int64_t)(zl - 1) * a.nseg + s];
        t_sxy = wave_sum(t_sxy);
        t_mu = wave_sum(t_mu);
        t_ab = wave_sum(t_ab);
        const double r2 = 1.0 - (syy - t_sxy) / syy;
        double icpt = readlane_f64(mu, K) - t_mu;
        if (a.add_back) icpt += a.add_back[(int64_t)(zi[K + 1] - 1) * a.nseg + s] - t_ab;
        // b_{k-1} to lane k (all lanes active: a bpermute reads nothing from inactive lanes);
        // rs <= 34 < 64, so lane k writes record entry k
        const double bsh = __shfl(bi, lane > 0 ? lane - 1 : 0, WAVE);
        for (int k = lane; k < rs; k += WAVE) {
            double v = NAN;   // pad between the slopes and R^2
            if (k == 0) v = icpt;
            else if (k <= K) v = bsh;
            else if (k == a.pmax) v = r2;
            else if (k == a.pmax + 1) v = n;
            a.rec[ro + k] = v;
        }
        if (lane == 0) a.status[(int64_t)s * a.nprob + p] = st | FM_ST_FITTED;
    }
}

// ---------------------------------------------------------------------------------------
// zw == 16 (<= 15 panel columns): four problems per wave.  A problem owns one 16-lane row of
// the wave and lane i holds row i of its Gram (row 0 = the intercept, rows 1..K+1 = the
// centered moments S of x_1..x_K, y), so the pivot-row broadcasts of the Cholesky are DPP
// row_newbcast moves (VALU modifiers: no LDS round trip, no readlane hazards) and four
// factorizations run in the time of one.  Rank-deficient problems (rare) take the Jacobi
// pseudo-inverse path one at a time.

#ifndef FM_SOLVE_RSQ
#define FM_SOLVE_RSQ 1
#endif
// 1 / sqrt(x) for a positive normal x: v_rsq_f64 refined by two Newton steps
__device__ __forceinline__ double rsq_nr(double x) {
    double y = __builtin_amdgcn_rsq(x);
    const double h = 0.5 * x;
    y = y * fma(-h * y, y, 1.5);
    y = y * fma(-h * y, y, 1.5);
    return y;
}

template <int L>
__device__ __forceinline__ int rowbc_i(int v) {   // lane L of this lane's 16-lane row
    // every lane has a source (row_newbcast): mov_dpp needs no zero-initialised destination
    return __builtin_amdgcn_mov_dpp(v, 0x150 + L, 0xF, 0xF, true);
}
template <int L>
__device__ __forceinline__ double rowbc(double v) {
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = (uint32_t)rowbc_i<L>((int)(uint32_t)b), hi = (uint32_t)rowbc_i<L>((int)(uint32_t)(b >> 32));
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
__device__ __forceinline__ double rowsum(double v) { return row16_sum(v); }

constexpr int G16 = 16;   // lanes per problem

template <int NC, int NT>
union FixSmem;
inline __device__ bool fix_wanted(uint32_t st, int check_const);
template <int NC, int NT, class CA>
__device__ __forceinline__ void fix_one(int s, int p, uint32_t st, FixSmem<NC, NT>& sm, CA cols, int64_t stride,
                        const int64_t* seg_off, int nseg, const double* lo, const double* hi,
                        const double* shift, const double* inv_scale, const double* add_back,
                        const uint8_t* level, int nprob, const int32_t* prob_level, const int32_t* prob_z,
                        const int32_t* prob_nz, const double* moments, int mom_stride, int pmax, double* rec,
                        uint32_t* status, int check_const);

// 192 threads (three waves, twelve problems at a time: a Table-2 month's 11 problems in ONE
// round, so no wave factors twice) at two waves per SIMD: 256 VGPRs (the factorization's
// register rows and columns fit without spills); every month of a 600-month panel is
// resident at once.
constexpr int S16T = 192;
constexpr int S16W = S16T / WAVE;
constexpr int S16_MAXP = 32;   // problems per group held in LDS tables
__global__ __launch_bounds__(S16T, 3) void solve16_kernel(fm_solve_args a) {
    extern __shared__ double bs[];   // [nb][136] packed bucket sums of this month
    // per wave: four transpose tiles, or (afterwards, one problem at a time) the Jacobi
    // fallback's scratch (a union)
    constexpr int TT = G16 * (G16 + 1);
    static_assert(sizeof(WaveScratch<16>) <= 4 * TT * sizeof(double), "scratch union");
    __shared__ double wsc[S16W][4 * TT];
    const int s = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & (WAVE - 1);
    const int w = __builtin_amdgcn_readfirstlane(tid / WAVE);
    constexpr int zw = 16, zz = 136;
    const int nl = a.nlevels, npat = a.npatterns, nb = npat * nl;
    // The small per-problem tables and this month's add-back values go to LDS first, all
    // loads issued together with the partials' (read in place, each would be a dependent
    // memory round trip inside the problem loop)
    __shared__ int t_model[S16_MAXP], t_level[S16_MAXP], t_nz[S16_MAXP], t_flags[S16_MAXP];
    __shared__ int t_slot[S16_MAXP];   // wave slot -> problem, by descending K
    __shared__ uint32_t t_st[S16_MAXP];   // the month's solve status (inline fix-ups)
    __shared__ uint8_t t_z[S16_MAXP][32];
    __shared__ uint32_t t_pat[64];
    __shared__ double t_ab[32];
    for (int e = tid; e < a.nprob * 32; e += S16T) t_z[e >> 5][e & 31] = (uint8_t)a.prob_z[e];
    if (tid < a.nprob) {
        t_model[tid] = a.prob_model[tid];
        t_level[tid] = a.prob_level[tid];
        const int nzp = a.prob_nz[tid];
        t_nz[tid] = nzp;
        t_flags[tid] = a.prob_flags[tid];
        // Problems go to wave slots by descending K (ties: index order): the factorization
        // loops run to the largest K of the wave's four problems, so grouping similar K
        // cuts the issued work (Table 2: 3 x K 14, 3 x 7, 2 x 5, 3 x 3 per month)
        int rank = 0;
        for (int q = 0; q < a.nprob; ++q) {
            const int nzq = a.prob_nz[q];
            rank += (nzq > nzp || (nzq == nzp && q < tid)) ? 1 : 0;
        }
        t_slot[rank] = tid;
    }
    if (tid < npat) t_pat[tid] = a.pattern_models[tid];
    if (a.add_back && tid >= 64 && tid < 96) {
        const int c = tid - 64;   // panel columns past ncols are never indexed
        t_ab[c] = c < a.ab_ncols ? a.add_back[(int64_t)c * a.nseg + s] : 0.0;
    }
    FM_PROBE_AT(solve, 0);
    const int c0 = a.seg_chunk_off[s], c1 = a.seg_chunk_off[s + 1];
    sum_partials<S16T>(a.partial, c0, c1, nb * zz, bs);
    __syncthreads();
    FM_PROBE_AT(solve, 1);
    for (int e = tid; e < npat * zz; e += S16T) {   // level-cumulative buckets
        const int pid = e / zz, f = e - pid * zz;
        double* b0 = bs + (int64_t)pid * nl * zz + f;
        double run = b0[(nl - 1) * zz];
        for (int l = nl - 2; l >= 0; --l) {
            run += b0[l * zz];
            b0[l * zz] = run;
        }
    }
    __syncthreads();
    FM_PROBE_AT(solve, 2);
    if (FM_AB_SOLVE_STOP == 1) {
        if (tid == 0) a.status[(int64_t)s * a.nprob] = (uint32_t)bs[0];
        return;
    }
    const int g = lane >> 4, i = lane & 15;
    const int rs = a.pmax + 2;
    double* T = wsc[w] + g * TT;
    for (int p0 = w * 4; p0 < a.nprob; p0 += S16W * 4) {
        const int p = p0 + g;
        const bool live = p < a.nprob;
        const int pp = t_slot[live ? p : p0];
        const int m = t_model[pp], u = t_level[pp], nz = t_nz[pp];
        const int K = nz - 2, K1 = K + 1;
        // wave-uniform loop bound: the largest K of this wave's problems (slots by
        // descending K: the first live slot's)
        const int kw = __builtin_amdgcn_readfirstlane(K);
        const int zi = i < nz ? t_z[pp][i] : 0;   // z index of this lane's row
        // ---- row i of the problem Gram: one level-cumulative bucket per pattern with m.
        // A lambda, so the rare rank-deficient path re-reads G from LDS instead of keeping it
        // (and the offsets) live through the factorization: 48 VGPRs, no spills at 3 waves/SIMD
        auto gram_row = [&](double (&G)[G16]) {
            int off[G16];
            static_for<0, G16>([&](auto jc) {
                constexpr int j = decltype(jc)::value;
                const int zj = rowbc_i<j>(zi);
                const int r = zi < zj ? zi : zj, c = zi < zj ? zj : zi;
                off[j] = r * zw - (r * (r - 1)) / 2 + (c - r);
            });
#pragma unroll
            for (int j = 0; j < G16; ++j) G[j] = 0.0;
            for (int q = 0; q < npat; ++q) {
                if (!((t_pat[q] >> m) & 1u)) continue;   // per problem
                const double* bq = bs + (q * nl + u) * zz;
#pragma unroll
                for (int j = 0; j < G16; ++j)
                    if (j < kw + 2) G[j] += bq[off[j]];   // columns past the wave's K: unused
            }
        };
        double G[G16];
        gram_row(G);
        const double n = rowbc<0>(G[0]);
        const double ninv = 1.0 / n;   // one division per lane (centering below multiplies)
        // centered moments: lane i (1 <= i <= K1) holds S row r = i - 1, S[r][c] in row[c]
        const bool srow = i >= 1 && i <= K1;
        double row[G16];
        double sii = 0.0, sxy = 0.0, gdiag = 0.0;
        static_for<0, G16>([&](auto jc) {
            constexpr int j = decltype(jc)::value;
            gdiag = i == j ? G[j] : gdiag;   // selects, not conditional stores (see below)
            if constexpr (j + 1 < G16) {
                if (j > kw) {   // wave-uniform: past every problem's last column
                    row[j] = 0.0;
                    return;
                }
                const double g0j = rowbc<0>(G[j + 1]);   // G[0][j+1]
                const double v = srow && j < K1 ? G[j + 1] - G[0] * g0j * ninv : 0.0;
                row[j] = v;
                // conditional assignments to these per-lane scalars were merged by the
                // compiler into a store through a selected address, which kept them in
                // scratch memory; plain selects keep them in registers
                sii = i == j + 1 ? v : sii;
                sxy = j == K ? v : sxy;
            } else {
                row[j] = 0.0;
            }
        });
        FM_PROBE_AT(solve, 4);
        const double mu = G[0] * ninv;   // lane i: mean of its variable
        const uint64_t gm = 0xFFFFull << (16 * g);
        uint32_t st = 0;
        if ((__ballot(i >= 1 && i <= K && isinf(gdiag)) & gm) != 0) st |= FM_ST_INF_IN_X;
        if ((__ballot(i == K1 && isinf(gdiag)) & gm) != 0) st |= FM_ST_INF_IN_Y;
        const int64_t ro = ((int64_t)s * a.nprob + pp) * rs;
        const bool skip = !(n >= (double)(K + 1));
        if (live && skip) {
            for (int k = i; k < rs; k += G16) a.rec[ro + k] = k == a.pmax + 1 ? n : NAN;
            if (i == 0) a.status[(int64_t)s * a.nprob + pp] = t_st[pp] = FM_ST_SKIPPED;
        }
        const bool act0 = live && !skip;
        if (act0 && a.moments && !FM_AB_SOLVE_NOMOM) {
            double* mo = a.moments + ((int64_t)s * a.nprob + pp) * a.mom_stride;
            if (i == 0) mo[0] = n;
            if (srow) {
                mo[i] = mu;   // mo[1 + r]
                // S is exactly symmetric (S[r][c] and S[c][r] are the same products of the
                // same packed sums), so lane r stores column r of S: S[c][r] for every c, and
                // each store instruction writes K1 consecutive doubles (a row-per-lane store
                // strides K1 doubles between lanes)
#pragma unroll
                for (int c = 0; c < G16 - 1; ++c)
                    if (c < K1) {
                        if (FM_AB_SOLVE_MOMROW) mo[1 + K1 + (i - 1) * K1 + c] = row[c];
                        else mo[1 + K1 + c * K1 + (i - 1)] = row[c];
                    }
            }
        }
        if (act0 && (t_flags[pp] & 1) != 0) {
            if ((__ballot(i >= 1 && i <= K && !(sii > 1e-10 * gdiag)) & gm) != 0) st |= FM_ST_CONST_SUSPECT;
        }
        if (FM_AB_SOLVE_STOP == 2) {
            if (live && i == 0) a.rec[ro] = row[0] + row[1] + mu;
            continue;
        }
        FM_PROBE_AT(solve, 5);
        // ---- augmented Cholesky of S (pivot r = k sits in lane k + 1)
        bool ok = act0, illc = false;
        double dinv = 0.0;   // lane k + 1: 1 / L[k][k] (the back substitution multiplies by it)
        static_for<0, G16 - 1>([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            if (k >= kw) return;   // wave-uniform: no problem of the wave has pivot k
            const bool act = ok && k < K;
            const double orig = rowbc<k + 1>(sii);
            const double piv = rowbc<k + 1>(row[k]);
            if (act && !(piv > REFIT_REL * orig)) illc = true;
            const bool bad = act && (!(orig > 0.0) || !(piv > CHOL_REL * orig));
            if (bad) ok = false;
            const bool go = act && !bad;
#if FM_SOLVE_RSQ
            // 1 / sqrt(piv) by the hardware estimate and two Newton steps (error ~1 ulp), sqrt
            // as piv times it: no IEEE sqrt and division sequences on the pivot chain
            const double rinv = rsq_nr(piv);
            const double lkk = piv * rinv;
#else
            const double lkk = sqrt(piv);
            const double rinv = 1.0 / lkk;
#endif
            const double lik = row[k] * rinv;
            // unguarded: the entries a guard would keep are never read again -- columns past
            // the problem's K (and, once k >= K, everything this step touches) are not used by
            // the back substitution, and a problem whose pivot failed is refactored from G by
            // the Jacobi path below -- so the two selects per entry are not needed
            static_for<k + 1, G16>([&](auto jc) {
                constexpr int j = decltype(jc)::value;
                if (j > kw) return;   // wave-uniform
                const double sj = rowbc<k + 1>(row[j]) * rinv;   // L[j][k] = S(k)[k][j] / lkk
                row[j] = row[j] - lik * sj;
            });
            row[k] = go ? (i == k + 1 ? lkk : lik) : row[k];
            dinv = i == k + 1 ? rinv : dinv;
        });
        FM_PROBE_AT(solve, 6);
        // lanes of a live, unskipped problem with a collapsed pivot: rank deficient
        const bool rank_def = act0 && !ok;
        // ---- back substitution L' b = l on the transposed factor: lane i then holds
        // column r = i - 1 of L (col[c] = L[c][r]) and t = l_r
        if (srow) {
#pragma unroll
            for (int c = 0; c < G16; ++c) T[(i - 1) * (G16 + 1) + c] = row[c];
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        double col[G16];
        const int rr = i >= 1 ? i - 1 : 0;
#pragma unroll
        for (int c = 0; c < G16 - 1; ++c) col[c] = T[c * (G16 + 1) + rr];
        col[G16 - 1] = 0.0;
        double t = (i >= 1 && i <= K) ? T[K * (G16 + 1) + rr] : 0.0;
        static_for<0, G16 - 1>([&](auto jc) {
            constexpr int j = 14 - decltype(jc)::value;   // descending
            if (j >= kw) return;   // wave-uniform
            const double bj = rowbc<j + 1>(t) * rowbc<j + 1>(dinv);   // t_j / L[j][j]
            if (ok && j < K) {
                if (i == j + 1) t = bj;
                else if (i >= 1 && i - 1 < j) t -= col[j] * bj;
            }
        });
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        FM_PROBE_AT(solve, 7);
        double bi = (ok && i >= 1 && i <= K) ? t : 0.0;   // slope of x_{i-1}
        // ---- rank-deficient problems of this wave: Jacobi pseudo-inverse, one at a time
        const uint64_t rd = __ballot(rank_def && i == 0);
        double G2[G16];
        if (rd) gram_row(G2);   // wave-uniform
        for (uint64_t q = rd; q; q &= q - 1) {
            const int gq = __builtin_ctzll(q) >> 4;   // wave-uniform
            WaveScratch<16>& J = *reinterpret_cast<WaveScratch<16>*>(wsc[w]);
            const int Kq = __shfl(K, gq * 16, WAVE);
            const double (&G)[G16] = G2;
            // rebuild Sxx (rows were overwritten) from G, the shuffles with every lane active
            {
                double g0c[G16 - 1];
#pragma unroll
                for (int c = 0; c < G16 - 1; ++c) g0c[c] = __shfl(G[c + 1], gq * 16, WAVE);
                const double nq = __shfl(n, gq * 16, WAVE);
                if (g == gq && i >= 1 && i <= Kq) {
#pragma unroll
                    for (int c = 0; c < G16 - 1; ++c)
                        if (c < Kq) J.A[(i - 1) * 16 + c] = G[c + 1] - G[0] * g0c[c] / nq;
                    J.sxy[i - 1] = sxy;
                }
                if (g == gq && i >= 1 && i <= Kq + 1)   // raw means of x_0..x_{K-1}, y
                    J.mu[i - 1] = mu + (a.add_back ? t_ab[zi - 1] : 0.0);
            }
            wave_sync();
            if (lane == 0) jacobi_pinv<16>(J.A, J.V, Kq, J.sxy, J.mu, J.b);
            wave_sync();
            if (g == gq && i >= 1 && i <= Kq) bi = J.b[i - 1];
            wave_sync();
        }
        if (rank_def) st |= FM_ST_RANK_DEF;
        if (illc) st |= FM_ST_REFIT;
        // ---- R^2 = 1 - SSR/SST (centered), raw-coordinate intercept
        const bool xl = i >= 1 && i <= K;
        double t_sxy = xl ? bi * sxy : 0.0;
        double t_mu = xl ? bi * mu : 0.0;
        double t_abx = 0.0;
        if (a.add_back && xl && act0) t_abx = bi * t_ab[zi - 1];
        t_sxy = rowsum(t_sxy);
        t_mu = rowsum(t_mu);
        t_abx = rowsum(t_abx);
        const double syy = __shfl(sii, g * 16 + (K1 < 16 ? K1 : 15), WAVE);   // S[K][K]
        const double muy = __shfl(mu, g * 16 + (K1 < 16 ? K1 : 15), WAVE);
        const double r2 = 1.0 - (syy - t_sxy) / syy;
        double icpt = muy - t_mu;
        if (a.add_back && act0) {
            const int zy = t_z[pp][K + 1];
            icpt += t_ab[zy - 1] - t_abx;
        }
        if (act0) {
            for (int k = i; k < rs; k += G16) {
                double v = NAN;   // pad between the slopes and R^2
                if (k == 0) v = icpt;
                else if (k <= K) v = k == i ? bi : NAN;   // k == i on the first pass
                else if (k == a.pmax) v = r2;
                else if (k == a.pmax + 1) v = n;
                a.rec[ro + k] = v;
            }
            if (i == 0) a.status[(int64_t)s * a.nprob + pp] = t_st[pp] = st | FM_ST_FITTED;
        }
    }
    FM_PROBE_AT(solve, 3);
    // the statsmodels fix-ups of this month's flagged problems (fm_solve_fixup's work, rare),
    // by this workgroup: its own rec / moments / status writes are visible after the barrier
    // the rows come from the FP64 columns, else (a planes-only panel) from the two planes: one
    // instantiation per layout (a per-access branch raised the kernel to 231 VGPRs)
    auto fix_all = [&](auto cols) {
        __syncthreads();
        const int ckc = a.fix_check_const;
        for (int q = 0; q < a.nprob; ++q) {
            const uint32_t st = t_st[q];
            if (!fix_wanted(st, ckc)) continue;   // block-uniform
            fix_one<G16, S16T>(s, q, st, *reinterpret_cast<FixSmem<G16, S16T>*>(&wsc[0][0]), cols,
                               a.fix_stride, a.fix_seg_off, a.nseg, a.fix_lo, a.fix_hi, a.fix_shift,
                               a.fix_inv_scale, a.add_back, a.fix_level, a.nprob, a.prob_level, a.prob_z,
                               a.prob_nz, a.moments, a.mom_stride, a.pmax, a.rec, a.status, ckc);
        }
    };
    if (a.fix_cols != nullptr) fix_all(F64Cols{a.fix_cols});   // block-uniform
    else if (a.fix_hi_plane != nullptr) fix_all(PlaneCols{a.fix_hi_plane, (int64_t)(a.fix_lo_plane - a.fix_hi_plane)});
}

// Exact nonzero-constant test for problems flagged CONST_SUSPECT (statsmodels
// add_constant(has_constant='skip'): np.ptp(x)==0 & all(x != 0), src/regressions.py:50).
template <int NT = VT, class CA = F64Cols>
__device__ __forceinline__ void const_pair(int s, int p, uint64_t* red, CA cols, int64_t stride,
                                           const int64_t* seg_off, int nseg, const double* lo,
                                           const double* hi, const uint8_t* level, int nprob,
                                           const int32_t* prob_level, const int32_t* prob_z,
                                           const int32_t* prob_nz, uint32_t* status) {
    const int nz = prob_nz[p], K = nz - 2, u = prob_level[p];
    const int* zi = prob_z + p * 32;
    const int64_t r0 = seg_off[s], r1 = seg_off[s + 1];
    bool any_const = false;
    for (int j = 0; j < K; ++j) {
        const int cx = zi[1 + j] - 1;
        uint64_t kmin = SENT, kmax = 0;
        bool allnz = true;
        for (int64_t r = r0 + threadIdx.x; r < r1; r += NT) {
            if (level && (int)level[r] < u) continue;
            bool ok = true;
            double xv = 0.0;
            for (int q = 1; q < nz; ++q) {
                const int c = zi[q] - 1;
                double x = cols[(int64_t)c * stride + r];
                if (lo) {
                    const double l = lo[(int64_t)c * nseg + s], h = hi[(int64_t)c * nseg + s];
                    if (x < l) x = l;
                    if (x > h) x = h;
                }
                if (isnan(x)) ok = false;
                if (c == cx) xv = x;
            }
            if (!ok) continue;
            const uint64_t k = dkey(xv == 0.0 ? 0.0 : xv);
            kmin = k < kmin ? k : kmin;
            kmax = k > kmax ? k : kmax;
            if (xv == 0.0) allnz = false;
        }
        kmin = block_min_u64<NT / WAVE>(kmin, red);
        kmax = block_max_u64<NT / WAVE>(kmax, red);
        const int nzr = block_sum<NT / WAVE>(allnz ? 0 : 1, (int*)red);
        if (kmin != SENT && kmin == kmax && nzr == 0) any_const = true;
    }
    if (threadIdx.x == 0 && any_const) status[(int64_t)s * nprob + p] |= FM_ST_CONST_COL;
}

__global__ __launch_bounds__(VT) void const_kernel(F64Cols cols, int64_t stride, int ncols,
                                                   const int64_t* seg_off, int nseg,
                                                   const double* lo, const double* hi,
                                                   const uint8_t* level, int nprob,
                                                   const int32_t* prob_level, const int32_t* prob_z,
                                                   const int32_t* prob_nz, const int32_t* pairs,
                                                   int npairs, uint32_t* status) {
    __shared__ uint64_t red[VNW];
    // npairs < 0: scan every (month, problem) and take those the solve flagged, so the
    // check needs no host round trip; else the listed pairs.
    const int total = npairs < 0 ? nseg * nprob : npairs;
    for (int e = blockIdx.x; e < total; e += gridDim.x) {
        int s, p;
        if (npairs < 0) {
            s = e / nprob;
            p = e - s * nprob;
            if (!(status[e] & FM_ST_CONST_SUSPECT)) continue;
        } else {
            s = pairs[2 * e];
            p = pairs[2 * e + 1];
        }
        const_pair(s, p, red, cols, stride, seg_off, nseg, lo, hi, level, nprob, prob_level, prob_z,
                   prob_nz, status);
    }
}

// inf in y (statsmodels keeps the month): params = pinv(X) @ y, so each coefficient is the
// IEEE sum of pinv[j,i] * y_i; with y_i = +-inf the finite rows do not matter and the
// result is +inf, -inf or NaN (mixed signs, or 0*inf).  pinv[:,i] for the slopes is
// Sxx^{-1}(x_i - xbar) and for the intercept 1/n - xbar'Sxx^{-1}(x_i - xbar).  One
// workgroup per flagged (month, problem); R^2 becomes NaN as in statsmodels.
struct InfySmem {
    double Lm[32 * 32];
    double mu[32], xb[32];
    unsigned bits[32];
    int okf;
};

template <int NT = VT, int NC = 32, class CA = F64Cols>
__device__ __forceinline__ void infy_pair(int s, int p, InfySmem& sm, CA cols, int64_t stride,
                                          const int64_t* seg_off, int nseg, const double* lo,
                                          const double* hi, const double* shift,
                                          const double* inv_scale, const double* add_back,
                                          const uint8_t* level, int nprob,
                                          const int32_t* prob_level, const int32_t* prob_z,
                                          const int32_t* prob_nz, const double* moments,
                                          int mom_stride, int pmax, double* rec) {
    double* Lm = sm.Lm;
    double* mu = sm.mu;
    double* xb = sm.xb;
    unsigned* bits = sm.bits;
    int& okf = sm.okf;
    const int nz = prob_nz[p], K = nz - 2, K1 = K + 1, u = prob_level[p];
    const int* zi = prob_z + p * 32;
    const double* mo = moments + ((int64_t)s * nprob + p) * mom_stride;
    const double n = mo[0];
    for (int e = threadIdx.x; e < K * K; e += NT) Lm[(e / K) * 32 + e % K] = mo[1 + K1 + (e / K) * K1 + e % K];
    if (threadIdx.x < K1) mu[threadIdx.x] = mo[1 + threadIdx.x];
    if (threadIdx.x < 32) bits[threadIdx.x] = 0u;
    __syncthreads();
    if (threadIdx.x < K) {
        const int c = zi[1 + threadIdx.x] - 1;
        xb[threadIdx.x] = mu[threadIdx.x] + (add_back ? add_back[(int64_t)c * nseg + s] : 0.0);
    }
    if (threadIdx.x == 0) {
        int ok = 1;
        for (int k = 0; k < K && ok; ++k) {
            double d = Lm[k * 32 + k];
            for (int j = 0; j < k; ++j) d -= Lm[k * 32 + j] * Lm[k * 32 + j];
            if (!(d > 0.0)) { ok = 0; break; }
            d = sqrt(d);
            Lm[k * 32 + k] = d;
            for (int i = k + 1; i < K; ++i) {
                double t = Lm[i * 32 + k];
                for (int j = 0; j < k; ++j) t -= Lm[i * 32 + j] * Lm[k * 32 + j];
                Lm[i * 32 + k] = t / d;
            }
        }
        okf = ok;
    }
    __syncthreads();
    if (!okf) return;   // rank-deficient with an inf y: left as computed (NaN)
    const int64_t r0 = seg_off[s], r1 = seg_off[s + 1];
    if constexpr (NC <= 16) {
        // register arrays (fully unrolled, statically indexed: no scratch, which would throttle
        // the waves of the solve kernel these fix-ups ride); the opaque zero keeps the factor's
        // LDS reads inside the row loop instead of hoisted into ~120 live registers
        for (int64_t r = r0 + threadIdx.x; r < r1; r += NT) {
            if (level && (int)level[r] < u) continue;
            int zo = 0;
            asm volatile("" : "+v"(zo));
            double d[NC];
            double y = 0.0;
            bool valid = true;
#pragma unroll
            for (int q = 1; q <= NC; ++q) {
                if (q < nz) {
                    const int c = zi[q] - 1;
                    double x = cols[(int64_t)c * stride + r];
                    if (lo) {
                        const double l = lo[(int64_t)c * nseg + s], h = hi[(int64_t)c * nseg + s];
                        if (x < l) x = l;
                        if (x > h) x = h;
                    }
                    if (isnan(x)) valid = false;
                    if (q == nz - 1) {
                        y = x;
                    } else {
                        if (shift) x -= shift[(int64_t)c * nseg + s];
                        if (inv_scale) x *= inv_scale[(int64_t)c * nseg + s];
                        d[q - 1] = x - mu[q - 1 + zo];
                    }
                }
            }
            if (!valid || !isinf(y)) continue;
#pragma unroll
            for (int i = 0; i < NC; ++i) {          // L w = d
                if (i < K) {
                    double t = d[i];
#pragma unroll
                    for (int j = 0; j < i; ++j) t -= Lm[i * 32 + j + zo] * d[j];
                    d[i] = t / Lm[i * 32 + i + zo];
                }
            }
#pragma unroll
            for (int i = NC - 1; i >= 0; --i) {     // L' c = w
                if (i < K) {
                    double t = d[i];
#pragma unroll
                    for (int j = i + 1; j < NC; ++j)
                        if (j < K) t -= Lm[j * 32 + i + zo] * d[j];
                    d[i] = t / Lm[i * 32 + i + zo];
                }
            }
            double c0 = 1.0 / n;
#pragma unroll
            for (int j = 0; j < NC; ++j)
                if (j < K) c0 -= xb[j + zo] * d[j];
#pragma unroll
            for (int j = 0; j <= NC; ++j) {
                if (j <= K) {
                    const double term = (j == 0 ? c0 : d[j == 0 ? 0 : j - 1]) * y;
                    const unsigned b = isnan(term) ? 4u : (term > 0.0 ? 1u : 2u);
                    atomicOr(&bits[j], b);
                }
            }
        }
    } else
    for (int64_t r = r0 + threadIdx.x; r < r1; r += NT) {
        if (level && (int)level[r] < u) continue;
        double v[32];
        bool valid = true;
        for (int q = 1; q < nz; ++q) {
            const int c = zi[q] - 1;
            double x = cols[(int64_t)c * stride + r];
            if (lo) {
                const double l = lo[(int64_t)c * nseg + s], h = hi[(int64_t)c * nseg + s];
                if (x < l) x = l;
                if (x > h) x = h;
            }
            if (isnan(x)) valid = false;
            v[q - 1] = x;
        }
        if (!valid || !isinf(v[K])) continue;
        const double y = v[K];
        double d[32];
        for (int j = 0; j < K; ++j) {
            const int c = zi[1 + j] - 1;
            double x = v[j];
            if (shift) x -= shift[(int64_t)c * nseg + s];
            if (inv_scale) x *= inv_scale[(int64_t)c * nseg + s];
            d[j] = x - mu[j];
        }
        for (int i = 0; i < K; ++i) {          // L w = d
            double t = d[i];
            for (int j = 0; j < i; ++j) t -= Lm[i * 32 + j] * d[j];
            d[i] = t / Lm[i * 32 + i];
        }
        for (int i = K - 1; i >= 0; --i) {     // L' c = w
            double t = d[i];
            for (int j = i + 1; j < K; ++j) t -= Lm[j * 32 + i] * d[j];
            d[i] = t / Lm[i * 32 + i];
        }
        double c0 = 1.0 / n;
        for (int j = 0; j < K; ++j) c0 -= xb[j] * d[j];
        for (int j = 0; j <= K; ++j) {
            const double term = (j == 0 ? c0 : d[j - 1]) * y;
            const unsigned b = isnan(term) ? 4u : (term > 0.0 ? 1u : 2u);
            atomicOr(&bits[j], b);
        }
    }
    __syncthreads();
    const int64_t ro = ((int64_t)s * nprob + p) * (pmax + 2);
    if (threadIdx.x <= K) {
        const unsigned b = bits[threadIdx.x];
        if (b != 0u) {
            double val = NAN;
            if (!(b & 4u) && b != 3u) val = (b & 1u) ? INFINITY : -INFINITY;
            rec[ro + threadIdx.x] = val;
        }
    }
    if (threadIdx.x == 0) rec[ro + pmax] = NAN;
}

// ---------------------------------------------------------------------------------------
// Row-level refit of FM_ST_REFIT problems (ill-conditioned or rank-deficient Sxx), so that
// statsmodels' pinv semantics hold where the normal equations cannot: pinv_extended takes
// the SVD of the UNCENTERED design X = [1, x_1..x_K] (rcond 1e-15) and returns
// params = V S^+ U' y (min-norm over [1, X]), rsquared = 1 - SSR / centered TSS.
//   1. Householder TSQR of [X | y] over the problem's rows (the Gram's row set: universe
//      level >= u, every model column non-NaN after the clip), each wave absorbing 64-row
//      tiles into its own triangular factor, the four factors then merged by wave 0.
//      Backward stable: the factor's error is ~eps * |X|, not eps * |X|^2.
//   2. One-sided (Hestenes) Jacobi SVD of R_xx, cut at SVD_REL * sigma_max, and
//      beta = V S^+ U' r_y with r_y = Q'y.  SSR = |r_y - R_xx beta|^2 + rho^2 (rho = y's
//      diagonal of R), centered TSS = sum_{i >= 1} r_y[i]^2 + rho^2 (column 0 is the
//      constant, so Q's first column is 1/sqrt(n)).
// SVD_REL is 1e-13, not statsmodels' 1e-15: an exact dependence (a zero column, x2 = 2 x1,
// a regressor constant within the month) leaves a singular value at the QR's rounding
// floor (~N eps sigma_max), which must be cut; genuine near-dependences down to 1e-13 are
// kept.
constexpr double SVD_REL = 1e-13;

__device__ __forceinline__ double wave_sum_dpp(double v) {
    v += xor_lanes_f64(v, 1);
    v += xor_lanes_f64(v, 2);
    v += xor_lanes_f64(v, 4);
    v += xor_lanes_f64(v, 8);
    v += xor_lanes_f64(v, 16);
    v += xor_lanes_f64(v, 32);
    return v;
}

template <int NC, int NW = VNW>
struct RefitSmem {
    double R[NW][NC][NC + 1];    // per-wave triangular factors of [1, x, y]
    double Ac[NC][NC + 1];       // Jacobi: rotated columns of R_xx, Ac[j][i] = (R_xx V)[i][j]
    double Vc[NC][NC + 1];       // Jacobi: V[i][j] at Vc[j][i]
    double bv[NC];
};

// Absorb one 64-row tile (lane = row, a[] = its NC values, zero rows allowed) into the
// wave's triangular factor R: Householder reflections over [R row k; tile column k].
template <int NC>
__device__ __forceinline__ void hh_absorb(double (&a)[NC], double (*R)[NC + 1], int nzc) {
    const int lane = lane_id();
    static_for<0, NC>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        if (k < nzc) {
            const double ss = wave_sum_dpp(a[k] * a[k]);
            if (ss != 0.0) {   // wave-uniform: a zero tile column leaves R as it is
                const double alpha = R[k][k];
                const double nrm = sqrt(alpha * alpha + ss);
                const double beta = alpha > 0.0 ? -nrm : nrm;
                const double v0 = alpha - beta;
                const double tau = -v0 / beta;
                const double vl = a[k] / v0;   // v = (1, a[:,k] / v0)
                double w[NC];
                static_for<k + 1, NC>([&](auto jc) {
                    constexpr int j = decltype(jc)::value;
                    w[j] = vl * a[j];
                });
                static_for<k + 1, NC>([&](auto jc) {
                    constexpr int j = decltype(jc)::value;
                    w[j] = wave_sum_dpp(w[j]) + R[k][j];
                });
                static_for<k + 1, NC>([&](auto jc) {
                    constexpr int j = decltype(jc)::value;
                    a[j] -= (tau * w[j]) * vl;
                });
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                if (lane == 0) {
                    R[k][k] = beta;
                    static_for<k + 1, NC>([&](auto jc) {
                        constexpr int j = decltype(jc)::value;
                        R[k][j] -= tau * w[j];
                    });
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                a[k] = 0.0;
            }
        }
    });
}

template <int NC, int NT = VT, class CA = F64Cols>
__device__ void refit_pair(int s, int p, RefitSmem<NC, NT / WAVE>& sm, CA cols, int64_t stride,
                           const int64_t* seg_off, int nseg, const double* lo, const double* hi,
                           const double* shift, const double* inv_scale, const double* add_back,
                           const uint8_t* level, int nprob, const int32_t* prob_level,
                           const int32_t* prob_z, const int32_t* prob_nz, int pmax, double* rec,
                           uint32_t* status) {
    const int tid = threadIdx.x, lane = tid & (WAVE - 1), w = tid / WAVE;
    const int nz = prob_nz[p], P = nz - 1, u = prob_level[p];
    const int* zi = prob_z + p * 32;
    constexpr int NW = NT / WAVE;
    for (int e = tid; e < NW * NC * (NC + 1); e += NT) (&sm.R[0][0][0])[e] = 0.0;
    __syncthreads();
    int zc[NC];   // panel column of z index q (q >= 1)
    static_for<0, NC>([&](auto qc) {
        constexpr int q = decltype(qc)::value;
        zc[q] = (q >= 1 && q < nz) ? zi[q] - 1 : 0;
    });
    const int64_t r0 = seg_off[s], r1 = seg_off[s + 1];
    for (int64_t base = r0 + (int64_t)w * WAVE; base < r1; base += NT) {
        const int64_t r = base + lane;
        bool valid = r < r1 && !(level && (int)level[r] < u);
        double a[NC];
        static_for<0, NC>([&](auto qc) {
            constexpr int q = decltype(qc)::value;
            double v = 0.0;
            if constexpr (q == 0) {
                v = 1.0;
            } else {
                if (valid && q < nz) {
                    const int c = zc[q];
                    double x = cols[(int64_t)c * stride + r];
                    if (lo) {
                        const double l = lo[(int64_t)c * nseg + s], h = hi[(int64_t)c * nseg + s];
                        if (x < l) x = l;
                        if (x > h) x = h;
                    }
                    if (inv_scale) {
                        x = (x - shift[(int64_t)c * nseg + s]) * inv_scale[(int64_t)c * nseg + s];
                        if (add_back) x += add_back[(int64_t)c * nseg + s];
                    }
                    if (isnan(x)) valid = false;
                    v = x;
                }
            }
            a[q] = v;
        });
        static_for<0, NC>([&](auto qc) {
            constexpr int q = decltype(qc)::value;
            if (!valid) a[q] = 0.0;
        });
        hh_absorb<NC>(a, sm.R[w], nz);
    }
    __syncthreads();
    if (w == 0) {   // merge the other waves' factors into wave 0's
        for (int o = 1; o < NW; ++o) {
            double a[NC];
            static_for<0, NC>([&](auto jc) {
                constexpr int j = decltype(jc)::value;
                a[j] = (lane < NC && j >= lane) ? sm.R[o][lane < NC ? lane : 0][j] : 0.0;
            });
            hh_absorb<NC>(a, sm.R[0], nz);
        }
        // ---- one-sided Jacobi SVD of R_xx (P x P upper triangular), lane i = row i
        double (*R)[NC + 1] = sm.R[0];
        const bool li = lane < P;
        const int lr = li ? lane : 0;
        if (li)
            for (int j = 0; j < P; ++j) {
                sm.Ac[j][lane] = j >= lane ? R[lane][j] : 0.0;
                sm.Vc[j][lane] = j == lane ? 1.0 : 0.0;
            }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (int sweep = 0; sweep < 60; ++sweep) {
            bool rotated = false;
            for (int pc = 0; pc < P - 1; ++pc) {
                for (int qc = pc + 1; qc < P; ++qc) {
                    const double ap = li ? sm.Ac[pc][lr] : 0.0, aq = li ? sm.Ac[qc][lr] : 0.0;
                    const double al = wave_sum_dpp(ap * ap);
                    const double be = wave_sum_dpp(aq * aq);
                    const double ga = wave_sum_dpp(ap * aq);
                    if (!(fabs(ga) > 1e-15 * sqrt(al * be))) continue;   // wave-uniform
                    rotated = true;
                    const double zeta = (be - al) / (2.0 * ga);
                    const double t = fabs(zeta) > 1e150
                                         ? 0.5 / zeta
                                         : (zeta >= 0.0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
                    const double c = 1.0 / sqrt(1.0 + t * t), sn = c * t;
                    const double vp = li ? sm.Vc[pc][lr] : 0.0, vq = li ? sm.Vc[qc][lr] : 0.0;
                    if (li) {
                        sm.Ac[pc][lane] = c * ap - sn * aq;
                        sm.Ac[qc][lane] = sn * ap + c * aq;
                        sm.Vc[pc][lane] = c * vp - sn * vq;
                        sm.Vc[qc][lane] = sn * vp + c * vq;
                    }
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                }
            }
            if (!rotated) break;
        }
        // ---- beta = V S^+ (R_xx V)' r_y; singular values below SVD_REL * sigma_max cut
        const double ry = li ? R[lane][P] : 0.0;   // Q'y
        const double rho = R[P][P];
        double smax = 0.0;
        for (int j = 0; j < P; ++j) smax = fmax(smax, wave_sum_dpp(li ? sm.Ac[j][lr] * sm.Ac[j][lr] : 0.0));
        smax = sqrt(smax);
        double bi = 0.0;
        bool cut = false;
        for (int j = 0; j < P; ++j) {
            const double aj = li ? sm.Ac[j][lr] : 0.0;
            const double s2 = wave_sum_dpp(aj * aj);
            if (!(sqrt(s2) > SVD_REL * smax)) {
                cut = true;
                continue;
            }
            const double cj = wave_sum_dpp(aj * ry) / s2;
            if (li) bi += sm.Vc[j][lane] * cj;
        }
        if (li) sm.bv[lane] = bi;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        double fit = 0.0;
        if (li)
            for (int j = lane; j < P; ++j) fit += R[lane][j] * sm.bv[j];
        const double e = li ? ry - fit : 0.0;
        const double ssr = wave_sum_dpp(e * e) + rho * rho;
        const double tss = wave_sum_dpp((li && lane >= 1) ? ry * ry : 0.0) + rho * rho;
        const int64_t ro = ((int64_t)s * nprob + p) * (pmax + 2);
        if (li) rec[ro + lane] = bi;
        if (lane == 0) {
            rec[ro + pmax] = 1.0 - ssr / tss;
            const uint32_t st = status[(int64_t)s * nprob + p];
            status[(int64_t)s * nprob + p] = (st & ~FM_ST_RANK_DEF) | (cut ? FM_ST_RANK_DEF : 0u);
        }
    }
}

// statsmodels fix-ups after fm_solve, one workgroup per flagged (month, problem):
// CONST_SUSPECT (with check_const) -> const_pair; FITTED|INF_IN_Y -> infy_pair;
// FITTED|REFIT (no inf) -> refit_pair.
template <int NC, int NT>
union FixSmem {
    InfySmem infy;
    RefitSmem<NC, NT / WAVE> refit;
    uint64_t red[NT / WAVE];
};
static_assert(sizeof(FixSmem<G16, S16T>) <= sizeof(double) * S16W * 4 * G16 * (G16 + 1),
              "solve16's inline fix-ups reuse its per-wave scratch");
inline __device__ bool fix_wanted(uint32_t st, int check_const) {
    return (check_const && (st & FM_ST_CONST_SUSPECT)) ||
           ((st & FM_ST_FITTED) && (st & (FM_ST_INF_IN_Y | FM_ST_REFIT)));
}
// The fix-ups of one flagged (month, problem) whose solve status is `st`, by the whole
// NT-thread workgroup (block-uniform; ends with the workgroup synchronized)
template <int NC, int NT, class CA>
__device__ __forceinline__ void fix_one(int s, int p, uint32_t st, FixSmem<NC, NT>& sm, CA cols,
                                        int64_t stride, const int64_t* seg_off, int nseg, const double* lo,
                                        const double* hi, const double* shift, const double* inv_scale,
                                        const double* add_back, const uint8_t* level, int nprob,
                                        const int32_t* prob_level, const int32_t* prob_z,
                                        const int32_t* prob_nz, const double* moments, int mom_stride,
                                        int pmax, double* rec, uint32_t* status, int check_const) {
    if (check_const && (st & FM_ST_CONST_SUSPECT)) {
        const_pair<NT>(s, p, sm.red, cols, stride, seg_off, nseg, lo, hi, level, nprob, prob_level, prob_z,
                       prob_nz, status);
        __syncthreads();
    }
    if (!(st & FM_ST_FITTED)) return;
    if (st & FM_ST_INF_IN_Y) {
        infy_pair<NT, NC>(s, p, sm.infy, cols, stride, seg_off, nseg, lo, hi, shift, inv_scale, add_back, level,
                      nprob, prob_level, prob_z, prob_nz, moments, mom_stride, pmax, rec);
    } else if ((st & FM_ST_REFIT) && !(st & FM_ST_INF_IN_X) && prob_nz[p] <= NC) {
        refit_pair<NC, NT>(s, p, sm.refit, cols, stride, seg_off, nseg, lo, hi, shift, inv_scale, add_back,
                           level, nprob, prob_level, prob_z, prob_nz, pmax, rec, status);
    } else {
        return;
    }
    __syncthreads();   // sm is reused by the next pair
}

template <int NC>
__global__ __launch_bounds__(VT) void fixup_kernel(F64Cols cols, int64_t stride,
                                                   const int64_t* seg_off, int nseg, const double* lo,
                                                   const double* hi, const double* shift,
                                                   const double* inv_scale, const double* add_back,
                                                   const uint8_t* level, int nprob,
                                                   const int32_t* prob_level, const int32_t* prob_z,
                                                   const int32_t* prob_nz, const int32_t* pairs,
                                                   int npairs, const double* moments, int mom_stride,
                                                   int pmax, double* rec, uint32_t* status,
                                                   int check_const) {
    __shared__ FixSmem<NC, VT> sm;
    // npairs < 0: scan every (month, problem) for the flags (no host round trip).  Each
    // workgroup reads VT status words at once and lists the flagged pairs in LDS (a
    // pair-by-pair scan would wait out one memory round trip per pair), then fixes them.
    __shared__ int flagged[VT];
    __shared__ int nflag;
    const int total = npairs < 0 ? nseg * nprob : npairs;
    const int tid = threadIdx.x;
    FM_PROBE_AT(solve, 4);
    for (int base = blockIdx.x * VT; base < total; base += gridDim.x * VT) {
        if (tid == 0) nflag = 0;
        __syncthreads();
        {
            const int e = base + tid;
            if (e < total) {
                int s, p;
                if (npairs < 0) {
                    s = e / nprob;
                    p = e - s * nprob;
                } else {
                    s = pairs[2 * e];
                    p = pairs[2 * e + 1];
                }
                if (fix_wanted(status[(int64_t)s * nprob + p], check_const))
                    flagged[atomicAdd(&nflag, 1)] = s * nprob + p;
            }
        }
        __syncthreads();
        const int nf = nflag;
        for (int f = 0; f < nf; ++f) {
            const int sp = flagged[f];
            const int s = sp / nprob, p = sp - s * nprob;
            fix_one<NC, VT>(s, p, status[(int64_t)s * nprob + p], sm, cols, stride, seg_off, nseg, lo, hi, shift,
                            inv_scale, add_back, level, nprob, prob_level, prob_z, prob_nz, moments, mom_stride,
                            pmax, rec, status, check_const);
        }
        __syncthreads();   // the list is rebuilt for the next range
    }
    FM_PROBE_AT(solve, 5);
}

}  // namespace
}  // namespace fm

extern "C" int fm_solve(const fm_solve_args* args, void* stream) {
    using namespace fm;
    FM_REQUIRE(args != nullptr, "fm_solve: null args");
    const fm_solve_args& a = *args;
    FM_REQUIRE(a.partial && a.seg_chunk_off && a.pattern_models && a.prob_model && a.prob_level &&
                   a.prob_z && a.prob_nz && a.prob_flags && a.rec && a.status,
               "fm_solve: null pointer");
    FM_REQUIRE(a.zw == 16 || a.zw == 32, "fm_solve: zw must be 16 or 32");
    FM_REQUIRE(a.npatterns * a.nlevels * (a.zw * (a.zw + 1) / 2) <= MAXB_LDS,
               "fm_solve: %d buckets of a %d-wide Gram exceed the LDS budget", a.npatterns * a.nlevels, a.zw);
    FM_REQUIRE(a.pmax >= 2 && a.pmax <= 32, "fm_solve: pmax must be 2..32");
    FM_REQUIRE(a.moments == nullptr || a.mom_stride > 0, "fm_solve: bad mom_stride");
    FM_REQUIRE(a.add_back == nullptr || (a.ab_ncols >= 1 && a.ab_ncols <= FM_MAX_COLS),
               "fm_solve: add_back needs ab_ncols in 1..%d", FM_MAX_COLS);
    FM_REQUIRE(a.zw == 32 || a.nprob <= S16_MAXP, "fm_solve: at most %d problems per group", S16_MAXP);
    FM_REQUIRE((a.fix_hi_plane == nullptr) == (a.fix_lo_plane == nullptr),
               "fm_solve: fix_hi_plane and fix_lo_plane go together");
    FM_REQUIRE((a.fix_cols == nullptr && a.fix_hi_plane == nullptr) || (a.zw == 16 && a.fix_seg_off && a.moments && a.pmax + 1 <= 16 &&
                                         (a.fix_lo == nullptr) == (a.fix_hi == nullptr) &&
                                         (a.fix_inv_scale == nullptr || a.fix_shift != nullptr)),
               "fm_solve: inline fix-ups need zw 16, fix_seg_off, moments, pmax <= 15, lo with hi, "
               "shift with inv_scale");
    if (a.nseg == 0 || a.nprob == 0) return FM_OK;
    const size_t dyn = (size_t)a.npatterns * a.nlevels * (a.zw * (a.zw + 1) / 2) * sizeof(double);
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)solve16_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                            MAXB_LDS * (int)sizeof(double));
        (void)hipFuncSetAttribute((const void*)solve_kernel<32>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            MAXB_LDS * (int)sizeof(double));
        attr_set = true;
    }
    if (a.zw == 16)
        hipLaunchKernelGGL(solve16_kernel, dim3(a.nseg), dim3(S16T), dyn, (hipStream_t)stream, a);
    else
        hipLaunchKernelGGL(solve_kernel<32>, dim3(a.nseg), dim3(VT), dyn, (hipStream_t)stream, a);
    FM_CHECK_LAUNCH("fm_solve");
    return FM_OK;
}

extern "C" int fm_const_check(const double* cols, int64_t col_stride, int32_t ncols,
                              const int64_t* seg_off, int32_t nseg, const double* lo,
                              const double* hi, const uint8_t* level, int32_t nprob,
                              const int32_t* prob_level, const int32_t* prob_z,
                              const int32_t* prob_nz, const int32_t* pairs, int32_t npairs,
                              uint32_t* status, void* stream) {
    using namespace fm;
    FM_REQUIRE(cols && seg_off && prob_level && prob_z && prob_nz && status &&
                   (pairs || npairs < 0), "fm_const_check: null pointer");
    FM_REQUIRE((lo == nullptr) == (hi == nullptr), "fm_const_check: lo/hi must both be set or NULL");
    const int64_t work = npairs < 0 ? (int64_t)nseg * nprob : npairs;
    if (work == 0) return FM_OK;
    const int grid = (int)(npairs < 0 ? (work < SCAN_GRID ? work : SCAN_GRID) : work);
    hipLaunchKernelGGL(const_kernel, dim3(grid), dim3(VT), 0, (hipStream_t)stream, F64Cols{cols},
                       col_stride, ncols, seg_off, nseg, lo, hi, level, nprob, prob_level, prob_z,
                       prob_nz, pairs, npairs, status);
    FM_CHECK_LAUNCH("fm_const_check");
    return FM_OK;
}

extern "C" int fm_solve_fixup(const double* cols, int64_t col_stride, const int64_t* seg_off,
                              int32_t nseg, const double* lo, const double* hi, const double* shift,
                              const double* inv_scale, const double* add_back, const uint8_t* level,
                              int32_t nprob, const int32_t* prob_level, const int32_t* prob_z,
                              const int32_t* prob_nz, const int32_t* pairs, int32_t npairs,
                              const double* moments, int32_t mom_stride, int32_t pmax, double* rec,
                              uint32_t* status, int32_t check_const, void* stream) {
    using namespace fm;
    FM_REQUIRE(cols && seg_off && prob_level && prob_z && prob_nz && moments && rec && status &&
                   (pairs || npairs < 0), "fm_solve_fixup: null pointer");
    FM_REQUIRE((lo == nullptr) == (hi == nullptr), "fm_solve_fixup: lo/hi must both be set or NULL");
    FM_REQUIRE(inv_scale == nullptr || shift != nullptr, "fm_solve_fixup: inv_scale needs shift");
    FM_REQUIRE(pmax >= 2 && pmax <= 32, "fm_solve_fixup: pmax must be 2..32");
    const int64_t work = npairs < 0 ? (int64_t)nseg * nprob : npairs;
    if (work == 0) return FM_OK;
    const int64_t ranges = (work + VT - 1) / VT;   // VT pairs per workgroup pass
    const int grid = (int)(ranges < SCAN_GRID ? ranges : SCAN_GRID);
    if (pmax + 1 <= 16)
        hipLaunchKernelGGL(fixup_kernel<16>, dim3(grid), dim3(VT), 0, (hipStream_t)stream, F64Cols{cols},
                           col_stride, seg_off, nseg, lo, hi, shift, inv_scale, add_back, level, nprob, prob_level,
                           prob_z, prob_nz, pairs, npairs, moments, mom_stride, pmax, rec, status, check_const);
    else
        hipLaunchKernelGGL(fixup_kernel<32>, dim3(grid), dim3(VT), 0, (hipStream_t)stream, F64Cols{cols},
                           col_stride, seg_off, nseg, lo, hi, shift, inv_scale, add_back, level, nprob, prob_level,
                           prob_z, prob_nz, pairs, npairs, moments, mom_stride, pmax, rec, status, check_const);
    FM_CHECK_LAUNCH("fm_solve_fixup");
    return FM_OK;
}

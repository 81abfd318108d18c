// fm_gram: clip -> dropna-validity -> shifted Gram accumulation on FP64 MFMA.
//
// Replaces, for every (month, model, universe) problem at once, the row filtering of
// run_monthly_cs_regressions (`.dropna()`, reference src/regressions.py:39), the universe
// subsetting of get_subsets (src/calc_Lewellen_2014.py:95-105) and the X'X / X'y / y'y
// formation inside sm.OLS (src/regressions.py:57, src/calc_Lewellen_2014.py:917-919).
//
// Data flow per workgroup (one chunk of one month; 256 threads = 4 waves):
//   1. each thread streams one row of the chunk tile: ncols coalesced FP64 loads (one per
//      column, SoA), clip to the month's winsorize cuts, NaN/inf tests, shift by the
//      month's pivot (optional standardize scale), z = [1, x..., y] with NaN -> 0;
//   2. the row's validity pattern (bit m: every column model m needs is non-NaN) and its
//      universe level give a bucket id; a wave-ballot counting sort scatters the tile
//      into LDS grouped by bucket, each bucket padded to a multiple of 4 rows;
//   3. each wave walks 4-row groups of the sorted tile and issues
//      v_mfma_f64_16x16x4_f64 with A = B = the group's z rows (lane l holds
//      z[row l>>4][col l&15]), accumulating Z^T Z per bucket in registers (16x16 FP64
//      tile = 4 doubles per lane; two tiles wide for up to 31 columns).
// At chunk end the four waves' accumulators are summed through LDS and written as one
// packed upper-triangular Gram per (chunk, bucket).  fm_solve combines buckets into problems: model m's
// Gram is the sum over patterns that contain m and levels >= the problem's universe,
// restricted to m's columns.  One HBM read of the panel serves every model x universe.
#include <math.h>
#include <stdlib.h>

#include "fm_common.h"

namespace fm {
namespace {

constexpr int GT = 256;
constexpr int GNW = GT / WAVE;

typedef double d4 __attribute__((ext_vector_type(4)));

// DBG (measurement builds only, FM_GRAM_DEBUG): 1 = stream the tiles and skip sort/MFMA,
// 2 = clip + sort + scatter but no MFMA.  Results are wrong in debug modes.
template <int NT, int NB, int MINW, bool PF, int DBG = 0>
__global__ __launch_bounds__(GT, MINW) void gram_kernel(fm_gram_args a) {
    constexpr int ZW = 16 * NT;
    constexpr int RS = ZW + 1;          // LDS row stride (doubles): conflict-free scatter
    constexpr int ROWS = GT + 3 * NB;   // sorted tile incl. padding rows
    constexpr int TILE = ROWS * RS > GNW * ZW * ZW ? ROWS * RS : GNW * ZW * ZW;
    __shared__ double tile[TILE];
    __shared__ double prm[4][32];
    __shared__ int wcnt[GNW][NB];
    __shared__ int woff[GNW][NB];
    __shared__ int boff[NB + 1];
    __shared__ int btot[NB];
    __shared__ uint8_t lut[64];
    __shared__ uint32_t mmask[FM_MAX_MODELS], ymask[FM_MAX_MODELS];

    const int tid = threadIdx.x;
    const int lane = tid & (WAVE - 1);
    const int w = __builtin_amdgcn_readfirstlane(tid / WAVE);   // wave-uniform (SGPR loops)
    const int chunk = blockIdx.x;
    const int seg = a.chunk_seg[chunk];
    const int64_t r0 = a.chunk_row[2 * chunk], r1 = a.chunk_row[2 * chunk + 1];
    const int ncols = a.ncols, nseg = a.nseg, nmodels = a.nmodels, nlevels = a.nlevels;

    // Prologue loads are unconditional (pointer/index selected, value masked after) and are
    // issued before the first tile, so they cost one HBM round trip, not one per load.
    double pv;
    int lutv, mmv, ymv;
    {
        const int kind = tid >> 5, c = tid & 31;
        const double* src = kind == 0 ? a.lo : kind == 1 ? a.hi : kind == 2 ? a.shift : a.inv_scale;
        const bool on = tid < 128 && c < ncols && src != nullptr;
        const double* pp = on ? src + (int64_t)c * nseg + seg : a.cols;
        const double v = *pp;
        const double dflt = kind < 2 ? NAN : (kind == 2 ? 0.0 : 1.0);
        pv = on ? v : dflt;
        const int npat = 1 << nmodels;
        lutv = a.pattern_id[tid < npat ? tid : 0];
        const int mi = tid < nmodels ? tid : 0;
        mmv = (int)a.model_mask[mi];
        ymv = (int)a.model_ymask[mi];
    }
    d4 acc0[NB], acc1[NB], acc2[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        acc0[b] = d4{0.0, 0.0, 0.0, 0.0};
        if (NT == 2) {
            acc1[b] = d4{0.0, 0.0, 0.0, 0.0};
            acc2[b] = d4{0.0, 0.0, 0.0, 0.0};
        }
    }
    uint32_t fl = 0;   // bit 2m: inf in a regressor of model m; bit 2m+1: inf in its y

    // Software pipeline, two register buffers: tile t+1's loads are issued before tile t
    // is sorted and accumulated (no copy between buffers, which would force vmcnt(0)).
    // Loads are unconditional (row and column clamped in range, results masked after): a
    // load under a runtime condition makes hipcc wait vmcnt(0) per load.
    // Without universes the level load reads byte 0 of the panel and is masked to 0.  The base
    // must be a kernel-argument pointer: a __device__ global would make it a flat load, which
    // also counts in lgkmcnt, so every LDS wait of the tile would wait for HBM.
    const uint8_t* lvbase = a.level ? a.level : (const uint8_t*)a.cols;
    const int64_t lvmask = a.level ? ~(int64_t)0 : 0;   // address select, not a conditional load
    const int lvand = a.level ? 0xFF : 0;
    auto load_tile = [&](double (&xv)[ZW - 1], int& lv, int64_t t0) {
        const int64_t lrow = t0 + tid < r1 ? t0 + tid : r1 - 1;
#pragma unroll
        for (int c = 0; c < ZW - 1; ++c) {
            const int cc = c < ncols ? c : ncols - 1;
            xv[c] = a.cols[(int64_t)cc * a.col_stride + lrow];
        }
        lv = lvbase[lrow & lvmask] & lvand;
    };
    const int col = lane & 15, sub = lane >> 4;
    double dbg_sink = 0.0;
    auto process_tile = [&](double (&xv)[ZW - 1], int lvraw, int64_t t0) {
        if (DBG == 1) {
#pragma unroll
            for (int c = 0; c < ZW - 1; ++c) dbg_sink += xv[c];
            dbg_sink += (double)lvraw;
            return;
        }
        const int64_t row = t0 + tid;
        const bool inr = row < r1;
        uint32_t nn = 0, infb = 0;
#pragma unroll
        for (int c = 0; c < ZW - 1; ++c) {
            double x = xv[c];
            const double l = prm[0][c], h = prm[1][c];
            if (x < l) x = l;   // pandas clip semantics: NaN stays, NaN bound ignored
            if (x > h) x = h;
            const bool ok = c < ncols && inr && !isnan(x);
            nn |= ok ? 1u << c : 0u;
            infb |= (ok && isinf(x)) ? 1u << c : 0u;
            xv[c] = x;
        }
        uint32_t pat = 0;
        for (int m = 0; m < nmodels; ++m)
            if ((nn & mmask[m]) == mmask[m]) pat |= 1u << m;
        const int pid = inr ? (int)lut[pat] : 255;
        int bucket = -1;
        if (pid != 255) {
            const int lvl = lvraw < nlevels ? lvraw : nlevels - 1;
            bucket = pid * nlevels + lvl;
        }
        if (infb != 0 && bucket >= 0) {
            for (int m = 0; m < nmodels; ++m) {
                if (!((pat >> m) & 1u)) continue;
                if (infb & mmask[m] & ~ymask[m]) fl |= 1u << (2 * m);
                if (infb & ymask[m]) fl |= 1u << (2 * m + 1);
            }
        }
        // ---- counting sort of the tile by bucket (wave ballots; deterministic order)
        int rank = 0;
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            const uint64_t mb = __ballot(bucket == b);
            if (bucket == b) rank = mask_rank(mb);
            if (lane == 0) wcnt[w][b] = __popcll(mb);
        }
        __syncthreads();
        if (w == 0) {
            // bucket offsets, each bucket padded to a multiple of 4 rows (lane b = bucket b)
            int c0 = 0, c1 = 0, c2 = 0, c3 = 0;
            if (lane < NB) {
                c0 = wcnt[0][lane];
                c1 = wcnt[1][lane];
                c2 = wcnt[2][lane];
                c3 = wcnt[3][lane];
            }
            const int tot = c0 + c1 + c2 + c3;
            const int pad = (tot + 3) & ~3;
            int x = pad;
#pragma unroll
            for (int o = 1; o < 32; o <<= 1) {
                const int y = __shfl_up(x, o, WAVE);
                if (lane >= o) x += y;
            }
            const int off = x - pad;
            if (lane < NB) {
                boff[lane] = off;
                btot[lane] = tot;
                woff[0][lane] = off;
                woff[1][lane] = off + c0;
                woff[2][lane] = off + c0 + c1;
                woff[3][lane] = off + c0 + c1 + c2;
            }
            if (lane == NB - 1) boff[NB] = off + pad;
        }
        __syncthreads();
        if (bucket >= 0) {
            // z = [1, (x - shift) * inv_scale ..., 0 pad], NaN -> 0
            double* dst = tile + (woff[w][bucket] + rank) * RS;
            dst[0] = 1.0;
#pragma unroll
            for (int c = 0; c < ZW - 1; ++c)
                dst[1 + c] = ((nn >> c) & 1u) ? (xv[c] - prm[2][c]) * prm[3][c] : 0.0;
        }
        if (tid < NB * 3) {
            const int b = tid / 3, k = tid - 3 * (tid / 3);
            const int rp = boff[b] + btot[b] + k;
            if (rp < boff[b + 1]) {
#pragma unroll
                for (int c = 0; c < ZW; ++c) tile[rp * RS + c] = 0.0;
            }
        }
        __syncthreads();
        // ---- MFMA accumulation.  Wave w takes the contiguous quarter [W0, W1) of the sorted
        // tile's 4-row groups, so it touches only the few buckets that overlap it (one LDS
        // wait per bucket, not per bucket of the whole tile) and the waves stay balanced to
        // one group.  Bucket bounds live in SGPRs via readlane; accumulators are indexed
        // statically, so the bucket loop is unrolled and skips the buckets outside the range.
        const int bo = lane <= NB ? boff[lane] : 0;
        const int gtot = __builtin_amdgcn_readlane(bo, NB) >> 2;
        const int W0 = (gtot * w) / GNW, W1 = (gtot * (w + 1)) / GNW;
        const double* base = tile + sub * RS + col;
#pragma unroll
        for (int b = 0; b < (DBG == 2 ? 0 : NB); ++b) {
            const int gb0 = __builtin_amdgcn_readlane(bo, b) >> 2;
            const int gb1 = __builtin_amdgcn_readlane(bo, b + 1) >> 2;
            const int g0 = gb0 > W0 ? gb0 : W0;
            const int g1 = gb1 < W1 ? gb1 : W1;
            if (g0 >= g1) continue;
            // 4 groups per trip: the LDS operand reads are issued together so one wait covers
            // four MFMAs
            int g = g0;
            for (; g + 3 < g1; g += 4) {
                double x0[4], x1[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const double* rp = base + 4 * (g + u) * RS;
                    x0[u] = rp[0];
                    x1[u] = NT == 2 ? rp[16] : 0.0;
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    acc0[b] = __builtin_amdgcn_mfma_f64_16x16x4f64(x0[u], x0[u], acc0[b], 0, 0, 0);
                    if (NT == 2) {
                        acc1[b] = __builtin_amdgcn_mfma_f64_16x16x4f64(x0[u], x1[u], acc1[b], 0, 0, 0);
                        acc2[b] = __builtin_amdgcn_mfma_f64_16x16x4f64(x1[u], x1[u], acc2[b], 0, 0, 0);
                    }
                }
            }
            for (; g < g1; ++g) {
                const double* rp = base + 4 * g * RS;
                const double x0 = rp[0];
                const double x1 = NT == 2 ? rp[16] : 0.0;
                acc0[b] = __builtin_amdgcn_mfma_f64_16x16x4f64(x0, x0, acc0[b], 0, 0, 0);
                if (NT == 2) {
                    acc1[b] = __builtin_amdgcn_mfma_f64_16x16x4f64(x0, x1, acc1[b], 0, 0, 0);
                    acc2[b] = __builtin_amdgcn_mfma_f64_16x16x4f64(x1, x1, acc2[b], 0, 0, 0);
                }
            }
        }
        __syncthreads();
    };

    double xa[ZW - 1], xb[ZW - 1];
    int la = 0, lb = 0;
    load_tile(xa, la, r0);
    if (tid < 128) prm[tid >> 5][tid & 31] = pv;
    if (tid < 64) lut[tid] = (uint8_t)lutv;
    if (tid < nmodels) {
        mmask[tid] = (uint32_t)mmv;
        ymask[tid] = (uint32_t)ymv;
    }
    __syncthreads();
    for (int64_t t0 = r0; t0 < r1;) {
        if (PF) load_tile(xb, lb, t0 + GT);
        process_tile(xa, la, t0);
        t0 += GT;
        if (t0 >= r1) break;
        if (!PF) load_tile(xb, lb, t0);
        if (PF) load_tile(xa, la, t0 + GT);
        process_tile(xb, lb, t0);
        t0 += GT;
        if (!PF && t0 < r1) load_tile(xa, la, t0);
    }

    if (DBG == 1 && dbg_sink == 12345.678) a.partial[0] = dbg_sink;
    // ---- inf flags (rare): one atomic per wave per model
    const uint32_t wf = wave_or_u32(fl);
    if (lane == 0 && wf != 0) {
        for (int m = 0; m < nmodels; ++m) {
            uint32_t bits = 0;
            if ((wf >> (2 * m)) & 1u) bits |= FM_ST_INF_IN_X;
            if ((wf >> (2 * m + 1)) & 1u) bits |= FM_ST_INF_IN_Y;
            if (bits) atomicOr(&a.flags[(int64_t)seg * nmodels + m], bits);
        }
    }

    // ---- cross-wave reduction and store: partial[chunk][bucket][packed upper triangle]
    // (ZW*(ZW+1)/2 doubles per bucket: Z'Z is symmetric, half the bytes of a full tile)
    constexpr int PK = ZW * (ZW + 1) / 2;
    constexpr int ZZ = ZW * ZW;
    constexpr int NBATCH = TILE / (GNW * ZZ) < NB ? TILE / (GNW * ZZ) : NB;   // buckets per LDS pass
    const int nbr = a.npatterns * nlevels;
    double* outp = a.partial + (int64_t)chunk * nbr * PK;
#pragma unroll
    for (int b0 = 0; b0 < NB; b0 += NBATCH) {
        if (b0 >= nbr) break;   // block-uniform
#pragma unroll
        for (int bb = 0; bb < NBATCH; ++bb) {
            const int b = b0 + bb;
            if (b >= NB) continue;
            double* red = tile + (bb * GNW + w) * ZZ;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = sub + 4 * r;
                red[i * ZW + col] = acc0[b][r];
                if (NT == 2) {
                    red[i * ZW + 16 + col] = acc1[b][r];
                    red[(16 + i) * ZW + 16 + col] = acc2[b][r];
                }
            }
        }
        __syncthreads();
        for (int e = tid; e < NBATCH * ZZ; e += GT) {
            const int bb = e / ZZ, f = e - bb * ZZ;
            const int i = f / ZW, j = f - i * ZW;
            const int b = b0 + bb;
            if (b < nbr && i <= j) {
                double s = tile[bb * GNW * ZZ + f];
#pragma unroll
                for (int ww = 1; ww < GNW; ++ww) s += tile[(bb * GNW + ww) * ZZ + f];
                outp[(int64_t)b * PK + i * ZW - (i * (i - 1)) / 2 + (j - i)] = s;
            }
        }
        __syncthreads();
    }
}

template <int NT, int NB, int MINW>
void launch_gram(const fm_gram_args& a, hipStream_t st) {
    // FM_GRAM_PREFETCH=0 selects the non-pipelined variant (A/B measurements)
    static const int pf = [] {
        const char* e = getenv("FM_GRAM_PREFETCH");
        return e ? atoi(e) : 1;
    }();
    static const int dbg = [] {
        const char* e = getenv("FM_GRAM_DEBUG");
        return e ? atoi(e) : 0;
    }();
    if (NT == 1 && NB == 16 && dbg == 1)
        hipLaunchKernelGGL((gram_kernel<NT, NB, MINW, true, 1>), dim3(a.nchunks), dim3(GT), 0, st, a);
    else if (NT == 1 && NB == 16 && dbg == 2)
        hipLaunchKernelGGL((gram_kernel<NT, NB, MINW, true, 2>), dim3(a.nchunks), dim3(GT), 0, st, a);
    else if (pf)
        hipLaunchKernelGGL((gram_kernel<NT, NB, MINW, true>), dim3(a.nchunks), dim3(GT), 0, st, a);
    else
        hipLaunchKernelGGL((gram_kernel<NT, NB, MINW, false>), dim3(a.nchunks), dim3(GT), 0, st, a);
}

}  // namespace
}  // namespace fm

extern "C" int fm_gram(const fm_gram_args* args, void* stream) {
    using namespace fm;
    FM_REQUIRE(args != nullptr, "fm_gram: null args");
    const fm_gram_args& a = *args;
    FM_REQUIRE(a.cols && a.seg_off && a.chunk_seg && a.chunk_row && a.partial && a.flags &&
                   a.model_mask && a.model_ymask && a.pattern_id,
               "fm_gram: null pointer");
    FM_REQUIRE(a.ncols >= 1 && a.ncols <= FM_MAX_COLS, "fm_gram: ncols must be 1..%d", FM_MAX_COLS);
    FM_REQUIRE(a.nmodels >= 1 && a.nmodels <= FM_MAX_MODELS, "fm_gram: nmodels must be 1..%d",
               FM_MAX_MODELS);
    FM_REQUIRE(a.nlevels >= 1 && a.nlevels <= FM_MAX_LEVELS, "fm_gram: nlevels must be 1..%d",
               FM_MAX_LEVELS);
    FM_REQUIRE(a.npatterns >= 1, "fm_gram: npatterns must be >= 1");
    if (a.nchunks == 0) return FM_OK;
    const int nb = a.npatterns * a.nlevels;
    hipStream_t st = (hipStream_t)stream;
    if (a.ncols <= 15) {
        if (nb <= 1) launch_gram<1, 1, 2>(a, st);
        else if (nb <= 4) launch_gram<1, 4, 2>(a, st);
        else if (nb <= 8) launch_gram<1, 8, 2>(a, st);
        else if (nb <= 16) launch_gram<1, 16, 2>(a, st);
        else {
            set_error("fm_gram: %d buckets exceed 16 for <=15 columns", nb);
            return FM_ETOOBIG;
        }
    } else {
        if (nb <= 1) launch_gram<2, 1, 1>(a, st);
        else if (nb <= 4) launch_gram<2, 4, 1>(a, st);
        else if (nb <= 8) launch_gram<2, 8, 1>(a, st);
        else {
            set_error("fm_gram: %d buckets exceed 8 for >15 columns", nb);
            return FM_ETOOBIG;
        }
    }
    FM_CHECK_LAUNCH("fm_gram");
    return FM_OK;
}

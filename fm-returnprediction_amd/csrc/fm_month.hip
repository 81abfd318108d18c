// fm_month_pass: the winsorize cuts AND the batched Gram of a whole month in ONE workgroup,
// so the month's panel rows are fetched from HBM once (the Gram phase re-reads the rows the
// cut phase has just streamed: they are still in the XCD L2 / Infinity Cache) and no
// per-(column, month) cut table makes a round trip through HBM between two launches.
//
// Replaces, for every month: np.percentile(vals, 1/99) + clip of every winsorized column
// (reference src/calc_Lewellen_2014.py:519-524), the `.dropna()` row filter and universe
// subsetting (src/regressions.py:39, src/calc_Lewellen_2014.py:95-105) and the X'X / X'y /
// y'y formation inside sm.OLS (src/regressions.py:57, :917-919) for all models x universes.
//
// One 256-thread workgroup (4 waves) per month:
//   cut phase   wave w takes columns w, w+4, ...: the whole month column in registers
//               (VPL values per lane, one coalesced read; the next column's loads are
//               issued as soon as this column's tail candidates sit in LDS), exact tail
//               order statistics by wave_cut (fm_select_dev.h) -> lo / hi / pivot in LDS
//               and in HBM ([ncols][nseg]: fm_solve, fm_solve_fixup and fm_const_check read
//               them).  A column the one-wave path cannot decide is redone exactly by the
//               whole workgroup (select_unit_wg, radix select) before the Gram phase.
//   Gram phase  fm_gram_dev.h's GramWave over the month's rows with the cuts from LDS
//               (clip, validity pattern x universe level -> bucket, FP64 MFMA), then the
//               cross-wave sum -> partial[month][bucket][136].
// Two workgroups per CU (<= 256 VGPRs): one's cut phase (VALU / sorts) overlaps the other's
// Gram phase (MFMA / LDS) and both keep HBM loads in flight.
#include <math.h>
#include <stdlib.h>

#include "fm_common.h"
#include "fm_gram_dev.h"
#include "fm_select_dev.h"

namespace fm {
namespace {

constexpr int MT = 256;
constexpr int MNW = MT / WAVE;

struct MonthSmem {
    union {
        double tile[MNW * GramShape<1>::WT];   // Gram phase: the waves' sorted row tiles
        double cand[MNW][2][WCAP];             // cut phase: per wave lower / upper candidates
        SelSmem wg;                            // exact workgroup fallback of one column
    } u;
    double zblk[4 * GramShape<1>::RS];         // four zero rows (padded MFMA groups)
    double prm[4][32];                         // lo, hi, pivot, scale (1) per column
    uint8_t lut[64];
    uint32_t fail;                             // columns the one-wave path left undecided
};

template <int VPL, int NB, int MINW>
__global__ __launch_bounds__(MT, MINW) void month_kernel(fm_month_args ma) {
    const fm_gram_args& a = ma.gram;
    __shared__ MonthSmem sm;
    const int tid = threadIdx.x, lane = tid & (WAVE - 1);
    const int w = __builtin_amdgcn_readfirstlane(tid / WAVE);
    const int s = blockIdx.x;
    const int64_t r0 = a.seg_off[s], r1 = a.seg_off[s + 1];
    const int L = (int)(r1 - r0);
    const int ncols = a.ncols, nseg = a.nseg;
    const int64_t cs = a.col_stride;

    // ---- cut phase: this wave's first column is in flight before any shared state is set
    double xv[VPL];
    int c = w;
    if (c < ncols) load_seg_col<VPL>(a.cols + (int64_t)c * cs + r0, L, xv);
    {
        const int npat = 1 << a.nmodels;
        const int lutv = a.pattern_id[tid < npat ? tid : 0];
        if (tid < 64) sm.lut[tid] = (uint8_t)lutv;
        for (int e = tid; e < 4 * GramShape<1>::RS; e += MT) sm.zblk[e] = 0.0;
        if (tid < 128) {
            // columns past ncols: no cut, pivot 0 (their z is never read by fm_solve)
            const int k = tid >> 5, cc = tid & 31;
            if (cc >= ncols) sm.prm[k][cc] = k < 2 ? NAN : 0.0;
            sm.prm[3][tid & 31] = 1.0;
        }
        if (tid == 0) sm.fail = 0u;
    }
    __syncthreads();
    while (c < ncols) {
        const int cn = c + MNW;
        const WaveCut r = wave_cut<VPL>(xv, L, ma.q_lo, ma.q_hi, ma.min_count, 0, sm.u.cand[w][0],
                                        sm.u.cand[w][1], [&] {
                                            if (cn < ncols) load_seg_col<VPL>(a.cols + (int64_t)cn * cs + r0, L, xv);
                                        });
        if (lane == 0) {
            if (r.ok) {
                const int64_t o = (int64_t)c * nseg + s;
                sm.prm[0][c] = r.lo;
                sm.prm[1][c] = r.hi;
                sm.prm[2][c] = r.cen;
                ma.lo[o] = r.lo;
                ma.hi[o] = r.hi;
                ma.center[o] = r.cen;
                if (ma.nvalid) ma.nvalid[o] = r.n;
            } else {
                atomicOr(&sm.fail, 1u << c);
            }
        }
        c = cn;
    }
    __syncthreads();
    uint32_t fail = sm.fail;   // block-uniform
    if (fail) {
        // rare: ranks >= 64 (short-tailed huge months never reach here: VPL <= 96), or a
        // candidate overflow (many ties just inside a tail); exact radix select by the
        // whole workgroup, one column at a time
        constexpr int VPT = (VPL * WAVE + MT - 1) / MT;
        SelArgs sa{a.cols, cs,      a.seg_off, nseg,     ncols,   nullptr,  ma.q_lo,
                   ma.q_hi, ma.min_count, 0,  ma.lo,    ma.hi,   ma.nvalid, nullptr,
                   nullptr, ma.center, &sm.prm[0][0]};
        while (fail) {
            const int cc = __builtin_ctz(fail);
            fail &= fail - 1u;
            __syncthreads();
            select_unit_wg<VPT>(sa, s, cc, sm.u.wg);
        }
        __syncthreads();
    }
    // ---- Gram phase
    GramWave<1, NB, MNW> g(a, r0, r1, w);
    g.prefetch();
    __syncthreads();   // cuts complete; the candidate lists are dead (tile aliases them)
    g.run(sm.prm, sm.lut, false, sm.u.tile, sm.zblk);
    const int nbr = a.npatterns * a.nlevels;
    g.epilogue(sm.u.tile, a.partial + (int64_t)s * nbr * GramShape<1>::PK, nbr);
}

template <int VPL, int NB>
void launch_month(const fm_month_args& a, hipStream_t st) {
    hipLaunchKernelGGL((month_kernel<VPL, NB, 2>), dim3(a.gram.nseg), dim3(MT), 0, st, a);
}

template <int VPL>
int launch_month_nb(const fm_month_args& a, int nb, hipStream_t st) {
    if (nb <= 4) launch_month<VPL, 4>(a, st);
    else if (nb <= 8) launch_month<VPL, 8>(a, st);
    else if (nb <= 12) launch_month<VPL, 12>(a, st);
    else if (nb <= 15) launch_month<VPL, 15>(a, st);   // 5 patterns x 3 universes (Table 2)
    else launch_month<VPL, 16>(a, st);
    return FM_OK;
}

}  // namespace
}  // namespace fm

extern "C" int fm_month_pass(const fm_month_args* args, void* stream) {
    using namespace fm;
    FM_REQUIRE(args != nullptr, "fm_month_pass: null args");
    const fm_month_args& m = *args;
    const fm_gram_args& a = m.gram;
    FM_REQUIRE(a.cols && a.seg_off && a.partial && a.model_mask && a.pattern_id && m.lo && m.hi && m.center,
               "fm_month_pass: null pointer");
    FM_REQUIRE(a.nmodels >= 1 && a.nmodels <= FM_MAX_MODELS, "fm_month_pass: nmodels must be 1..%d",
               FM_MAX_MODELS);
    FM_REQUIRE(a.nlevels >= 1 && a.nlevels <= FM_MAX_LEVELS, "fm_month_pass: nlevels must be 1..%d",
               FM_MAX_LEVELS);
    FM_REQUIRE(a.npatterns >= 1 && a.ncols >= 1 && a.nseg >= 0 && m.max_seg_len >= 0,
               "fm_month_pass: bad sizes");
    FM_REQUIRE(m.q_lo >= 0.0 && m.q_lo <= 1.0 && m.q_hi >= 0.0 && m.q_hi <= 1.0,
               "fm_month_pass: quantiles must be in [0,1]");
    const int nb = a.npatterns * a.nlevels;
    if (a.ncols > 15 || nb > 16 || m.max_seg_len > FM_MONTH_MAX_ROWS) {
        set_error("fm_month_pass: %d columns / %d buckets / %d-row months exceed the fused pass "
                  "(<= 15 / 16 / %d); use fm_select + fm_gram",
                  a.ncols, nb, m.max_seg_len, FM_MONTH_MAX_ROWS);
        return FM_ETOOBIG;
    }
    if (a.nseg == 0) return FM_OK;
    hipStream_t st = (hipStream_t)stream;
    const int vpl = (m.max_seg_len + WAVE - 1) / WAVE;
    if (vpl <= 16) launch_month_nb<16>(m, nb, st);
    else if (vpl <= 32) launch_month_nb<32>(m, nb, st);
    else if (vpl <= 48) launch_month_nb<48>(m, nb, st);
    else if (vpl <= 64) launch_month_nb<64>(m, nb, st);
    else if (vpl <= 80) launch_month_nb<80>(m, nb, st);
    else launch_month_nb<96>(m, nb, st);
    FM_CHECK_LAUNCH("fm_month_pass");
    return FM_OK;
}

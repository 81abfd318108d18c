// fm_gram: clip -> dropna-validity -> shifted Gram accumulation on FP64 MFMA.
//
// Replaces, for every (month, model, universe) problem at once, the row filtering of
// run_monthly_cs_regressions (`.dropna()`, reference src/regressions.py:39), the universe
// subsetting of get_subsets (src/calc_Lewellen_2014.py:95-105) and the X'X / X'y / y'y
// formation inside sm.OLS (src/regressions.py:57, src/calc_Lewellen_2014.py:917-919).
//
// One workgroup (256 threads = 4 waves) per chunk of one month; the waves work
// independently on 64-row tiles (fm_gram_dev.h: validity pattern x universe level ->
// bucket, wave counting sort into LDS, v_mfma_f64_4x4x4_4b accumulation per bucket) and
// sum their accumulators through LDS at chunk end into one packed upper-triangular Gram
// per (chunk, bucket).  fm_solve combines buckets into problems: model m's Gram is the sum
// over patterns that contain m and levels >= the problem's universe, restricted to m's
// columns.  One HBM read of the panel serves every model x universe.
#include <math.h>
#include <stdlib.h>

#include "fm_common.h"
#include "fm_gram_dev.h"

namespace fm {
namespace {

constexpr int GT = 256;
constexpr int GNW = GT / WAVE;
#ifndef FM_GRAM_MINW
#define FM_GRAM_MINW (FM_GRAM_PF2 ? 2 : 3)
#endif
constexpr int GRAM_MINW = FM_GRAM_MINW;   // waves per SIMD the register budget allows
#ifndef FM_GRAM_WGTIME
#define FM_GRAM_WGTIME 0   // probe builds only (tools/gram_wgtime.py): per-workgroup start / end
#endif                     // times and hardware id (never the shipped library)
#if FM_GRAM_WGTIME
constexpr int WGT_MAX = 1 << 16;
__device__ uint32_t g_wgtime[4 * WGT_MAX];   // the probe's own buffer, bounds-checked
#endif

// One workgroup per chunk (normally a whole month: the chunk plan makes chunks as large as
// the chip's resident workgroup slots allow, so the prologue and the cross-wave epilogue run
// once per month and every wave streams ~20 tiles back to back).  MINW = waves per SIMD.
template <int NT, int NB, int MINW, bool PL, bool FULLC>
__global__ __launch_bounds__(GT, MINW) void gram_kernel(fm_gram_args a) {
    using S = GramShape<NT>;
    __shared__ double tile[GNW * S::WT];
    __shared__ double zblk[4 * S::RS];      // four zero rows: operands of padded group slots
    __shared__ double prm[4][32];
    __shared__ uint8_t lut[64];

    const int tid = threadIdx.x;
    const int w = __builtin_amdgcn_readfirstlane(tid / WAVE);   // wave-uniform (SGPR loops)
    const int ncols = a.ncols, nseg = a.nseg;
    const int nbr = a.npatterns * a.nlevels;
#if FM_GRAM_WGTIME
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
#endif
    // default order last-first: fm_select streams the panel month by month, so the months it
    // read last are still in the memory-side cache when they are read here; with a
    // chunk_order (the split-month plan) the big chunks go first, the small ones fill in; with
    // a balanced plan (wg_chunk_off) workgroup b takes its run of consecutive chunks
    int c0, c1;
    if (a.wg_chunk_off != nullptr) {
        const int b = (int)gridDim.x - 1 - (int)blockIdx.x;
        c0 = a.wg_chunk_off[b];
        c1 = a.wg_chunk_off[b + 1];
    } else {
        c0 = a.chunk_order ? a.chunk_order[blockIdx.x] : (int)gridDim.x - 1 - (int)blockIdx.x;
        c1 = c0 + 1;
    }
    const int npat = 1 << a.nmodels;
    const int lutv = a.pattern_id[tid < npat ? tid : 0];
    for (int chunk = c0; chunk < c1; ++chunk) {
        const int seg = a.chunk_seg[chunk];
        const int64_t r0 = a.chunk_row[2 * chunk], r1 = a.chunk_row[2 * chunk + 1];
        // Prologue loads (month parameters) are unconditional (pointer/index selected, value
        // masked after) and issued before the first tile's row loads, so waiting for them does
        // not wait for the tile.
        double pv;
        {
            const int kind = tid >> 5, c = tid & 31;
            const double* src = kind == 0 ? a.lo : kind == 1 ? a.hi : kind == 2 ? a.shift : a.inv_scale;
            const bool on = tid < 128 && c < ncols && src != nullptr;
            // a valid dummy address when off (the FP64 columns may be absent on a split panel)
            const double* pp = on ? src + (int64_t)c * nseg + seg : (const double*)a.seg_off;
            const double v = *pp;
            const double dflt = kind < 2 ? NAN : (kind == 2 ? 0.0 : 1.0);
            pv = on ? v : dflt;
        }
        GramWave<NT, NB, GNW, PL, FULLC> g(a, r0, r1, w);
        g.prefetch();
        if (chunk == c0) {
            for (int e = tid; e < 4 * S::RS; e += GT) zblk[e] = 0.0;
            if (tid < 64) lut[tid] = (uint8_t)lutv;
        }
        if (tid < 128) prm[tid >> 5][tid & 31] = pv;   // the previous chunk's epilogue ended in a barrier
        __syncthreads();
        g.run(prm, lut, a.inv_scale != nullptr, tile, zblk);
        g.epilogue(tile, a.partial + (int64_t)chunk * nbr * S::PK, nbr);
    }
#if FM_GRAM_WGTIME
    if (tid == 0 && blockIdx.x < WGT_MAX) {
        const uint64_t t_end = __builtin_amdgcn_s_memrealtime();
        uint32_t* f = g_wgtime + 4 * (int64_t)blockIdx.x;
        f[0] = (uint32_t)t_start;
        f[1] = (uint32_t)t_end;
        f[2] = (uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_ID
        f[3] = (uint32_t)(c1 - c0);
    }
#endif
}

template <int NT, int NB, int MINW>
void launch_gram(const fm_gram_args& a, hipStream_t st) {
    const int grid = a.wg_chunk_off != nullptr ? a.nwg : a.nchunks;
    // ncols == ZW - 1 (the Table-2 panel's 15 columns): the row loads step through the columns
    // without the "past ncols" test (the Gram's scalar stream had 4 instructions per column
    // and plane for it)
    const bool full = a.ncols == 16 * NT - 1;
    if (a.hi_plane != nullptr) {
        if (full) hipLaunchKernelGGL((gram_kernel<NT, NB, MINW, true, true>), dim3(grid), dim3(GT), 0, st, a);
        else hipLaunchKernelGGL((gram_kernel<NT, NB, MINW, true, false>), dim3(grid), dim3(GT), 0, st, a);
    } else {
        if (full) hipLaunchKernelGGL((gram_kernel<NT, NB, MINW, false, true>), dim3(grid), dim3(GT), 0, st, a);
        else hipLaunchKernelGGL((gram_kernel<NT, NB, MINW, false, false>), dim3(grid), dim3(GT), 0, st, a);
    }
}

}  // namespace
}  // namespace fm

#if FM_GRAM_WGTIME
extern "C" int fm_gram_wgtime_copy(uint32_t* host, int32_t n) {   // probe builds only
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(fm::g_wgtime), (size_t)4 * (n < fm::WGT_MAX ? n : fm::WGT_MAX) * 4) ==
                   hipSuccess ? 0 : -1;
}
#endif

extern "C" int fm_gram(const fm_gram_args* args, void* stream) {
    using namespace fm;
    FM_REQUIRE(args != nullptr, "fm_gram: null args");
    const fm_gram_args& a = *args;
    FM_REQUIRE((a.cols || a.hi_plane) && a.seg_off && a.chunk_seg && a.chunk_row && a.partial && a.flags &&
                   a.model_mask && a.model_ymask && a.pattern_id,
               "fm_gram: null pointer");
    FM_REQUIRE(a.ncols >= 1 && a.ncols <= FM_MAX_COLS, "fm_gram: ncols must be 1..%d", FM_MAX_COLS);
    FM_REQUIRE((a.hi_plane == nullptr) == (a.lo_plane == nullptr) && (a.hi_plane == nullptr || a.plane_stride > 0),
               "fm_gram: hi_plane and lo_plane go together (plane_stride > 0)");
    FM_REQUIRE(a.nmodels >= 1 && a.nmodels <= FM_MAX_MODELS, "fm_gram: nmodels must be 1..%d",
               FM_MAX_MODELS);
    FM_REQUIRE(a.nlevels >= 1 && a.nlevels <= FM_MAX_LEVELS, "fm_gram: nlevels must be 1..%d",
               FM_MAX_LEVELS);
    FM_REQUIRE(a.npatterns >= 1, "fm_gram: npatterns must be >= 1");
    if (a.nchunks == 0) return FM_OK;
    FM_REQUIRE(a.wg_chunk_off == nullptr || (a.nwg >= 1 && a.chunk_order == nullptr),
               "fm_gram: a balanced plan needs nwg >= 1 and no chunk_order");
    const int nb = a.npatterns * a.nlevels;
    hipStream_t st = (hipStream_t)stream;
    if (a.ncols <= 15) {
        if (nb <= 1) launch_gram<1, 1, GRAM_MINW>(a, st);
        else if (nb <= 4) launch_gram<1, 4, GRAM_MINW>(a, st);
        else if (nb <= 8) launch_gram<1, 8, GRAM_MINW>(a, st);
        else if (nb <= 12) launch_gram<1, 12, GRAM_MINW>(a, st);
        else if (nb <= 15) launch_gram<1, 15, GRAM_MINW>(a, st);   // 5 patterns x 3 universes (Table 2)
        else if (nb <= 16) launch_gram<1, 16, GRAM_MINW>(a, st);
        else {
            set_error("fm_gram: %d buckets exceed 16 for <=15 columns", nb);
            return FM_ETOOBIG;
        }
    } else {
        if (nb <= 1) launch_gram<2, 1, 2>(a, st);
        else if (nb <= 4) launch_gram<2, 4, 2>(a, st);
        else if (nb <= 8) launch_gram<2, 8, 2>(a, st);
        else {
            set_error("fm_gram: %d buckets exceed 8 for >15 columns", nb);
            return FM_ETOOBIG;
        }
    }
    FM_CHECK_LAUNCH("fm_gram");
    return FM_OK;
}

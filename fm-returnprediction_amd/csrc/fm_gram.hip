// fm_gram: clip -> dropna-validity -> shifted Gram accumulation on FP64 MFMA.
//
// Replaces, for every (month, model, universe) problem at once, the row filtering of
// run_monthly_cs_regressions (`.dropna()`, reference src/regressions.py:39), the universe
// subsetting of get_subsets (src/calc_Lewellen_2014.py:95-105) and the X'X / X'y / y'y
// formation inside sm.OLS (src/regressions.py:57, src/calc_Lewellen_2014.py:917-919).
//
// One workgroup (256 threads = 4 waves) per chunk of one month.  The waves work
// independently (no workgroup barrier inside the row loop): wave w takes the 64-row tiles
// w, w+4, w+8, ... of the chunk, and per tile
//   1. each lane streams one row: ncols coalesced FP64 loads (SoA; the next tile's loads are
//      in flight while this one is processed), clip to the month's winsorize cuts, NaN/inf
//      tests, shift by the month's pivot (optional standardize scale), z = [1, x..., y] with
//      NaN -> 0;
//   2. the row's validity pattern (bit m: every column model m needs is non-NaN) and its
//      universe level give a bucket id; per bucket one wave ballot gives the bucket's row
//      count (SGPR) and the lane's rank, so the counting sort needs no LDS counters; each
//      lane writes its z row to the wave's private LDS tile at (bucket offset + rank);
//   3. per bucket, v_mfma_f64_4x4x4_4b (__builtin_amdgcn_mfma_f64_4x4x4f64, four 4x4
//      blocks per instruction) with A = B = 4 rows of that bucket accumulates Z^T Z in
//      registers: three instructions per 4-row group cover the 16x16 Gram (block pairs, see
//      BlockPairs below; rows past the bucket's count read the zero rows).
// At chunk end the four waves' accumulators are summed through LDS and written as one
// packed upper-triangular Gram per (chunk, bucket).  fm_solve combines buckets into
// problems: model m's Gram is the sum over patterns that contain m and levels >= the
// problem's universe, restricted to m's columns.  One HBM read of the panel serves every
// model x universe.
#include <math.h>
#include <stdlib.h>

#include "fm_common.h"

namespace fm {
namespace {

constexpr int GT = 256;
constexpr int GNW = GT / WAVE;

typedef double d4 __attribute__((ext_vector_type(4)));

// nn = 2 * nn + (x is not NaN): one compare + one add-with-carry
__device__ __forceinline__ uint32_t push_valid(uint32_t nn, double x) {
    asm("v_cmp_o_f64 vcc, %1, %1\n\tv_addc_co_u32 %0, vcc, %0, %0, vcc" : "+v"(nn) : "v"(x) : "vcc");
    return nn;
}

// 4x4 block pairs (I, J) of the ZW x ZW Gram covered by the 4x4x4 MFMAs of one 4-row group.
// v_mfma_f64_4x4x4_4b: lane l = x + 4*blk + 16*k holds A[blk][x][k] and B[blk][k][x], and
// D[blk][i][j] lands at lane j + 4*blk + 16*i.
//  * NT == 1 (16 columns): "rotation" cover.  Instruction k pairs block row blk with block
//    column (blk + k) % 4, k = 0..2: the diagonal blocks, the 4 blocks one step off (one of
//    them transposed) and the 2 blocks two steps off (computed twice).  Every lane's A
//    operand is z[row][q] (q = lane & 15) for all three instructions and its B operands are
//    z[row][q + 4k] with the row's columns 0..7 repeated at 16..23 in LDS, so one address
//    VGPR serves all three reads (immediate offsets).
//  * NT == 2 (32 columns): the 36 upper pairs in row order, 4 per instruction (9), A / B
//    column offsets per lane from the table.
template <int NBLK>
struct BlockPairs {
    static constexpr int P = NBLK * (NBLK + 1) / 2;
    static constexpr int NI = (P + 3) / 4;
    int I[NI * 4], J[NI * 4];
    constexpr BlockPairs() : I(), J() {
        int p = 0;
        for (int i = 0; i < NBLK; ++i)
            for (int j = i; j < NBLK; ++j) {
                I[p] = i;
                J[p] = j;
                ++p;
            }
        for (; p < NI * 4; ++p) I[p] = J[p] = 0;
    }
};

// One workgroup per chunk (normally a whole month: the chunk plan makes chunks as large as
// the chip's resident workgroup slots allow, so the prologue and the cross-wave epilogue run
// once per month and every wave streams ~20 tiles back to back).  MINW = waves per SIMD.
template <int NT, int NB, int MINW>
__global__ __launch_bounds__(GT, MINW) void gram_kernel(fm_gram_args a) {
    constexpr int ZW = 16 * NT;
    constexpr int RS = ZW + 1;              // LDS row stride (doubles): conflict-free scatter
    constexpr int TR = WAVE;                // rows per wave tile (one per lane)
    constexpr int WT = TR * RS;             // one wave's sorted tile
    constexpr int PK = ZW * (ZW + 1) / 2;   // packed upper triangle
    constexpr BlockPairs<4 * NT> BP{};
    constexpr int NI = NT == 1 ? 3 : BlockPairs<8>::NI;   // 4x4x4 MFMAs per 4-row group
    constexpr int NBATCH = (GNW * WT) / (GNW * PK) < NB ? (GNW * WT) / (GNW * PK) : NB;
    static_assert(NBATCH >= 1, "epilogue image does not fit the tile area");
    __shared__ double tile[GNW * WT];
    __shared__ double zblk[4 * RS];         // four zero rows: operands of padded group slots
    __shared__ double prm[4][32];
    __shared__ uint8_t lut[64];

    const int tid = threadIdx.x;
    const int lane = tid & (WAVE - 1);
    const int w = __builtin_amdgcn_readfirstlane(tid / WAVE);   // wave-uniform (SGPR loops)
    // chunks run last-month-first: fm_select streams the panel month by month, so the
    // months it read last are still in the memory-side cache when they are read here
    const int chunk = (int)gridDim.x - 1 - (int)blockIdx.x;
    const int seg = a.chunk_seg[chunk];
    const int64_t r0 = a.chunk_row[2 * chunk], r1 = a.chunk_row[2 * chunk + 1];
    const int ncols = a.ncols, nseg = a.nseg, nmodels = a.nmodels, nlevels = a.nlevels;
    const int ntile = (int)((r1 - r0 + TR - 1) / TR);
    const bool scaled = a.inv_scale != nullptr;

    // Prologue loads (month parameters, pattern table, model masks) are unconditional
    // (pointer/index selected, value masked after) and issued before the first tile's row
    // loads, so waiting for them does not wait for the tile.
    double pv;
    int lutv, mmv;
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
        const int mi = lane < nmodels ? lane : 0;   // read back per wave by readlane
        mmv = (int)a.model_mask[mi];
    }

    // Row loads: one wave-uniform base per column (s_add in the scalar unit) + the lane's
    // 32-bit row offset, so every load is a global_load with an SGPR base and no per-load
    // address VALU.  Lanes past the chunk end re-read its last row (masked later).  Without
    // universes the level load reads byte 0 of the panel and is masked to 0.
    const uint8_t* lvbase = a.level ? a.level : (const uint8_t*)a.cols;
    const int lvand = a.level ? 0xFF : 0;
    const uint32_t colmask = ncols >= 32 ? ~0u : (1u << ncols) - 1u;
    typedef const __attribute__((address_space(1))) char* gptr;   // global_load, not flat_load
    auto load_row = [&](double (&xv)[ZW - 1], int& lv, int t) {
        const int64_t t0 = r0 + (int64_t)t * TR;
        const int64_t last = r1 - 1 - t0;
        const uint32_t lo = last < 0 ? 0u : (last < lane ? (uint32_t)last : (uint32_t)lane);
        const int64_t tb = last < 0 ? r1 - 1 : t0;   // wave-uniform tile base (clamped)
        const double* cb = a.cols + tb;               // column 0; s_add per column
#pragma unroll
        for (int c = 0; c < ZW - 1; ++c) {
            xv[c] = *(const __attribute__((address_space(1))) double*)((gptr)cb + lo * 8u);
            cb += c + 1 < ncols ? a.col_stride : 0;   // columns past ncols re-read the last
            // opaque to the optimizer: otherwise it turns a repeated address into a register
            // copy of the previous load behind a branch, i.e. a vmcnt(0) wait per column
            asm("" : "+s"(cb));
        }
        // raw byte; masked where it is used (masking here would wait for the load)
        lv = *((gptr)(a.level ? lvbase + tb : lvbase) + (a.level ? lo : 0u));
    };
    double xv[ZW - 1];   // ONE register buffer: the next tile's loads are issued as soon as
    int lv = 0;          // this tile's values sit in LDS, and fly during its MFMAs
    if (w < ntile) load_row(xv, lv, w);

    double acc[NB][NI];
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int k = 0; k < NI; ++k) acc[b][k] = 0.0;
    double* wt = tile + w * WT;   // this wave's sorted tile
    // MFMA operand offsets (lane l = x + 4*blk + 16*kr holds row kr of the 4-row group):
    //  NT 1: A = z[kr][q] (q = l & 15) for all three instructions, B = z[kr][(q + 4k) & 15]
    //  NT 2: A / B columns of block pair 4k + blk from the table
    const int kx = lane & 3, kb = (lane >> 2) & 3, kr = lane >> 4;
    int oa[NI], ob[NI];
#pragma unroll
    for (int k = 0; k < NI; ++k) {
        oa[k] = kr * RS + (NT == 1 ? lane & 15 : 4 * BP.I[4 * k + kb] + kx);
        ob[k] = kr * RS + (NT == 1 ? ((lane & 15) + 4 * k) & 15 : 4 * BP.J[4 * k + kb] + kx);
    }
    for (int e = tid; e < 4 * RS; e += GT) zblk[e] = 0.0;
    if (tid < 128) prm[tid >> 5][tid & 31] = pv;
    if (tid < 64) lut[tid] = (uint8_t)lutv;
    __syncthreads();
    // model column masks in SGPRs (wave-uniform; statically indexed below)
    uint32_t mm[FM_MAX_MODELS];
#pragma unroll
    for (int m = 0; m < FM_MAX_MODELS; ++m)
        mm[m] = (uint32_t)__builtin_amdgcn_readlane(mmv, m < nmodels ? m : 0);

    for (int t = w; t < ntile; t += GNW) {
        const int64_t row = r0 + (int64_t)t * TR + lane;
        // validity bits of the raw values (NaN = missing; clipping never makes or removes
        // a NaN: pandas clip ignores NaN bounds)
        uint32_t nn = 0;
#pragma unroll
        for (int c = ZW - 2; c >= 0; --c) nn = push_valid(nn, xv[c]);
        const bool inr = row < r1;
        nn &= inr ? colmask : 0u;
        uint32_t pat = 0;
#pragma unroll
        for (int m = 0; m < FM_MAX_MODELS; ++m)
            if (m < nmodels && (nn & mm[m]) == mm[m]) pat |= 1u << m;
        const int pid = inr ? (int)lut[pat] : 255;
        const int lvm = lv & lvand;
        const int lvl = lvm < nlevels ? lvm : nlevels - 1;
        const int bucket = pid != 255 ? pid * nlevels + lvl : -1;
        // ---- wave counting sort by bucket, from KB bit ballots: this lane's slot is the
        // number of valid lanes with a smaller bucket plus its rank among equal buckets
        // (bitwise magnitude compare, MSB first); per-bucket counts are scalar.
        constexpr int KB = NB <= 1 ? 0 : NB <= 2 ? 1 : NB <= 4 ? 2 : NB <= 8 ? 3 : 4;
        const bool valid = bucket >= 0;
        const uint64_t bv = __ballot(valid);
        uint64_t bit[KB > 0 ? KB : 1];
#pragma unroll
        for (int i = 0; i < KB; ++i) bit[i] = __ballot(valid && ((bucket >> i) & 1));
        uint32_t eql = (uint32_t)bv, eqh = (uint32_t)(bv >> 32), ltl = 0, lth = 0;
#pragma unroll
        for (int i = KB - 1; i >= 0; --i) {
            const uint32_t tm = 0u - (uint32_t)((bucket >> i) & 1);
            const uint32_t bl = (uint32_t)bit[i], bh = (uint32_t)(bit[i] >> 32);
            ltl |= eql & ~bl & tm;
            lth |= eqh & ~bh & tm;
            eql &= ~(bl ^ tm);
            eqh &= ~(bh ^ tm);
        }
        const int dest = __popc(ltl) + __popc(lth) +
                         (int)__builtin_amdgcn_mbcnt_hi(eqh, __builtin_amdgcn_mbcnt_lo(eql, 0u));
        // z = [1, (clip(x) - shift) * inv_scale ...].  Missing values are NOT zeroed: a
        // column that is NaN in a row belongs to no model of the row's pattern, so the
        // Gram entries it pollutes are never read by fm_solve.  clip = hardware max/min: a
        // NaN bound is ignored, a NaN x gives a don't-care value.  Dropped rows are not
        // stored.
        if (valid) {
            double* dst = wt + dest * RS;
            dst[0] = 1.0;
            if (scaled) {
#pragma unroll
                for (int c = 0; c < ZW - 1; ++c)
                    dst[1 + c] = (hw_min(hw_max(xv[c], prm[0][c]), prm[1][c]) - prm[2][c]) * prm[3][c];
            } else {
#pragma unroll
                for (int c = 0; c < ZW - 1; ++c)
                    dst[1 + c] = hw_min(hw_max(xv[c], prm[0][c]), prm[1][c]) - prm[2][c];
            }
        }
        // this tile's values are consumed: the next tile's loads fly during the MFMAs
        if (t + GNW < ntile) load_row(xv, lv, t + GNW);
        // the operand reads below read other lanes' rows of this wave: LDS executes one
        // wave's DS instructions in order, so only compiler reordering must be prevented
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // ---- MFMA accumulation per bucket: NI independent 4x4x4 block products per 4-row
        // group; in the bucket's last (partial) group the lanes of rows past the count read
        // the zero rows instead.
        // per-bucket counts are popcounts of the ballot masks, formed on the fly (scalar)
        const double* rp = wt;
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            uint64_t mb = bv;
#pragma unroll
            for (int i = 0; i < KB; ++i) mb &= ((b >> i) & 1) ? bit[i] : ~bit[i];
            const int n = (int)__popcll(mb);
            int g = 0;
            for (; g + 4 <= n; g += 4, rp += 4 * RS) {
#pragma unroll
                for (int k = 0; k < NI; ++k)
                    acc[b][k] = __builtin_amdgcn_mfma_f64_4x4x4f64(rp[oa[k]], rp[ob[k]], acc[b][k], 0, 0, 0);
            }
            if (g < n) {
                const double* bp = g + kr < n ? rp : zblk;
#pragma unroll
                for (int k = 0; k < NI; ++k)
                    acc[b][k] = __builtin_amdgcn_mfma_f64_4x4x4f64(bp[oa[k]], bp[ob[k]], acc[b][k], 0, 0, 0);
                rp += (n - g) * RS;
            }
        }
        // the next tile's scatter overwrites this tile: every operand read above has been
        // consumed by its MFMA (data dependence), and the fences keep the order
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }

    // ---- cross-wave reduction and store: partial[chunk][bucket][packed upper triangle].
    // v_mfma_f64_4x4x4f64 leaves D[blk][i][j] in lane j + 4*blk + 16*i; each lane maps its
    // entry of instruction k to the packed index of (min(r, c), max(r, c)), or -1 where the
    // entry is a duplicate (NT 1: the two-step blocks computed twice; diagonal blocks: the
    // strictly lower half), so every packed entry is written exactly once per wave.
    const int nbr = a.npatterns * nlevels;
    double* outp = a.partial + (int64_t)chunk * nbr * PK;
    int od[NI];
#pragma unroll
    for (int k = 0; k < NI; ++k) {
        int r, c;
        bool keep;
        if (NT == 1) {
            r = 4 * kb + kr;
            c = 4 * ((kb + k) & 3) + kx;
            keep = !(k == 2 && kb >= 2) && !(k == 0 && kr > kx);
        } else {
            const int p = 4 * k + kb;
            r = 4 * BP.I[p] + kr;
            c = 4 * BP.J[p] + kx;
            keep = p < BlockPairs<8>::P && !(BP.I[p] == BP.J[p] && kr > kx);
        }
        const int i = r < c ? r : c, j = r < c ? c : r;
        od[k] = keep ? i * ZW - (i * (i - 1)) / 2 + (j - i) : -1;
    }
    __syncthreads();   // every wave is done with its sorted tile
#pragma unroll
    for (int b0 = 0; b0 < NB; b0 += NBATCH) {
        if (b0 >= nbr) break;   // block-uniform
#pragma unroll
        for (int bb = 0; bb < NBATCH; ++bb) {
            const int b = b0 + bb;
            if (b >= NB) continue;
            double* img = tile + (w * NBATCH + bb) * PK;
#pragma unroll
            for (int k = 0; k < NI; ++k)
                if (od[k] >= 0) img[od[k]] = acc[b][k];
        }
        __syncthreads();
        for (int e = tid; e < NBATCH * PK; e += GT) {
            const int bb = e / PK, f = e - bb * PK;
            const int b = b0 + bb;
            if (b < nbr) {
                double s = tile[bb * PK + f];
#pragma unroll
                for (int ww = 1; ww < GNW; ++ww) s += tile[(ww * NBATCH + bb) * PK + f];
                outp[(int64_t)b * PK + f] = s;
            }
        }
        __syncthreads();
    }
}

template <int NT, int NB, int MINW>
void launch_gram(const fm_gram_args& a, hipStream_t st) {
    hipLaunchKernelGGL((gram_kernel<NT, NB, MINW>), dim3(a.nchunks), dim3(GT), 0, st, a);
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
        if (nb <= 1) launch_gram<1, 1, 3>(a, st);
        else if (nb <= 4) launch_gram<1, 4, 3>(a, st);
        else if (nb <= 8) launch_gram<1, 8, 3>(a, st);
        else if (nb <= 12) launch_gram<1, 12, 3>(a, st);
        else if (nb <= 15) launch_gram<1, 15, 3>(a, st);   // 5 patterns x 3 universes (Table 2)
        else if (nb <= 16) launch_gram<1, 16, 3>(a, st);
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

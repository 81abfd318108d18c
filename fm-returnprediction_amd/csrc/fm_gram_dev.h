// Device-side Gram accumulation of fm_gram (one workgroup per month chunk).
//
// Per wave, 64-row tiles (one row per lane):
//   1. ncols coalesced FP64 loads per row (SoA; the next tile's loads are in flight while
//      this one is processed), clip to the month's winsorize cuts, shift by the month's
//      pivot (optional standardize scale), z = [1, x..., y];
//   2. the row's validity pattern (bit m: every column model m needs is non-NaN) and its
//      universe level give a bucket id; per bucket one wave ballot gives the bucket's row
//      count (SGPR) and the lane's rank, so the counting sort needs no LDS counters; each
//      lane writes its z row to the wave's private LDS tile at (bucket offset + rank);
//   3. per bucket, v_mfma_f64_4x4x4_4b (__builtin_amdgcn_mfma_f64_4x4x4f64, four 4x4
//      blocks per instruction) with A = B = 4 rows of that bucket accumulates Z^T Z in
//      registers: three instructions per 4-row group cover the 16x16 Gram (block pairs, see
//      BlockPairs; rows past the bucket's count read the zero rows).
// At the end the waves' accumulators are summed through LDS and written as one packed
// upper-triangular Gram per bucket.
#pragma once
#include <math.h>

#include "fm_common.h"

// A/B and ablation knobs: timing builds only (tools/kbench.py), never the shipped library
#ifndef FM_AB_GRAM_NOMFMA
#define FM_AB_GRAM_NOMFMA 0
#endif
#ifndef FM_AB_GRAM_NOLOAD
#define FM_AB_GRAM_NOLOAD 0
#endif
#ifndef FM_AB_GRAM_NOSCATTER
#define FM_AB_GRAM_NOSCATTER 0
#endif
#ifndef FM_AB_GRAM_DPPOLD
#define FM_AB_GRAM_DPPOLD 0   // 1: the rotations through update_dpp(0, ...) (zero-initialised)
#endif
#ifndef FM_GRAM_PF2
#define FM_GRAM_PF2 0   // 1: two tiles of row loads in flight per wave (two register buffers)
#endif
#ifndef FM_GRAM_TOUCH
#define FM_GRAM_TOUCH 0   // 1: one 4-byte load per 128-byte line of the tile after next (L2 warm-up;
                          // measured 123.4 vs 110.3 us without: not used)
#endif

namespace fm {
namespace {

// nn = 2 * nn + (x is not NaN): one compare + one add-with-carry
__device__ __forceinline__ uint32_t push_valid(uint32_t nn, double x) {
    asm("v_cmp_o_f64 vcc, %1, %1\n\tv_addc_co_u32 %0, vcc, %0, %0, vcc" : "+v"(nn) : "v"(x) : "vcc");
    return nn;
}

// Lane value rotated within each 16-lane row: DPP row_ror:N gives lane i the value of lane
// (i - N) & 15 of its row (fm_common.h xor_lanes<4> relies on the same rule).
// Every lane of a rotation has a source lane, so the DPP "old" value is never used: mov_dpp
// (no old operand) spares the two zero-initialising moves update_dpp(0, ...) costs per half.
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double x) {
    const uint64_t u = (uint64_t)__double_as_longlong(x);
#if FM_AB_GRAM_DPPOLD
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)u, CTRL, 0xF, 0xF, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(u >> 32), CTRL, 0xF, 0xF, false);
#else
    const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)u, CTRL, 0xF, 0xF, true);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(u >> 32), CTRL, 0xF, 0xF, true);
#endif
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// 4x4 block pairs (I, J) of the ZW x ZW Gram covered by the 4x4x4 MFMAs of one 4-row group.
// v_mfma_f64_4x4x4_4b: lane l = x + 4*blk + 16*k holds A[blk][x][k] and B[blk][k][x], and
// D[blk][i][j] lands at lane j + 4*blk + 16*i.
//  * NT == 1 (16 columns): "rotation" cover.  Instruction k pairs block row blk with block
//    column (blk + k) % 4, k = 0..2: the diagonal blocks, the 4 blocks one step off (one of
//    them transposed) and the 2 blocks two steps off (computed twice).  Every lane's A
//    operand is z[row][q] (q = lane & 15) for all three instructions and its B operands are
//    z[row][q + 4k], so one address VGPR serves all three reads (immediate offsets).
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

template <int NT>
struct GramShape {
    static constexpr int ZW = 16 * NT;
    static constexpr int RS = ZW + 1;              // LDS row stride (doubles)
    static constexpr int TR = WAVE;                // rows per wave tile (one per lane)
    static constexpr int TPAD = 4;                 // pad rows after each wave's tile (see run)
    static constexpr int WT = (TR + TPAD) * RS;    // one wave's sorted tile + its pad rows
    static constexpr int PK = ZW * (ZW + 1) / 2;   // packed upper triangle
    static constexpr int NI = NT == 1 ? 3 : BlockPairs<8>::NI;   // 4x4x4 MFMAs per 4-row group
};

// One wave's share of the Gram of rows [r0, r1) (tiles w, w + NWV, ...).  Usage:
//   GramWave g(a, r0, r1, w);  g.prefetch();   (first tile's loads in flight)
//   ... fill the month parameters (prm) / pattern table (lut) / zero rows, barrier ...
//   g.run(prm, lut, scaled, tile, zblk);  barrier-free per wave
//   g.epilogue(tile, outp);   (all waves: cross-wave sum + packed store, barriers inside)
template <int NT, int NB, int NWV, bool PL = false, bool FULLC = false>
struct GramWave {
    using S = GramShape<NT>;
    static constexpr int ZW = S::ZW, RS = S::RS, TR = S::TR, WT = S::WT, PK = S::PK, NI = S::NI;

    const fm_gram_args& a;
    int64_t r0, r1;
    int w, lane, ntile;
    // register buffers of row loads: the next tile's loads are issued as soon as this tile's
    // values sit in LDS, and fly during its MFMAs (FM_GRAM_PF2: two tiles ahead)
    double xv[ZW - 1];
    int lv = 0;
    double xw[FM_GRAM_PF2 ? ZW - 1 : 1];
    int lw = 0;
    double acc[NB][NI];
    // touch loads: the previous touch's word (consumed a tile later, when it has landed) and
    // their xor (kept live so the loads stay; never meaningful)
    uint32_t tpend = 0, tacc = 0;

    __device__ __forceinline__ GramWave(const fm_gram_args& a_, int64_t r0_, int64_t r1_, int w_)
        : a(a_), r0(r0_), r1(r1_), w(w_), lane((int)threadIdx.x & (WAVE - 1)),
          ntile((int)((r1_ - r0_ + TR - 1) / TR)) {}

    // Row loads: one wave-uniform base per column (s_add in the scalar unit) + the lane's
    // 32-bit row offset, so every load is a global_load with an SGPR base and no per-load
    // address VALU.  Lanes past the chunk end re-read its last row (masked later).  Without
    // universes the level load reads byte 0 of the panel and is masked to 0.
    __device__ __forceinline__ void load_row(int t) { load_row_into(t, xv, lv); }

    template <int N>
    __device__ __forceinline__ void load_row_into(int t, double (&xv)[N], int& lv) {
        typedef const __attribute__((address_space(1))) char* gptr;   // global_load, not flat_load
        const int64_t t0 = r0 + (int64_t)t * TR;
        const int64_t last = r1 - 1 - t0;
        const uint32_t lo = last < 0 ? 0u : (last < lane ? (uint32_t)last : (uint32_t)lane);
        const int64_t tb = last < 0 ? r1 - 1 : t0;   // wave-uniform tile base (clamped)
        const double* cb = a.cols + tb;               // column 0; s_add per column
        if (FM_AB_GRAM_NOLOAD) {
#pragma unroll
            for (int c = 0; c < ZW - 1; ++c) xv[c] = (double)(lo + t) * 0.001 + c;
            lv = (int)(lo & 3);
            return;
        }
        if constexpr (PL) {
            // the split panel: high and low words from their planes (4-byte loads, the same
            // SGPR-base + lane-offset addressing), joined in registers
            const uint32_t* hb = a.hi_plane + tb;
            const uint32_t* lb = a.lo_plane + tb;
#pragma unroll
            for (int c = 0; c < ZW - 1; ++c) {
                const uint32_t h = *(const __attribute__((address_space(1))) uint32_t*)((gptr)hb + lo * 4u);
                const uint32_t l = *(const __attribute__((address_space(1))) uint32_t*)((gptr)lb + lo * 4u);
                xv[c] = __longlong_as_double((long long)(((uint64_t)h << 32) | l));
                // FULLC (ncols == ZW - 1, the Table-2 panel): every column step is the stride --
                // no per-column compare and selects in the scalar stream
                const int64_t step = FULLC || c + 1 < a.ncols ? a.plane_stride : 0;
                hb += step;
                lb += step;
                asm("" : "+s"(hb), "+s"(lb));
            }
        } else {
#pragma unroll
            for (int c = 0; c < ZW - 1; ++c) {
                xv[c] = *(const __attribute__((address_space(1))) double*)((gptr)cb + lo * 8u);
                cb += FULLC || c + 1 < a.ncols ? a.col_stride : 0;   // columns past ncols re-read the last
                // opaque to the optimizer: otherwise it turns a repeated address into a register
                // copy of the previous load behind a branch, i.e. a vmcnt(0) wait per column
                asm("" : "+s"(cb));
            }
        }
        const uint8_t* lvbase = a.level ? a.level : (const uint8_t*)a.seg_off;   // any valid address
        // raw byte; masked where it is used (masking here would wait for the load)
        lv = *((gptr)(a.level ? lvbase + tb : lvbase) + (a.level ? lo : 0u));
    }

    // Warm the L2 for tile t: lane l loads one 4-byte word of 128-byte line (l & 3) of column
    // l >> 2 (FP64 columns: 16 rows a line; planes: 32 rows, lanes 0-1 the high plane, 2-3 the
    // low one), so ONE load instruction covers the tile's 60 lines; its data is consumed a tile
    // later.  The wave's own loads of tile t, issued a tile after, then hit the L2 instead of
    // waiting a loaded-HBM round trip with one tile in flight.
    __device__ __forceinline__ void touch(int t) {
        if constexpr (FM_GRAM_TOUCH == 0) return;
        tacc ^= tpend;
        if (t >= ntile) return;   // wave-uniform
        typedef const __attribute__((address_space(1))) uint32_t* gptr32;
        const int64_t t0 = r0 + (int64_t)t * TR;
        const int c = lane >> 2, q = lane & 3;
        const int cc = c < a.ncols ? c : a.ncols - 1;
        int64_t row = t0 + (PL ? (q & 1) * 32 : q * 16);
        row = row < r1 - 1 ? row : r1 - 1;
        const uint32_t* p;
        if constexpr (PL) p = (q < 2 ? a.hi_plane : a.lo_plane) + (int64_t)cc * a.plane_stride + row;
        else p = (const uint32_t*)(a.cols + (int64_t)cc * a.col_stride + row);
        tpend = *(gptr32)p;
    }
    __device__ __forceinline__ void touch_sink() {
        if constexpr (FM_GRAM_TOUCH == 0) return;
        tacc ^= tpend;
        if (tacc == 0x9E3779B9u && a.nseg == -7) a.flags[lane] = tacc;   // never true: keeps the loads
    }

    __device__ __forceinline__ void prefetch() {
        touch(w + NWV);
        if (w < ntile) load_row(w);
        if constexpr (FM_GRAM_PF2 != 0)
            if (w + NWV < ntile) load_row_into(w + NWV, xw, lw);
    }

    // prm: LDS [4][32] = lo, hi, shift, inv_scale per column; lut: LDS pattern table.
    __device__ __forceinline__ void run(const double (*prm)[32], const uint8_t* lut, bool scaled,
                                        double* tile, const double* zblk) {
        constexpr BlockPairs<4 * NT> BP{};
        const int nmodels = a.nmodels, nlevels = a.nlevels;
        const int lvand = a.level ? 0xFF : 0;
        const uint32_t colmask = a.ncols >= 32 ? ~0u : (1u << a.ncols) - 1u;
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
        // model column masks in SGPRs (wave-uniform; statically indexed below)
        const int mmv = (int)a.model_mask[lane < nmodels ? lane : 0];
        uint32_t mm[FM_MAX_MODELS];
#pragma unroll
        for (int m = 0; m < FM_MAX_MODELS; ++m)
            mm[m] = (uint32_t)__builtin_amdgcn_readlane(mmv, m < nmodels ? m : 0);

        auto tile_step = [&](auto& xv, int& lv, int t, int tnext) {
            const int64_t row = r0 + (int64_t)t * TR + lane;
            // validity bits of the raw values (NaN = missing; clipping never makes or
            // removes a NaN: pandas clip ignores NaN bounds)
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
            // Gram entries it pollutes are never read by fm_solve.  clip = hardware max/min:
            // a NaN bound is ignored, a NaN x gives a don't-care value.  Dropped rows are not
            // stored.
            if (valid && !FM_AB_GRAM_NOSCATTER) {
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
            // this tile's values are consumed: the next tile's loads fly during the MFMAs, and
            // the one after next is touched into the L2
            if (tnext < ntile) load_row_into(tnext, xv, lv);
            touch(tnext + NWV);
            // the operand reads below read other lanes' rows of this wave: LDS executes one
            // wave's DS instructions in order, so only compiler reordering must be prevented
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            // ---- MFMA accumulation per bucket: NI independent 4x4x4 block products per
            // 4-row group; rows past the bucket's count contribute zeros.  Per-bucket counts
            // are popcounts of the ballot masks, formed on the fly (scalar).
            if (FM_AB_GRAM_NOMFMA) {
                if (__popcll(bv) == 65) acc[0][0] += wt[oa[0]];   // keeps bv/dest alive
                return;
            }
            if constexpr (NT == 1) {
                // ONE LDS read per group: lane (kr, q) reads z[row kr][q] = the A operand; the
                // B operands z[kr][(q + 4k) & 15] are the same register of lane (kr, q + 4k),
                // i.e. a DPP rotation within the lane's 16-lane row (row_ror 12 / 8).  The
                // next group's read is issued before this group's MFMAs (the sorted tile is
                // contiguous: the next group starts 4 rows on, or at the next bucket's start
                // = this bucket's end, whatever buckets in between are empty).
                const int abase = (lane >> 4) * RS + (lane & 15);
                const double* rd = wt + abase;
                double An = rd[0];
                int off = 0;
#pragma unroll
                for (int b = 0; b < NB; ++b) {
                    uint64_t mb = bv;
#pragma unroll
                    for (int i = 0; i < KB; ++i) mb &= ((b >> i) & 1) ? bit[i] : ~bit[i];
                    const int n = (int)__popcll(mb);
                    // one 4-row group: operand `cur` (read one group ahead), the next group's
                    // read into `nxt`.  Rows past the tile end (rn + kr <= TR + 3: lanes of rows
                    // past a bucket's count) read this wave's own TPAD pad rows, never another
                    // wave's tile; their (unwritten) values are masked here
                    auto group = [&](int g, const double cur, double& nxt) {
                        const int rn = g + 4 < n ? off + g + 4 : off + n;
                        nxt = rd[rn * RS];
                        const double A = kr < n - g ? cur : 0.0;
                        const double B1 = dpp_f64<0x12C>(A), B2 = dpp_f64<0x128>(A);
                        acc[b][0] = __builtin_amdgcn_mfma_f64_4x4x4f64(A, A, acc[b][0], 0, 0, 0);
                        acc[b][1] = __builtin_amdgcn_mfma_f64_4x4x4f64(A, B1, acc[b][1], 0, 0, 0);
                        acc[b][2] = __builtin_amdgcn_mfma_f64_4x4x4f64(A, B2, acc[b][2], 0, 0, 0);
                    };
                    for (int g = 0; g < n; g += 4) {
                        const double Ar = An;
                        group(g, Ar, An);
                    }
                    off += n;
                }
            } else {
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
            }
            // the next tile's scatter overwrites this tile: every operand read above has been
            // consumed by its MFMA (data dependence), and the fences keep the order
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        };
        if constexpr (FM_GRAM_PF2 != 0) {
            for (int t = w; t < ntile; t += 2 * NWV) {
                tile_step(xv, lv, t, t + 2 * NWV);
                if (t + NWV < ntile) tile_step(xw, lw, t + NWV, t + 3 * NWV);
            }
        } else {
            for (int t = w; t < ntile; t += NWV) tile_step(xv, lv, t, t + NWV);
        }
        touch_sink();
    }

    // Cross-wave reduction and store: outp[bucket][packed upper triangle] for the nbr
    // buckets in use.  v_mfma_f64_4x4x4f64 leaves D[blk][i][j] in lane j + 4*blk + 16*i; each
    // lane maps its entry of instruction k to the packed index of (min(r, c), max(r, c)), or
    // -1 where the entry is a duplicate (NT 1: the two-step blocks computed twice; diagonal
    // blocks: the strictly lower half), so every packed entry is written once per wave.
    // `tile` (NWV * WT doubles) is reused as the reduction image; block-wide barriers.
    __device__ __forceinline__ void epilogue(double* tile, double* outp, int nbr) {
        constexpr BlockPairs<4 * NT> BP{};
        constexpr int NBATCH = (NWV * WT) / (NWV * PK) < NB ? (NWV * WT) / (NWV * PK) : NB;
        static_assert(NBATCH >= 1, "epilogue image does not fit the tile area");
        const int kx = lane & 3, kb = (lane >> 2) & 3, kr = lane >> 4;
        const int tid = (int)threadIdx.x;
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
            for (int e = tid; e < NBATCH * PK; e += NWV * WAVE) {
                const int bb = e / PK, f = e - bb * PK;
                const int b = b0 + bb;
                if (b < nbr) {
                    double s = tile[bb * PK + f];
#pragma unroll
                    for (int ww = 1; ww < NWV; ++ww) s += tile[(ww * NBATCH + bb) * PK + f];
                    outp[(int64_t)b * PK + f] = s;
                }
            }
            __syncthreads();
        }
    }
};

}  // namespace
}  // namespace fm

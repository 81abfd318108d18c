// Shared device/host helpers for libfm_hip (gfx950 / CDNA4, wave64).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "fm_hip.h"

namespace fm {

void set_error(const char* fmt, ...);
int check_launch(const char* what);

#define FM_REQUIRE(cond, ...)            \
    do {                                 \
        if (!(cond)) {                   \
            ::fm::set_error(__VA_ARGS__); \
            return FM_EINVAL;            \
        }                                \
    } while (0)

#define FM_CHECK_LAUNCH(name)                       \
    do {                                            \
        int rc_ = ::fm::check_launch(name);         \
        if (rc_ != FM_OK) return rc_;               \
    } while (0)

constexpr uint64_t SENT = ~0ull;   // key of NaN / absent values: sorts after +inf
constexpr int WAVE = 64;

// Panel values as FP64 columns or as the split panel's two 32-bit planes (high words, low
// words; fm_gen_panel_planes / fm_split_planes): element i (= c * stride + r) either way.
// The hot kernels read the planes with their own loads; this view serves the paths that
// read individual values (pick gathers, fix-ups, refits).
struct PCols {
    const double* f = nullptr;
    const uint32_t* h = nullptr;
    int64_t loff = 0;   // the low plane at this element offset from the high one
    __device__ __forceinline__ double operator[](int64_t i) const {
        if (f != nullptr) return f[i];
        return __longlong_as_double((long long)(((uint64_t)h[i] << 32) | h[i + loff]));
    }
    __device__ __forceinline__ PCols off(int64_t o) const {
        return f != nullptr ? PCols{f + o, nullptr, 0} : PCols{nullptr, h + o, loff};
    }
};
// The same two views as separate types, for code that is instantiated per layout (a branch
// per access inside a register-heavy unrolled loop costs registers: the solve's fix-ups)
struct F64Cols {
    const double* f;
    __device__ __forceinline__ double operator[](int64_t i) const { return f[i]; }
};
struct PlaneCols {   // the low plane at a fixed element offset from the high one (one base pointer)
    const uint32_t* h;
    int64_t loff;
    __device__ __forceinline__ double operator[](int64_t i) const {
        return __longlong_as_double((long long)(((uint64_t)h[i] << 32) | h[i + loff]));
    }
};

// Phase probe (timing builds only, tools/build_variant.sh probe "-DFM_PROBE=1" ...;
// tools/tail_probe.py): thread 0 of a workgroup writes s_memrealtime (100 MHz) at numbered
// points of a kernel into that translation unit's own bounded buffer (FM_PROBE_BUFFER), read
// back by fm_probe_copy_<tu>.  Compiled out of the shipped library.
#ifndef FM_PROBE
#define FM_PROBE 0
#endif
constexpr int PROBE_WG = 8192, PROBE_SLOTS = 8;
#if FM_PROBE
#define FM_PROBE_BUFFER(tu)                                                                  \
    namespace fm {                                                                           \
    __device__ uint32_t g_probe_##tu[PROBE_SLOTS * PROBE_WG];                                \
    }                                                                                        \
    extern "C" int fm_probe_copy_##tu(uint32_t* host, int32_t nwg) {                         \
        const int n = nwg < ::fm::PROBE_WG ? nwg : ::fm::PROBE_WG;                           \
        return hipMemcpyFromSymbol(host, HIP_SYMBOL(::fm::g_probe_##tu),                     \
                                   (size_t)n * ::fm::PROBE_SLOTS * 4) == hipSuccess ? 0 : -1; \
    }                                                                                        \
    extern "C" int fm_probe_clear_##tu() {                                                   \
        void* p_ = nullptr;                                                                  \
        if (hipGetSymbolAddress(&p_, HIP_SYMBOL(::fm::g_probe_##tu)) != hipSuccess) return -1; \
        return hipMemset(p_, 0, sizeof(::fm::g_probe_##tu)) == hipSuccess ? 0 : -1;          \
    }
#define FM_PROBE_AT(tu, slot)                                                                \
    do {                                                                                     \
        if (threadIdx.x == 0) {                                                              \
            const int64_t w_ = blockIdx.x + (int64_t)gridDim.x * (blockIdx.y + (int64_t)gridDim.y * blockIdx.z); \
            if (w_ < ::fm::PROBE_WG)                                                         \
                ::fm::g_probe_##tu[w_ * ::fm::PROBE_SLOTS + (slot)] =                        \
                    (uint32_t)__builtin_amdgcn_s_memrealtime();                              \
        }                                                                                    \
    } while (0)
#else
#define FM_PROBE_BUFFER(tu)
#define FM_PROBE_AT(tu, slot) \
    do {                      \
    } while (0)
#endif

// Order-preserving map double -> uint64 (total order with -0.0 < +0.0; callers map NaN
// to SENT before calling).
__device__ __forceinline__ uint64_t dkey(double v) {
    uint64_t b = (uint64_t)__double_as_longlong(v);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__device__ __forceinline__ double kval(uint64_t k) {
    uint64_t b = (k >> 63) ? (k & 0x7FFFFFFFFFFFFFFFull) : ~k;
    return __longlong_as_double((long long)b);
}

__device__ __forceinline__ int lane_id() { return (int)__lane_id(); }

// 64-bit readlane (the builtin takes 32-bit operands: a 64-bit argument is truncated)
__device__ __forceinline__ uint64_t readlane_u64(uint64_t v, int l) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}

// compile-time loop: f(std::integral_constant<int, i>) for i in [B, E)
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        static_for<B + 1, E>(f);
    }
}

// Value of lane (this lane ^ J), without LDS: DPP quad_perm (1, 2), two bank-masked DPP
// row rotations (4), DPP row_ror:8 (8), v_permlane16_swap / v_permlane32_swap (16, 32).
// Verified against __shfl_xor by tools/probes/xor_probe.hip.  Where every lane has a source
// lane (J = 1, 2, 8) mov_dpp is used: it has no "old" operand, so no copy of x is made first.
template <int J>
__device__ __forceinline__ uint32_t xor_lanes(uint32_t x) {
    if constexpr (J == 1) {
        return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, true);
    } else if constexpr (J == 2) {
        return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, true);
    } else if constexpr (J == 4) {
        const int t = __builtin_amdgcn_update_dpp((int)x, (int)x, 0x12C, 0xF, 0x5, false);   // lanes 0-3, 8-11
        return (uint32_t)__builtin_amdgcn_update_dpp(t, (int)x, 0x124, 0xF, 0xA, false);    // lanes 4-7, 12-15
    } else if constexpr (J == 8) {
        return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x128, 0xF, 0xF, true);
    } else if constexpr (J == 16) {
        const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
        return (__lane_id() & 16) ? r[0] : r[1];
    } else {
        static_assert(J == 32, "xor_lanes: J in {1,2,4,8,16,32}");
        const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
        return (__lane_id() & 32) ? r[0] : r[1];
    }
}
// run-time J that is a constant after unrolling (the switch folds away)
__device__ __forceinline__ uint32_t xor_lanes_u32(uint32_t x, int j) {
    switch (j) {
        case 1: return xor_lanes<1>(x);
        case 2: return xor_lanes<2>(x);
        case 4: return xor_lanes<4>(x);
        case 8: return xor_lanes<8>(x);
        case 16: return xor_lanes<16>(x);
        default: return xor_lanes<32>(x);
    }
}
__device__ __forceinline__ uint64_t xor_lanes_u64(uint64_t x, int j) {
    const uint32_t lo = xor_lanes_u32((uint32_t)x, j), hi = xor_lanes_u32((uint32_t)(x >> 32), j);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ double xor_lanes_f64(double x, int j) {
    return __longlong_as_double((long long)xor_lanes_u64((uint64_t)__double_as_longlong(x), j));
}
// Any 4- or 8-byte value of lane (this lane ^ J): xor_lanes per 32-bit half (bit-exact
// __shfl_xor, which is a ds_bpermute -- an LDS round trip per step)
template <int J, typename T>
__device__ __forceinline__ T xor_lane(T v) {
    static_assert(sizeof(T) == 4 || sizeof(T) == 8, "xor_lane: 4- or 8-byte values");
    if constexpr (sizeof(T) == 4) {
        return __builtin_bit_cast(T, xor_lanes<J>(__builtin_bit_cast(uint32_t, v)));
    } else {
        const uint64_t b = __builtin_bit_cast(uint64_t, v);
        const uint32_t lo = xor_lanes<J>((uint32_t)b), hi = xor_lanes<J>((uint32_t)(b >> 32));
        return __builtin_bit_cast(T, ((uint64_t)hi << 32) | lo);
    }
}
// Butterfly over the wave (distances 32, 16, .., 1: the order the __shfl_xor loops used, so
// floating-point sums keep their bits) or over each 16-lane row (8, 4, 2, 1).
template <typename T, typename Op>
__device__ __forceinline__ T wave_reduce(T v, Op op) {
    v = op(v, xor_lane<32>(v));
    v = op(v, xor_lane<16>(v));
    v = op(v, xor_lane<8>(v));
    v = op(v, xor_lane<4>(v));
    v = op(v, xor_lane<2>(v));
    v = op(v, xor_lane<1>(v));
    return v;
}
template <typename T, typename Op>
__device__ __forceinline__ T row16_reduce(T v, Op op) {
    v = op(v, xor_lane<8>(v));
    v = op(v, xor_lane<4>(v));
    v = op(v, xor_lane<2>(v));
    v = op(v, xor_lane<1>(v));
    return v;
}
template <typename T>
__device__ __forceinline__ T row16_sum(T v) {
    return row16_reduce(v, [](T a, T b) { return a + b; });
}
// Value of lane (this lane - O) within this lane's 16-lane row (DPP row_shr; lanes below O
// in their row get `v` back, like __shfl_up with width 16)
template <int O, typename T>
__device__ __forceinline__ T row_shr(T v) {
    static_assert(O >= 1 && O <= 15, "row_shr: 1..15");
    static_assert(sizeof(T) == 4 || sizeof(T) == 8, "row_shr: 4- or 8-byte values");
    if constexpr (sizeof(T) == 4) {
        const int x = __builtin_bit_cast(int, v);
        return __builtin_bit_cast(T, __builtin_amdgcn_update_dpp(x, x, 0x110 + O, 0xF, 0xF, false));
    } else {
        const uint64_t b = __builtin_bit_cast(uint64_t, v);
        const int lo = (int)(uint32_t)b, hi = (int)(uint32_t)(b >> 32);
        const uint32_t rl = (uint32_t)__builtin_amdgcn_update_dpp(lo, lo, 0x110 + O, 0xF, 0xF, false);
        const uint32_t rh = (uint32_t)__builtin_amdgcn_update_dpp(hi, hi, 0x110 + O, 0xF, 0xF, false);
        return __builtin_bit_cast(T, ((uint64_t)rh << 32) | rl);
    }
}
// Inclusive prefix sum of an int over the wave: four DPP row shifts, then row 15 / row 31
// broadcasts into the later rows (integer adds: the same result as the __shfl_up ladder)
__device__ __forceinline__ int wave_incl_scan(int x) {
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xF, 0xF, false);   // row_shr:1
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xF, 0xF, false);   // row_shr:2
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xF, 0xF, false);   // row_shr:4
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xF, 0xF, false);   // row_shr:8
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xA, 0xF, false);   // row_bcast:15 -> rows 1, 3
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xC, 0xF, false);   // row_bcast:31 -> rows 2, 3
    return x;
}

// Hardware v_max_f64 / v_min_f64 (IEEE mode: a quiet-NaN operand yields the other one).
// Inline asm, because the maxnum/minnum lowering canonicalizes its inputs first: an extra
// v_max_f64 per operand, and a second register copy of every value kept for later use.
__device__ __forceinline__ double hw_max(double a, double b) {
    double r;
    asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ double hw_min(double a, double b) {
    double r;
    asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

// Error-free sum a + b = s + e (Knuth TwoSum; the library builds with -ffp-contract=off, so
// no operation below is fused or reassociated).
__device__ __forceinline__ double two_sum(double a, double b, double* e) {
    const double s = a + b;
    const double bp = s - a;
    *e = (a - (s - bp)) + (b - bp);
    return s;
}

// Compensated running sum (s + c): adding and later removing a term far larger than the
// others leaves O(eps^2) of it behind instead of ulp(term) -- the sliding window sums of the
// rolling means (pandas roll_mean keeps a Kahan compensation for the same reason).
struct CSum {
    double s = 0.0, c = 0.0;
    __device__ __forceinline__ void add(double x) {
        double e;
        s = two_sum(s, x, &e);
        c += e;
    }
    __device__ __forceinline__ double value() const { return s + c; }
    __device__ __forceinline__ void reset() { s = c = 0.0; }
};

// LDS writes of this wave visible to its other lanes (a wave-local barrier)
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
}

// number of set bits of `mask` strictly below this lane
__device__ __forceinline__ int mask_rank(uint64_t mask) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                     __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
    return wave_reduce(v, [](T a, T b) { return a + b; });
}
__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
    return wave_reduce(v, [](uint64_t a, uint64_t b) { return b < a ? b : a; });
}
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
    return wave_reduce(v, [](uint64_t a, uint64_t b) { return b > a ? b : a; });
}
__device__ __forceinline__ uint32_t wave_or_u32(uint32_t v) {
    return wave_reduce(v, [](uint32_t a, uint32_t b) { return a | b; });
}

// Block-wide reductions for blocks of NW waves; `scratch` holds NW elements.  Every
// thread of the block must call; result is returned to all threads.
template <int NW, typename T>
__device__ __forceinline__ T block_sum(T v, T* scratch) {
    v = wave_sum(v);
    const int w = threadIdx.x / WAVE;
    __syncthreads();
    if (lane_id() == 0) scratch[w] = v;
    __syncthreads();
    T s = scratch[0];
#pragma unroll
    for (int i = 1; i < NW; ++i) s += scratch[i];
    return s;
}
template <int NW>
__device__ __forceinline__ uint64_t block_min_u64(uint64_t v, uint64_t* scratch) {
    v = wave_min_u64(v);
    const int w = threadIdx.x / WAVE;
    __syncthreads();
    if (lane_id() == 0) scratch[w] = v;
    __syncthreads();
    uint64_t s = scratch[0];
#pragma unroll
    for (int i = 1; i < NW; ++i) s = scratch[i] < s ? scratch[i] : s;
    return s;
}
template <int NW>
__device__ __forceinline__ uint64_t block_max_u64(uint64_t v, uint64_t* scratch) {
    v = wave_max_u64(v);
    const int w = threadIdx.x / WAVE;
    __syncthreads();
    if (lane_id() == 0) scratch[w] = v;
    __syncthreads();
    uint64_t s = scratch[0];
#pragma unroll
    for (int i = 1; i < NW; ++i) s = scratch[i] > s ? scratch[i] : s;
    return s;
}

template <int NW>
__device__ __forceinline__ double block_min_f64(double v, double* scratch) {
    v = wave_reduce(v, [](double a, double b) { return fmin(a, b); });
    const int w = threadIdx.x / WAVE;
    __syncthreads();
    if (lane_id() == 0) scratch[w] = v;
    __syncthreads();
    double s = scratch[0];
#pragma unroll
    for (int i = 1; i < NW; ++i) s = fmin(s, scratch[i]);
    return s;
}
// Two sums at once (one pair of barriers); `scratch` holds 2*NW doubles.
template <int NW>
__device__ __forceinline__ double2 block_sum2(double a, double b, double* scratch) {
    a = wave_sum(a);
    b = wave_sum(b);
    const int w = threadIdx.x / WAVE;
    __syncthreads();
    if (lane_id() == 0) {
        scratch[w] = a;
        scratch[NW + w] = b;
    }
    __syncthreads();
    double2 r = make_double2(scratch[0], scratch[NW]);
#pragma unroll
    for (int i = 1; i < NW; ++i) {
        r.x += scratch[i];
        r.y += scratch[NW + i];
    }
    return r;
}

// Exclusive prefix sum over the block (NW waves); returns this thread's offset and the
// block total via *total.
template <int NW>
__device__ __forceinline__ int block_excl_scan(int v, int* scratch, int* total) {
    const int lane = lane_id();
    const int w = threadIdx.x / WAVE;
    const int x = wave_incl_scan(v);
    __syncthreads();
    if (lane == WAVE - 1) scratch[w] = x;
    __syncthreads();
    int base = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < NW; ++i) {
        int s = scratch[i];
        if (i < w) base += s;
        tot += s;
    }
    *total = tot;
    return base + x - v;
}

}  // namespace fm

// fm_ffill_expand: the annual -> monthly Compustat expansion of
// expand_compustat_annual_to_monthly (reference src/transform_compustat.py:101-172).
//
// The reference reindexes every gvkey group onto all month-ends from its first report month
// to min(latest report month of the whole table, its own last report month + 12) and
// forward-fills (pandas reindex(method="ffill")): output month m of group g takes the whole
// record of the group's LAST report month <= m.  Here months are integer month codes, the
// records are sorted by (group, month) with CSR group offsets, and the output layout
// (out_off, a prefix over the groups' month counts) is planned on the host.  One thread per
// output row: binary search of its group (over out_off), then of its source record (over
// the group's months), then a coalesced-by-row gather of the FP64 columns; the source record
// index is returned too, so the caller gathers columns of any other dtype the same way.
#include "fm_common.h"

namespace fm {
namespace {

constexpr int XT = 256;

__global__ __launch_bounds__(XT) void ffill_expand_kernel(const int64_t* __restrict__ rec_off,
                                                          const int32_t* __restrict__ rec_month,
                                                          const int64_t* __restrict__ out_off,
                                                          int32_t ngroups, int64_t nout,
                                                          const double* __restrict__ vals,
                                                          int64_t v_stride, int32_t ncols,
                                                          double* __restrict__ out_vals,
                                                          int64_t o_stride,
                                                          int32_t* __restrict__ out_month,
                                                          int64_t* __restrict__ out_src) {
    for (int64_t i = (int64_t)blockIdx.x * XT + threadIdx.x; i < nout; i += (int64_t)gridDim.x * XT) {
        // group g: the last g with out_off[g] <= i
        int lo = 0, hi = ngroups - 1;
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (out_off[mid] <= i) lo = mid;
            else hi = mid - 1;
        }
        const int g = lo;
        const int64_t r0 = rec_off[g], r1 = rec_off[g + 1];
        const int32_t m = rec_month[r0] + (int32_t)(i - out_off[g]);
        // source record: the last r in [r0, r1) with rec_month[r] <= m (r0 always qualifies)
        int64_t a = r0, b = r1 - 1;
        while (a < b) {
            const int64_t mid = (a + b + 1) >> 1;
            if (rec_month[mid] <= m) a = mid;
            else b = mid - 1;
        }
        out_month[i] = m;
        out_src[i] = a;
        for (int c = 0; c < ncols; ++c) out_vals[(int64_t)c * o_stride + i] = vals[(int64_t)c * v_stride + a];
    }
}

// Equality join on a two-part int64 key (merge_CRSP_and_Compustat's gvkey and (permno,
// jdate) merges, reference src/transform_compustat.py:218-225): right keys sorted
// lexicographically (stable, so equal keys keep the right frame's order), one thread per left
// row, lower / upper bound by binary search.  Matches of left row i are right rows
// [lo[i], hi[i]) of the sorted order, i.e. pandas' merge order (left rows in order, each
// with its matches in right order).
__device__ __forceinline__ bool key_lt(int64_t a1, int64_t a2, int64_t b1, int64_t b2) {
    return a1 < b1 || (a1 == b1 && a2 < b2);
}

__global__ __launch_bounds__(XT) void sorted_join_kernel(const int64_t* __restrict__ lk1,
                                                         const int64_t* __restrict__ lk2, int64_t nl,
                                                         const int64_t* __restrict__ rk1,
                                                         const int64_t* __restrict__ rk2, int64_t nr,
                                                         int64_t* __restrict__ lo, int64_t* __restrict__ hi) {
    for (int64_t i = (int64_t)blockIdx.x * XT + threadIdx.x; i < nl; i += (int64_t)gridDim.x * XT) {
        const int64_t k1 = lk1[i], k2 = lk2 ? lk2[i] : 0;
        int64_t a = 0, b = nr;   // first right key >= (k1, k2)
        while (a < b) {
            const int64_t mid = (a + b) >> 1;
            if (key_lt(rk1[mid], rk2 ? rk2[mid] : 0, k1, k2)) a = mid + 1;
            else b = mid;
        }
        int64_t c = a, d = nr;   // first right key > (k1, k2)
        while (c < d) {
            const int64_t mid = (c + d) >> 1;
            if (!key_lt(k1, k2, rk1[mid], rk2 ? rk2[mid] : 0)) c = mid + 1;
            else d = mid;
        }
        lo[i] = a;
        hi[i] = c;
    }
}

}  // namespace
}  // namespace fm

extern "C" int fm_sorted_join(const int64_t* lk1, const int64_t* lk2, int64_t nl, const int64_t* rk1,
                              const int64_t* rk2, int64_t nr, int64_t* lo, int64_t* hi, void* stream) {
    using namespace fm;
    FM_REQUIRE(lk1 && rk1 && lo && hi, "fm_sorted_join: null pointer");
    FM_REQUIRE((lk2 == nullptr) == (rk2 == nullptr), "fm_sorted_join: second key parts must both be set or NULL");
    FM_REQUIRE(nl >= 0 && nr >= 0, "fm_sorted_join: bad sizes");
    if (nl == 0) return FM_OK;
    const int64_t blocks = (nl + XT - 1) / XT;
    const int grid = (int)(blocks < 65535 * 16 ? blocks : 65535 * 16);
    hipLaunchKernelGGL(sorted_join_kernel, dim3(grid), dim3(XT), 0, (hipStream_t)stream, lk1, lk2, nl, rk1, rk2,
                       nr, lo, hi);
    FM_CHECK_LAUNCH("fm_sorted_join");
    return FM_OK;
}

extern "C" int fm_ffill_expand(const int64_t* rec_off, const int32_t* rec_month, const int64_t* out_off,
                               int32_t ngroups, int64_t nout, const double* vals, int64_t v_stride,
                               int32_t ncols, double* out_vals, int64_t o_stride, int32_t* out_month,
                               int64_t* out_src, void* stream) {
    using namespace fm;
    FM_REQUIRE(rec_off && rec_month && out_off && out_month && out_src, "fm_ffill_expand: null pointer");
    FM_REQUIRE(ncols == 0 || (vals && out_vals), "fm_ffill_expand: null value pointers");
    FM_REQUIRE(ngroups >= 0 && nout >= 0 && ncols >= 0, "fm_ffill_expand: bad sizes");
    if (nout == 0 || ngroups == 0) return FM_OK;
    const int64_t blocks = (nout + XT - 1) / XT;
    const int grid = (int)(blocks < 65535 * 16 ? blocks : 65535 * 16);
    hipLaunchKernelGGL(ffill_expand_kernel, dim3(grid), dim3(XT), 0, (hipStream_t)stream, rec_off, rec_month,
                       out_off, ngroups, nout, vals, v_stride, ncols, out_vals, o_stride, out_month, out_src);
    FM_CHECK_LAUNCH("fm_ffill_expand");
    return FM_OK;
}

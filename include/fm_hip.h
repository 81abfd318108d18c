/*
 * fm_hip.h — C ABI of libfm_hip.so, the MI355X (gfx950) Fama-MacBeth engine.
 *
 * Drop-in boundary.  The reference (BaileyMeche/FM-ReturnPrediction) has no FFI layer: its
 * hot path is a set of pandas-in/pandas-out Python functions.  The Python mirror in
 * fm-returnprediction_amd/fmdrop/{regressions,calc_Lewellen_2014,transform_compustat}.py
 * keeps those names and signatures and calls the entry points below through ctypes.  Each entry point names
 * the reference computation it replaces:
 *
 *   fm_select_cuts  <- np.percentile(vals, 1/99) per month per var
 *                      (src/calc_Lewellen_2014.py:519-523) and pandas
 *                      groupby("mthcaldt")["me"].quantile([.2,.5]) over NYSE rows (:74-82)
 *   fm_select       <- the same, struct-argument form: wave-per-(month, column) tail
 *                      selection with an exact workgroup fallback, plus the Gram pivot
 *                      `center` (the Table-2 fast path; fm_select_cuts calls it); months
 *                      of 6,145 .. 20,480 rows (C5) one register-resident 512-thread
 *                      workgroup per (month, column), longer ones streamed; optionally the
 *                      universe level bytes from the cuts (get_subsets :95-105)
 *   fm_clip         <- subdf[var].clip(lower, upper) (src/calc_Lewellen_2014.py:524)
 *   fm_standardize  <- per-month z-score (north-star extension; no reference line)
 *   fm_universe_level <- me >= me_20 / me >= me_50 masks (src/calc_Lewellen_2014.py:95-96)
 *   fm_universe     <- get_subsets in one launch: the NYSE groupby.quantile([.2,.5]) of me
 *                      (src/calc_Lewellen_2014.py:74-82) and the nested masks (:95-105)
 *   fm_pilot_shift  <- (numerics only) per-month pivot used to center the Gram
 *   fm_gram         <- dropna (src/regressions.py:39) + X'X, X'y, y'y inside sm.OLS
 *                      (src/regressions.py:57; src/calc_Lewellen_2014.py:917-919), batched
 *                      over models x universes in one read of the panel
 *   fm_solve        <- sm.OLS(Y, X).fit() params / rsquared / N and the N<K+1 skip
 *                      (src/regressions.py:52-72; src/calc_Lewellen_2014.py:914-921)
 *   fm_solve_fixup  <- statsmodels' pinv semantics where fm_solve's normal equations do not
 *                      reach them (src/regressions.py:57-64): pinv(X) @ y with an infinite
 *                      return (+-inf/NaN params, NaN R2), and ill-conditioned / rank-
 *                      deficient months re-solved from their rows (Householder QR + SVD)
 *   fm_const_check  <- add_constant(has_constant='skip') nonzero-constant detection
 *                      (src/regressions.py:50, which leads to IndexError at :71)
 *   fm_ts_compact, fm_ts_summary <- fama_macbeth_summary + newey_west_mean_se
 *                      (src/regressions.py:78-131)
 *   fm_rolling_mean <- slopes_df.rolling(window=120, min_periods=60).mean()
 *                      (src/calc_Lewellen_2014.py:926)
 *   fm_predictive   <- build-defined extension: lagged-rolling-coefficient forecasts and
 *                      predictive-slope regressions (paper Table 3; no reference line)
 *   fm_ts_fused     <- fm_ts_compact + fm_ts_summary + fm_rolling_mean + fm_predictive in
 *                      one launch (src/regressions.py:78-131; src/calc_Lewellen_2014.py:926)
 *   fm_forecast     <- build-defined extension A7: per-row F = a_{t-1} + b_{t-1}'x_t
 *   fm_segment_moments, fm_distinct_count <- build_table_1's monthly mean / std(ddof=1)
 *                      and permno nunique (src/calc_Lewellen_2014.py:623-646)
 *   fm_firm_chars   <- get_factors' twelve monthly characteristics: groupby("permno")
 *                      .shift(k) lags, rolling(11).apply(np.prod), rolling(12).sum(),
 *                      rolling(24).sum() and the log / ratio arithmetic of calc_log_size ..
 *                      calc_sales_price (src/calc_Lewellen_2014.py:137-341, called at :537-548)
 *   fm_rolling_std  <- calc_std_12's groupby("permno")["retx"].rolling(252,
 *                      min_periods=100).std() * sqrt(252) (src/calc_Lewellen_2014.py:448-456)
 *   fm_rolling_beta <- calculate_rolling_beta's polars 156-week group_by_dynamic beta
 *                      (src/calc_Lewellen_2014.py:344-434)
 *   fm_ffill_expand <- expand_compustat_annual_to_monthly's per-gvkey monthly reindex +
 *                      forward fill (src/transform_compustat.py:101-172)
 *   fm_sorted_join  <- merge_CRSP_and_Compustat's gvkey and (permno, jdate) equality merges
 *                      (src/transform_compustat.py:218-225)
 *   fm_gen_panel    <- (bench/test data) counter-based synthetic panel, bit-identical to
 *                      fmcore/synth.py
 *
 * Conventions: every pointer is device memory allocated by the caller (PyTorch); the
 * library never allocates device memory and keeps no pointer after return.  `stream` is a
 * hipStream_t passed as void*; all work is enqueued on it asynchronously.  Return 0 on
 * success, < 0 on error (fm_last_error() has the message, per thread).  Panels are
 * column-major SoA: column c of a panel is cols[c*col_stride + row], rows sorted by
 * (month, permno); seg_off[nseg+1] are the month (segment) row offsets.
 */
#ifndef FM_HIP_H
#define FM_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FM_OK 0
#define FM_EINVAL (-1)
#define FM_EHIP (-2)
#define FM_ETOOBIG (-3)

/* per (segment, problem) status bits */
#define FM_ST_FITTED 0x1u
#define FM_ST_SKIPPED 0x2u        /* N < K+1: month absent from the output            */
#define FM_ST_INF_IN_X 0x4u       /* statsmodels MissingDataError('exog contains inf') */
#define FM_ST_INF_IN_Y 0x8u
#define FM_ST_CONST_SUSPECT 0x10u /* near-zero centered variance; exact check pending  */
#define FM_ST_CONST_COL 0x20u     /* nonzero constant regressor -> IndexError          */
#define FM_ST_RANK_DEF 0x40u      /* pinv min-norm solution (a null direction was cut)  */
#define FM_ST_REFIT 0x80u         /* ill-conditioned Sxx (pivot < 1e-6 of its diagonal):
                                     fm_solve_fixup re-solves from the rows (QR + SVD)   */

#define FM_MAX_COLS 31            /* z = [1, cols] fits two 16-wide MFMA tiles          */
#define FM_MAX_MODELS 6
#define FM_MAX_LEVELS 3

typedef struct fm_gram_args {
    const double* cols;       /* [ncols][col_stride] */
    int64_t col_stride;
    int32_t ncols;            /* <= FM_MAX_COLS */
    int32_t nseg;
    const int64_t* seg_off;   /* [nseg+1] */
    const int32_t* chunk_seg; /* [nchunks] segment of each chunk */
    const int64_t* chunk_row; /* [2*nchunks]: (row0, row1) of each chunk, inside one segment */
    int32_t nchunks;
    const double* lo;         /* [ncols][nseg] clip bounds or NULL (NaN bound = none) */
    const double* hi;
    const double* shift;      /* [ncols][nseg] pivot subtracted before accumulation, or NULL */
    const double* inv_scale;  /* [ncols][nseg] multiplier after the shift (standardize), or NULL */
    const uint8_t* level;     /* [rows] universe level 0..nlevels-1, or NULL */
    int32_t nlevels;
    const uint32_t* model_mask;   /* [nmodels] bit c: column c must be non-NaN */
    const uint32_t* model_ymask;  /* [nmodels] bit of the dependent column */
    int32_t nmodels;
    const uint8_t* pattern_id;    /* [1<<nmodels] validity pattern -> id, 255 = drop row */
    int32_t npatterns;            /* buckets = npatterns * nlevels */
    double* partial;              /* [nchunks][nbuckets][zw*(zw+1)/2] packed upper triangle, zw = 16 or 32 */
    uint32_t* flags;              /* [nseg][nmodels] reserved (not written: fm_solve detects inf in
                                     X / y per problem from the Gram diagonal); zeroed by caller */
    const int32_t* chunk_order;   /* [nchunks] chunk processed by workgroup b, or NULL: chunks in
                                     reverse index order (the months fm_select streamed last, still
                                     in the Infinity Cache, first).  Only the launch order: each
                                     chunk's partial is the same either way */
    /* optional: cols as 32-bit planes (fm_split_planes / fm_gen_panel_planes, [ncols][plane_stride]
     * each): rows are read from the planes instead of cols (the same bytes; the high plane
     * fm_select just streamed is still in the Infinity Cache), and cols may be NULL.  NULL: cols */
    const uint32_t* hi_plane;
    const uint32_t* lo_plane;
    int64_t plane_stride;
    /* optional balanced plan: workgroup b accumulates chunks [wg_chunk_off[b], wg_chunk_off[b+1])
     * one after another (a chunk still lies inside one segment; a workgroup's chunks are
     * consecutive, so a workgroup can take the tail of one month and the head of the next and
     * every workgroup gets the same number of rows).  NULL: one chunk per workgroup */
    const int32_t* wg_chunk_off;
    int32_t nwg;
} fm_gram_args;
/* The argument structs (fm_gram_args, fm_solve_args, fm_select_args, ...) grow at the end:
 * zero-initialize them before filling fields, so fields a caller does not know are NULL / 0. */

typedef struct fm_solve_args {
    const double* partial;        /* from fm_gram */
    const int32_t* seg_chunk_off; /* [nseg+1] chunk range of each segment */
    int32_t nseg;
    int32_t zw;                   /* 16 or 32 */
    int32_t nlevels;
    int32_t npatterns;
    const uint32_t* pattern_models; /* [npatterns] bitmask of models valid in that pattern */
    int32_t nprob;
    const int32_t* prob_model;    /* [nprob] */
    const int32_t* prob_level;    /* [nprob] universe level u: buckets with level >= u */
    const int32_t* prob_z;        /* [nprob][32] z indices: 0 (intercept), x..., y */
    const int32_t* prob_nz;       /* [nprob] number of z indices P+1 (<= 32) */
    const int32_t* prob_flags;    /* [nprob] bit0: check nonzero-constant columns */
    const double* add_back;       /* [ncols][nseg] shift to add back for raw intercept, or NULL */
    const uint32_t* gram_flags;   /* [nseg][nmodels] extra FM_ST_INF_* bits OR-ed in, or NULL */
    int32_t nmodels;
    int32_t pmax;                 /* >= max P (= K+1) over problems, <= 32 */
    double* rec;                  /* [nseg][nprob][pmax+2]: intercept, slopes..., NaN pad,
                                     R2 at [pmax], N at [pmax+1] */
    uint32_t* status;             /* [nseg][nprob] FM_ST_* bits */
    double* moments;              /* [nseg][nprob][mom_stride] or NULL: n, means(K+1), centered (K+1)^2 */
    int32_t mom_stride;
    int32_t ab_ncols;             /* rows of add_back ([ab_ncols][nseg]; the panel's ncols) */
    /* The statsmodels fix-ups of fm_solve_fixup (npairs = -1) inside this launch, by each
     * month's own workgroup right after its solve (zw 16 only; fix_cols NULL -- the
     * zero-initialised default -- leaves them to a separate fm_solve_fixup call).  The
     * arguments are fm_solve_fixup's: the panel columns the Gram read, its cuts, standardizing
     * shift / scale, universe levels; moments must be set. */
    const double* fix_cols;
    int64_t fix_stride;
    const int64_t* fix_seg_off;
    const double* fix_lo;
    const double* fix_hi;
    const double* fix_shift;
    const double* fix_inv_scale;
    const uint8_t* fix_level;
    int32_t fix_check_const;
    int32_t fix_pad;
    /* the fix-ups' rows from the split panel's planes instead (fix_cols NULL; plane stride =
     * fix_stride): a panel that holds no FP64 columns */
    const uint32_t* fix_hi_plane;
    const uint32_t* fix_lo_plane;
} fm_solve_args;

const char* fm_version(void);
const char* fm_last_error(void);
int fm_abi_sizes(int32_t* gram_args, int32_t* solve_args);
/* sizeof the named argument struct ("fm_gram_args", "fm_solve_args", "fm_select_args",
 * "fm_universe_args", "fm_ts_args", "fm_chars_args"); -1 for an unknown name.  Bindings
 * check their struct layouts against it before the first call. */
int64_t fm_struct_size(const char* name);
int fm_device_arch(char* buf, int32_t len);

int fm_select_cuts(const double* cols, int64_t col_stride, int32_t ncols,
                   const int64_t* seg_off, int32_t nseg, int32_t max_seg_len,
                   const uint8_t* row_mask, double q_lo, double q_hi, int32_t min_count,
                   int32_t lerp_mode, double* lo, double* hi, int32_t* nvalid,
                   double* mean, double* sd, void* ws, void* stream);

/* Bytes of fm_select_args.ws for a call over nseg x ncols units of <= max_seg_len rows (the
 * fix-up worklist; past 6,144 rows also the zero-sign replay slots).  The caller zeroes the
 * buffer ONCE; every fm_select / fm_select_cuts / fm_select_universe call leaves it zeroed,
 * so one buffer serves any number of calls on one stream.  < 0: bad sizes. */
int64_t fm_select_ws_bytes(int32_t nseg, int32_t ncols, int32_t max_seg_len);

/* fm_select: fm_select_cuts with an argument struct and one more optional output.
 * Outputs are [ncols][nseg]; every output pointer except lo / hi may be NULL.
 *   mean, sd: moments of the clipped values (ddof = 1), for the per-month standardization;
 *   center:   a pivot inside the data for the Gram (midpoint of the cuts, else of the
 *             segment's finite range, else 0); costs nothing beyond the cuts;
 *   level:    the universe level byte of every row from the two cuts (see the field).
 * ws is required (nvalid enables the wave fast paths).  Every path ends with a fix-up launch that redoes, exactly, the
 * units the fast kernels could not finish and the units whose numpy cut is exactly +-0: for
 * those, when the unit holds both -0.0 and +0.0, numpy 1.26.4's partition order is replayed
 * (np.percentile takes the sign of a zero cut from it; reference :519-524), so the cuts are
 * bit-exact including that sign.  The struct must be zero-initialized before filling it (new
 * trailing fields are then NULL / 0). */
typedef struct fm_select_args {
    const double* cols;
    int64_t col_stride;
    int32_t ncols;
    const int64_t* seg_off;
    int32_t nseg;
    int32_t max_seg_len;
    const uint8_t* row_mask;     /* [rows] nonzero = row takes part, or NULL */
    double q_lo, q_hi;           /* quantiles in [0, 1] */
    int32_t min_count;           /* fewer valid values: cuts are NaN (no clipping) */
    int32_t lerp_mode;           /* 0 numpy 'linear', 1 pandas groupby.quantile */
    double* lo;
    double* hi;
    int32_t* nvalid;
    double* mean;
    double* sd;
    double* center;
    uint8_t* level;              /* [rows] or NULL; ncols == 1 only: every row's universe level
                                    (x >= lo) + (x >= hi) of the UNMASKED column (NaN compares
                                    False), i.e. get_subsets' nested masks from the NYSE cuts
                                    (src/calc_Lewellen_2014.py:95-105), by a streaming
                                    launch after the cuts (same stream) */
    void* ws;                    /* fm_select_ws_bytes(nseg, ncols, max_seg_len) bytes, zeroed
                                    once by the caller, left zeroed by every call */
    const uint32_t* hi_plane;    /* optional: the high 32-bit words of cols ([ncols][plane_stride],
                                    fm_split_planes).  The two-wave (<= 6,144-row months) and
                                    long-month kernels then order values by these words (half the
                                    bytes) and gather full values from cols only at the target ranks */
    int64_t plane_stride;
    const uint32_t* lo_plane;    /* optional, with hi_plane: the low words.  With both planes cols may
                                    be NULL (a split panel without FP64 columns): the gathers and the
                                    fix-up paths then read values from the planes.  Paths that need
                                    FP64 columns (moments, row masks, > 20,480-row months) return
                                    FM_EINVAL for such a panel. */
} fm_select_args;

int fm_select(const fm_select_args* args, void* stream);

/* fm_select_universe: fm_select's cuts of `args` AND fm_universe's NYSE breakpoints + level
 * bytes (get_subsets, reference src/calc_Lewellen_2014.py:69-105) over the same month
 * segments (args->seg_off / nseg / max_seg_len), written to cut_a / cut_b [nseg] and level
 * [rows]: the winsorize cuts of calc_Lewellen_2014.py:516-527 and the universes of :74-96 in
 * one call.  Months of <= 5,120 rows (the register select paths) run the universe months in
 * the select fix-up's launch; months of 6,145 .. 20,480 rows (fm_select's long-month path,
 * no row mask, no moments) put them into the long-month launch (one more grid column);
 * otherwise the universe runs first, on its own (fm_universe, or the row-masked select +
 * level bytes past 16,384 rows).  Outputs are identical to fm_select + fm_universe. */
typedef struct fm_universe_args {
    const double* me;            /* [rows] */
    const uint8_t* nyse;         /* [rows] nonzero = NYSE row */
    double q_a, q_b;             /* pandas groupby.quantile levels (0.2, 0.5) */
    double* cut_a;               /* [nseg] */
    double* cut_b;               /* [nseg] */
    uint8_t* level;              /* [rows] (me >= cut_a) + (me >= cut_b) */
} fm_universe_args;

int fm_select_universe(const fm_select_args* args, const fm_universe_args* u, void* stream);

int fm_clip(const double* src, double* dst, int64_t col_stride, int32_t ncols,
            const int64_t* seg_off, int32_t nseg, int64_t nrows,
            const double* lo, const double* hi, void* stream);

int fm_standardize(const double* src, double* dst, int64_t col_stride, int32_t ncols,
                   const int64_t* seg_off, int32_t nseg, int64_t nrows,
                   const double* mean, const double* sd, void* stream);

int fm_universe_level(const double* me, const int64_t* seg_off, int32_t nseg, int64_t nrows,
                      const double* cut_a, const double* cut_b, uint8_t* level, void* stream);

/* fm_universe: per month the pandas-lerp q_a / q_b quantiles of `me` over rows with
 * nyse != 0 (NaN me skipped; no such row -> NaN cuts) into cut_a / cut_b [nseg], and every
 * row's level (me >= cut_a) + (me >= cut_b) (NaN compares False).  Months of at most
 * 64 * 256 rows; longer ones return FM_ETOOBIG (fm_select_cuts with a row mask +
 * fm_universe_level do any length). */
int fm_universe(const double* me, const uint8_t* nyse, const int64_t* seg_off, int32_t nseg,
                int32_t max_seg_len, double q_a, double q_b, double* cut_a, double* cut_b,
                uint8_t* level, void* stream);

int fm_pilot_shift(const double* cols, int64_t col_stride, int32_t ncols,
                   const int64_t* seg_off, int32_t nseg, double* shift, void* stream);

int fm_gram(const fm_gram_args* args, void* stream);

int fm_solve(const fm_solve_args* args, void* stream);

/* fm_const_check / fm_solve_fixup: `pairs` lists (month, problem) int32 pairs; npairs < 0
 * (pairs may be NULL) scans every pair on the device and takes those whose status bits ask
 * for the fix-up (CONST_SUSPECT; FITTED|INF_IN_Y or FITTED|REFIT), so callers need no host
 * round trip.  With check_const != 0, fm_solve_fixup also runs fm_const_check's test on
 * the CONST_SUSPECT pairs (one launch for every fix-up).  It reads the same row set as fm_gram (clip to lo/hi, NaN drop,
 * level >= the problem's); with inv_scale the design value is (x - shift) * inv_scale
 * (+ add_back), without it the raw clipped x (add_back must then restore the shift, as
 * fm_solve assumes). */
int fm_const_check(const double* cols, int64_t col_stride, int32_t ncols,
                   const int64_t* seg_off, int32_t nseg,
                   const double* lo, const double* hi, const uint8_t* level,
                   int32_t nprob, const int32_t* prob_level, const int32_t* prob_z,
                   const int32_t* prob_nz, const int32_t* pairs, int32_t npairs,
                   uint32_t* status, void* stream);

int fm_solve_fixup(const double* cols, int64_t col_stride, const int64_t* seg_off, int32_t nseg,
                   const double* lo, const double* hi, const double* shift, const double* inv_scale,
                   const double* add_back, const uint8_t* level, int32_t nprob,
                   const int32_t* prob_level, const int32_t* prob_z, const int32_t* prob_nz,
                   const int32_t* pairs, int32_t npairs, const double* moments, int32_t mom_stride,
                   int32_t pmax, double* rec, uint32_t* status, int32_t check_const, void* stream);

int fm_ts_compact(const uint32_t* status, int64_t s_seg, int64_t s_prob, int32_t nseg,
                  int32_t nprob, int32_t* idx, int32_t* count, void* stream);

/* fm_ts_summary: work holds nprob * kmax * (nseg + ceil(nseg / 2048) * 28) doubles (series of
 * >= 4096 months take the chunked one-pass kernels, whose partials follow the series). */
int fm_ts_summary(const double* rec, int64_t r_seg, int64_t r_prob, const int32_t* idx,
                  const int32_t* count, int32_t nseg, int32_t nprob, int32_t kmax,
                  int32_t nw_lags, double* mean, double* se, double* tstat, int32_t* nobs,
                  double* work, void* stream);

int fm_rolling_mean(const double* rec, int64_t r_seg, int64_t r_prob, const int32_t* idx,
                    const int32_t* count, int32_t nseg, int32_t nprob, int32_t kmax,
                    int32_t window, int32_t min_periods, double* out, void* stream);

/* fm_rolling_mean for a month-sharded rank: only the output rows a predictive stage of months
 * [seg_lo, seg_hi) reads (the fitted rows of those months and the `lag` rows before the
 * first), computed exactly as fm_rolling_mean computes them (same bits); other rows of `out`
 * are left unwritten (the per-thread row blocks that hold no such row are skipped). */
int fm_rolling_mean_own(const double* rec, int64_t r_seg, int64_t r_prob, const int32_t* idx,
                        const int32_t* count, int32_t nseg, int32_t nprob, int32_t kmax,
                        int32_t window, int32_t min_periods, int32_t seg_lo, int32_t seg_hi,
                        int32_t lag, double* out, void* stream);

int fm_predictive(const double* moments, int32_t mom_stride, int32_t nseg, int32_t nprob,
                  const int32_t* prob_k, const int32_t* idx, const int32_t* count,
                  const double* rolling, int32_t pmax, int32_t lag, int32_t seg_lo,
                  int32_t seg_hi, double* pred, uint32_t* pred_status, void* stream);

/* fm_ts_fused: fm_ts_compact + fm_ts_summary + fm_rolling_mean + fm_predictive in one
 * launch (per problem: a workgroup per coefficient summary and per 64 fitted-month rows of
 * rolling means + predictive slopes, each staging its records in LDS).  roll == NULL skips
 * the rolling and predictive phases, pred == NULL the predictive phase; called on the
 * predictive records (rec = pred, status = pred_status) it gives their FM summary.  Outputs
 * as in the separate entry points; work is unused (may be NULL). */
typedef struct fm_ts_args {
    const double* rec;            /* records, element (month s, problem p, k) at s*r_seg + p*r_prob + k */
    int64_t r_seg, r_prob;
    const uint32_t* status;       /* status of (s, p) at s*s_seg + p*s_prob */
    int64_t s_seg, s_prob;
    int32_t nseg, nprob, kmax, nw_lags;
    int32_t* idx;                 /* [nprob][nseg] fitted months, ascending */
    int32_t* count;               /* [nprob] */
    double* mean;                 /* [nprob][kmax] */
    double* se;
    double* tstat;
    int32_t* nobs;
    double* work;                 /* unused (ABI slot), may be NULL */
    int32_t window, min_periods, pmax;
    double* roll;                 /* [nprob][nseg][pmax] or NULL */
    const double* moments;        /* [seg_hi - seg_lo][nprob][mom_stride] */
    int32_t mom_stride;
    const int32_t* prob_k;        /* [nprob] */
    int32_t lag, seg_lo, seg_hi;
    double* pred;                 /* [nprob][nseg][4] or NULL */
    uint32_t* pred_status;        /* [nprob][nseg] */
    /* Month-sharded runs (zero-initialised = off; every rank runs the stage on the gathered
     * series, each doing only its share):
     *   sum_p_hi > 0: the FM summaries (mean, se, tstat, nobs) of problems [sum_p_lo,
     *     sum_p_hi) only; the other problems' summaries are written as -0.0 / 0, so a SUM
     *     all-reduce over the ranks returns every problem's summary bit for bit;
     *   roll_own != 0: rolling means only in the rolling workgroups whose rows hold a fitted
     *     month in [seg_lo, seg_hi) or one of the `lag` rows before the first such row (the
     *     rows this rank's predictive records read); the other workgroups write no rolling
     *     means (those roll rows are left unwritten) but still their predictive records
     *     (-0.0 / status 0 for other ranks' months).  Computed rows are bit-identical to a
     *     full run's. */
    int32_t sum_p_lo, sum_p_hi;
    int32_t roll_own;
    int32_t pad_ts;
} fm_ts_args;

/* LDS bytes the fused launch stages per workgroup; it must not exceed FM_TS_FUSED_MAX_LDS
 * (otherwise use fm_ts_compact / fm_ts_summary / fm_rolling_mean / fm_predictive). */
#define FM_TS_FUSED_MAX_LDS (128 * 1024)
size_t fm_ts_fused_lds_bytes(int32_t nseg, int32_t pmax, int32_t window, int32_t lag,
                             int32_t rolling, int32_t predictive);
int fm_ts_fused(const fm_ts_args* args, void* stream);

int fm_forecast(const double* cols, int64_t col_stride, int32_t K, const int64_t* seg_off,
                int32_t nseg, int64_t nrows, const double* coef, int32_t coef_stride,
                double* out, void* stream);

int fm_segment_moments(const double* cols, int64_t col_stride, int32_t ncols,
                       const int64_t* seg_off, int32_t nseg, const uint8_t* level,
                       int32_t min_level, int32_t finite_only, int32_t* count, double* mean,
                       double* sd, void* stream);

int fm_distinct_count(const int64_t* ids, int64_t nrows, const double* cols, int64_t col_stride,
                      int32_t ncols, const uint8_t* level, int32_t min_level, int32_t finite_only,
                      int64_t id_lo, int64_t id_range, uint32_t* bitmap, int32_t* out,
                      void* stream);

/* Firm-axis characteristic construction.  Rows are FIRM-major:
 * grouped by firm id (each firm's rows contiguous, in the reference frame's order inside the
 * group — get_factors sorts by (permno, mthcaldt), src/calc_Lewellen_2014.py:533).  Row i's
 * lag-k value exists iff ids[i-k] == ids[i].  field[f] / out[c] are device columns of n
 * doubles indexed by FM_FIELD_* / FM_CHAR_*; out[c] == NULL skips characteristic c, and a
 * requested characteristic needs its fields non-NULL (else FM_EINVAL).  Rolling windows turn
 * +-inf into NaN first (pandas _prep_values). */
#define FM_NFIELDS 12
#define FM_FIELD_ME 0
#define FM_FIELD_BE 1
#define FM_FIELD_RETX 2
#define FM_FIELD_ACCRUALS 3
#define FM_FIELD_DEPRECIATION 4
#define FM_FIELD_EARNINGS 5
#define FM_FIELD_ASSETS 6
#define FM_FIELD_DVC 7
#define FM_FIELD_PRC 8
#define FM_FIELD_SHROUT 9
#define FM_FIELD_TOTAL_DEBT 10
#define FM_FIELD_SALES 11

#define FM_NCHARS 12
#define FM_CHAR_LOG_SIZE 0          /* log(me[t-1])                       :137-147 */
#define FM_CHAR_LOG_BM 1            /* log(be[t-1]) - log(me[t-1])        :150-163 */
#define FM_CHAR_RETURN_12_2 2       /* prod(1 + retx[t-12..t-2]) - 1      :166-192 */
#define FM_CHAR_ACCRUALS_FINAL 3    /* accruals - depreciation            :195-204 */
#define FM_CHAR_ROA 4               /* earnings / assets                  :241-249 */
#define FM_CHAR_LOG_ASSETS_GROWTH 5 /* log(assets / assets[t-12])         :252-262 */
#define FM_CHAR_DY 6                /* sum(dvc[t-11..t], minp 1) / prc[t-1] :265-287 */
#define FM_CHAR_LOG_RETURN_13_36 7  /* sum(log(1 + retx[t-36..t-13]))     :290-313 */
#define FM_CHAR_LOG_ISSUES_12 8     /* log(shrout[t-1]) - log(shrout[t-12]) :224-238 */
#define FM_CHAR_LOG_ISSUES_36 9     /* log(shrout[t-1]) - log(shrout[t-36]) :207-221 */
#define FM_CHAR_DEBT_PRICE 10       /* total_debt / me[t-1]               :316-327 */
#define FM_CHAR_SALES_PRICE 11      /* sales / me[t-1]                    :330-341 */

typedef struct fm_chars_args {
    const int64_t* ids;                 /* [n] firm id per row (grouped)                 */
    int64_t n;
    const double* field[FM_NFIELDS];    /* FM_FIELD_* columns, NULL if absent           */
    double* out[FM_NCHARS];             /* FM_CHAR_* outputs, NULL = not computed       */
} fm_chars_args;

int fm_firm_chars(const fm_chars_args* args, void* stream);

/* Per-row rolling std (ddof=1) over the last `window` rows of each firm group (rows grouped
 * as for fm_firm_chars), NaN below `min_periods` observations, exactly 0 when all
 * observations are equal, times `scale`.  1 <= window <= 4096, 1 <= min_periods <= window
 * (a std needs at least 2 observations, so min_periods 1 behaves as 2).  ids, x and out must be
 * 16-byte aligned (row pairs move as 16-byte accesses); FM_EINVAL otherwise. */
int fm_rolling_std(const int64_t* ids, const double* x, int64_t n, int32_t window,
                   int32_t min_periods, double scale, double* out, void* stream);

/* calculate_rolling_beta's 156-week rolling market beta (src/calc_Lewellen_2014.py:344-434,
 * polars group_by_dynamic(every="1w", period="156w", by="permno"), closed left, label left,
 * windows from the Monday of each firm's first date while the start <= its last date,
 * empty windows not emitted).  Rows: the inner join of daily stock and market returns,
 * firm-major (seg_off[nseg+1] firm row ranges), days ascending within a firm (`day` =
 * days since 1970-01-01); ri / rm the raw daily returns (log(1 + r) is taken here).  Query
 * q = (firm segment q_seg, calendar month [q_day0, q_day1]): the beta of the LAST emitted
 * window starting in that month, NaN if none (the reference's drop_duplicates(keep="last")
 * + left merge, :426-431).  ws: [5][n] workspace.  Parity unpinned (no polars here). */
int fm_rolling_beta(const int32_t* day, const double* ri, const double* rm, int64_t n,
                    const int64_t* seg_off, int32_t nseg, int32_t period_days,
                    const int32_t* q_seg, const int32_t* q_day0, const int32_t* q_day1,
                    int32_t nq, double* ws, double* beta, void* stream);

int fm_gen_panel(uint64_t seed, int64_t month0, int32_t nmonths, int32_t nfirms,
                 double nan_rate, double nyse_rate, double* cols, int64_t col_stride,
                 double* me, uint8_t* nyse, void* stream);

/* fm_gen_panel writing the split layout directly: the values' high / low 32-bit words into
 * hi / lo ([ncols][plane_stride]), the FP64 columns into cols too when cols != NULL (else
 * not at all).  The same values as fm_gen_panel bit for bit; no separate layout pass. */
int fm_gen_panel_planes(uint64_t seed, int64_t month0, int32_t nmonths, int32_t nfirms,
                        double nan_rate, double nyse_rate, double* cols, int64_t col_stride,
                        uint32_t* hi, uint32_t* lo, int64_t plane_stride, double* me, uint8_t* nyse,
                        void* stream);

/* The inverse of fm_split_planes: FP64 columns from the two planes (for consumers of a split
 * panel that read FP64 columns: clip, forecasts, Table 1, moments). */
int fm_merge_planes(const uint32_t* hi, const uint32_t* lo, int64_t plane_stride, int32_t ncols, int64_t nrows,
                    double* cols, int64_t col_stride, void* stream);

/* The FP64 columns as two 32-bit planes: hi[c][r] / lo[c][r] = the high / low words of
 * cols[c][r] (plane_stride >= nrows).  The split panel's hi plane feeds fm_select_args.hi_plane
 * and, with the lo plane, fm_gram_args.hi_plane / lo_plane. */
int fm_split_planes(const double* cols, int64_t col_stride, int32_t ncols, int64_t nrows, uint32_t* hi,
                    uint32_t* lo, int64_t plane_stride, void* stream);
int fm_stream_probe(const double* src, int64_t n, double* out, void* stream);
/* Copy n doubles src -> dst as the probe's 16-byte stream (measures the HBM copy rate;
 * bench.py's measured_copy_peak).  src / dst 16-byte aligned, not overlapping. */
int fm_stream_copy_probe(const double* src, double* dst, int64_t n, void* stream);

/* fm_ffill_expand: records sorted by (group, month code) with CSR rec_off[ngroups+1];
 * out_off[ngroups+1] is the prefix of each group's output month count (planned by the
 * caller: from its first record month to its last output month).  Output row i of group g
 * is month rec_month[rec_off[g]] + (i - out_off[g]); it takes the group's last record with
 * rec_month <= that month: out_src[i] = that record, out_month[i] = the month, and the
 * ncols FP64 columns vals[c * v_stride + record] are gathered to out_vals[c * o_stride + i]. */
int fm_ffill_expand(const int64_t* rec_off, const int32_t* rec_month, const int64_t* out_off,
                    int32_t ngroups, int64_t nout, const double* vals, int64_t v_stride,
                    int32_t ncols, double* out_vals, int64_t o_stride, int32_t* out_month,
                    int64_t* out_src, void* stream);

/* fm_sorted_join: for each left key (lk1[i], lk2[i]) the range [lo[i], hi[i]) of equal keys
 * in the right keys (rk1, rk2), sorted lexicographically (stably: equal keys in the right
 * frame's order).  lk2 / rk2 may both be NULL (one-part key). */
int fm_sorted_join(const int64_t* lk1, const int64_t* lk2, int64_t nl, const int64_t* rk1,
                   const int64_t* rk2, int64_t nr, int64_t* lo, int64_t* hi, void* stream);

#ifdef __cplusplus
}
#endif
#endif

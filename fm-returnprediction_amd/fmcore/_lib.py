"""ctypes binding of libfm_hip.so (include/fm_hip.h).

The shared library is built in-tree (``fm-returnprediction_amd/lib/libfm_hip.so``, see
``csrc/Makefile`` / ``__graft_entry__.build()``).  There is no fallback: if the library is
missing, or no HIP device is present when a compute entry point is used, this module
raises.  All pointer arguments are device pointers taken from torch tensors.
"""
from __future__ import annotations

import ctypes as C
import os

_PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("FM_HIP_LIB", os.path.join(_PKG_DIR, "lib", "libfm_hip.so"))

FM_ST_FITTED = 0x1
FM_ST_SKIPPED = 0x2
FM_ST_INF_IN_X = 0x4
FM_ST_INF_IN_Y = 0x8
FM_ST_CONST_SUSPECT = 0x10
FM_ST_CONST_COL = 0x20
FM_ST_RANK_DEF = 0x40
FM_ST_REFIT = 0x80

FM_MAX_COLS = 31
FM_MAX_MODELS = 6
FM_MAX_LEVELS = 3
FM_TS_FUSED_MAX_LDS = 128 * 1024

_p = C.c_void_p
_i32 = C.c_int32
_i64 = C.c_int64
_f64 = C.c_double


class GramArgs(C.Structure):
    _fields_ = [
        ("cols", _p), ("col_stride", _i64), ("ncols", _i32), ("nseg", _i32),
        ("seg_off", _p), ("chunk_seg", _p), ("chunk_row", _p), ("nchunks", _i32),
        ("lo", _p), ("hi", _p), ("shift", _p), ("inv_scale", _p),
        ("level", _p), ("nlevels", _i32),
        ("model_mask", _p), ("model_ymask", _p), ("nmodels", _i32),
        ("pattern_id", _p), ("npatterns", _i32),
        ("partial", _p), ("flags", _p), ("chunk_order", _p),
        ("hi_plane", _p), ("lo_plane", _p), ("plane_stride", _i64),
        ("wg_chunk_off", _p), ("nwg", _i32),
    ]


class SelectArgs(C.Structure):
    _fields_ = [
        ("cols", _p), ("col_stride", _i64), ("ncols", _i32), ("seg_off", _p), ("nseg", _i32),
        ("max_seg_len", _i32), ("row_mask", _p), ("q_lo", _f64), ("q_hi", _f64),
        ("min_count", _i32), ("lerp_mode", _i32), ("lo", _p), ("hi", _p), ("nvalid", _p),
        ("mean", _p), ("sd", _p), ("center", _p), ("level", _p), ("ws", _p),
        ("hi_plane", _p), ("plane_stride", _i64), ("lo_plane", _p),
    ]


class UniverseArgs(C.Structure):
    _fields_ = [
        ("me", _p), ("nyse", _p), ("q_a", _f64), ("q_b", _f64), ("cut_a", _p), ("cut_b", _p),
        ("level", _p),
    ]


class TsArgs(C.Structure):
    _fields_ = [
        ("rec", _p), ("r_seg", _i64), ("r_prob", _i64), ("status", _p), ("s_seg", _i64),
        ("s_prob", _i64), ("nseg", _i32), ("nprob", _i32), ("kmax", _i32), ("nw_lags", _i32),
        ("idx", _p), ("count", _p), ("mean", _p), ("se", _p), ("tstat", _p), ("nobs", _p),
        ("work", _p), ("window", _i32), ("min_periods", _i32), ("pmax", _i32), ("roll", _p),
        ("moments", _p), ("mom_stride", _i32), ("prob_k", _p), ("lag", _i32), ("seg_lo", _i32),
        ("seg_hi", _i32), ("pred", _p), ("pred_status", _p),
        # month-sharded runs: problem range of the summaries, own-rows rolling (0 = off)
        ("sum_p_lo", _i32), ("sum_p_hi", _i32), ("roll_own", _i32), ("pad_ts", _i32),
    ]


class SolveArgs(C.Structure):
    _fields_ = [
        ("partial", _p), ("seg_chunk_off", _p), ("nseg", _i32), ("zw", _i32),
        ("nlevels", _i32), ("npatterns", _i32), ("pattern_models", _p),
        ("nprob", _i32), ("prob_model", _p), ("prob_level", _p), ("prob_z", _p),
        ("prob_nz", _p), ("prob_flags", _p), ("add_back", _p), ("gram_flags", _p),
        ("nmodels", _i32), ("pmax", _i32), ("rec", _p), ("status", _p),
        ("moments", _p), ("mom_stride", _i32), ("ab_ncols", _i32),
        # inline statsmodels fix-ups (fix_cols None: a separate fm_solve_fixup call)
        ("fix_cols", _p), ("fix_stride", _i64), ("fix_seg_off", _p), ("fix_lo", _p), ("fix_hi", _p),
        ("fix_shift", _p), ("fix_inv_scale", _p), ("fix_level", _p), ("fix_check_const", _i32),
        ("fix_pad", _i32),
        # a planes-only panel's fix-up rows (fix_cols None; stride = fix_stride)
        ("fix_hi_plane", _p), ("fix_lo_plane", _p),
    ]


FM_NFIELDS = 12
FM_NCHARS = 12


class CharsArgs(C.Structure):
    _fields_ = [("ids", _p), ("n", _i64), ("field", _p * FM_NFIELDS), ("out", _p * FM_NCHARS)]


# name -> (restype, argtypes)
_SIGS = {
    "fm_version": (C.c_char_p, []),
    "fm_last_error": (C.c_char_p, []),
    "fm_device_arch": (_i32, [C.c_char_p, _i32]),
    "fm_abi_sizes": (_i32, [C.POINTER(_i32), C.POINTER(_i32)]),
    "fm_struct_size": (_i64, [C.c_char_p]),
    "fm_select_cuts": (_i32, [_p, _i64, _i32, _p, _i32, _i32, _p, _f64, _f64, _i32, _i32,
                              _p, _p, _p, _p, _p, _p, _p]),
    "fm_select_ws_bytes": (_i64, [_i32, _i32, _i32]),
    "fm_split_planes": (_i32, [_p, _i64, _i32, _i64, _p, _p, _i64, _p]),
    "fm_select": (_i32, [C.POINTER(SelectArgs), _p]),
    "fm_select_universe": (_i32, [C.POINTER(SelectArgs), C.POINTER(UniverseArgs), _p]),
    "fm_clip": (_i32, [_p, _p, _i64, _i32, _p, _i32, _i64, _p, _p, _p]),
    "fm_standardize": (_i32, [_p, _p, _i64, _i32, _p, _i32, _i64, _p, _p, _p]),
    "fm_universe_level": (_i32, [_p, _p, _i32, _i64, _p, _p, _p, _p]),
    "fm_universe": (_i32, [_p, _p, _p, _i32, _i32, _f64, _f64, _p, _p, _p, _p]),
    "fm_sorted_join": (_i32, [_p, _p, _i64, _p, _p, _i64, _p, _p, _p]),
    "fm_ffill_expand": (_i32, [_p, _p, _p, _i32, _i64, _p, _i64, _i32, _p, _i64, _p, _p, _p]),
    "fm_pilot_shift": (_i32, [_p, _i64, _i32, _p, _i32, _p, _p]),
    "fm_gram": (_i32, [C.POINTER(GramArgs), _p]),
    "fm_solve": (_i32, [C.POINTER(SolveArgs), _p]),
    "fm_const_check": (_i32, [_p, _i64, _i32, _p, _i32, _p, _p, _p, _i32, _p, _p, _p, _p,
                              _i32, _p, _p]),
    "fm_solve_fixup": (_i32, [_p, _i64, _p, _i32, _p, _p, _p, _p, _p, _p, _i32, _p, _p, _p, _p, _i32,
                            _p, _i32, _i32, _p, _p, _i32, _p]),
    "fm_ts_compact": (_i32, [_p, _i64, _i64, _i32, _i32, _p, _p, _p]),
    "fm_ts_summary": (_i32, [_p, _i64, _i64, _p, _p, _i32, _i32, _i32, _i32, _p, _p, _p, _p,
                             _p, _p]),
    "fm_rolling_mean": (_i32, [_p, _i64, _i64, _p, _p, _i32, _i32, _i32, _i32, _i32, _p, _p]),
    "fm_rolling_mean_own": (_i32, [_p, _i64, _i64, _p, _p, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _i32,
                                   _p, _p]),
    "fm_predictive": (_i32, [_p, _i32, _i32, _i32, _p, _p, _p, _p, _i32, _i32, _i32, _i32, _p, _p,
                             _p]),
    "fm_ts_fused": (_i32, [C.POINTER(TsArgs), _p]),
    "fm_ts_fused_lds_bytes": (C.c_size_t, [_i32, _i32, _i32, _i32, _i32, _i32]),
    "fm_forecast": (_i32, [_p, _i64, _i32, _p, _i32, _i64, _p, _i32, _p, _p]),
    "fm_segment_moments": (_i32, [_p, _i64, _i32, _p, _i32, _p, _i32, _i32, _p, _p, _p, _p]),
    "fm_distinct_count": (_i32, [_p, _i64, _p, _i64, _i32, _p, _i32, _i32, _i64, _i64, _p, _p, _p]),
    "fm_firm_chars": (_i32, [C.POINTER(CharsArgs), _p]),
    "fm_rolling_std": (_i32, [_p, _p, _i64, _i32, _i32, _f64, _p, _p]),
    "fm_rolling_beta": (_i32, [_p, _p, _p, _i64, _p, _i32, _i32, _p, _p, _p, _i32, _p, _p, _p]),
    "fm_gen_panel": (_i32, [C.c_uint64, _i64, _i32, _i32, _f64, _f64, _p, _i64, _p, _p, _p]),
    "fm_gen_panel_planes": (_i32, [C.c_uint64, _i64, _i32, _i32, _f64, _f64, _p, _i64, _p, _p, _i64, _p, _p, _p]),
    "fm_merge_planes": (_i32, [_p, _p, _i64, _i32, _i64, _p, _i64, _p]),
    "fm_stream_probe": (_i32, [_p, _i64, _p, _p]),
    "fm_stream_copy_probe": (_i32, [_p, _p, _i64, _p]),
}

EXPORTED = tuple(_SIGS)
_STRUCTS = {"fm_gram_args": GramArgs, "fm_solve_args": SolveArgs, "fm_select_args": SelectArgs,
            "fm_universe_args": UniverseArgs, "fm_ts_args": TsArgs, "fm_chars_args": CharsArgs}

_lib = None


class FMError(RuntimeError):
    """A libfm_hip entry point returned an error code."""


def load():
    """Load libfm_hip.so (once).  Raises ImportError if it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"libfm_hip.so not found at {LIB_PATH}; build it with "
            "`make -C fm-returnprediction_amd/csrc` or `python -c 'import __graft_entry__ as g; g.build()'`")
    lib = C.CDLL(LIB_PATH)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    # the argument structs must match the library's layouts byte for byte (a struct shorter
    # than the C one leaves the library reading past it)
    for cname, cls in _STRUCTS.items():
        want = lib.fm_struct_size(cname.encode())
        if want != C.sizeof(cls):
            raise ImportError(f"ABI mismatch: {cname} is {want} bytes in libfm_hip.so, "
                              f"{C.sizeof(cls)} in fmcore._lib.{cls.__name__}")
    _lib = lib
    return lib


def call(name, *args):
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        msg = lib.fm_last_error().decode(errors="replace")
        raise FMError(f"{name} failed ({rc}): {msg}")
    return rc


def version():
    return load().fm_version().decode()

"""ctypes binding of the C ABI in ``include/fv3net_amd.h``.

The product path has exactly one implementation: the HIP library.  If it is
missing or fails to load, every call raises ``NativeLibraryError`` — there is no
CPU fallback anywhere in ``fv3net_amd``.
"""
import ctypes
import os
import threading

from .build import LIB

FV3_OK = 0
FV3_ERR_INVALID = 1
FV3_ERR_HIP = 2
FV3_ERR_UNSUPPORTED = 3

# every symbol include/fv3net_amd.h declares
EXPORTED_SYMBOLS = (
    "fv3_last_error",
    "fv3_abi_version",
    "fv3_build_kind",
    "fv3_mappm",
    "fv3_mappm_ex",
    "fv3_mappm_multi",
    "fv3_dense_create",
    "fv3_dense_destroy",
    "fv3_dense_k_in",
    "fv3_dense_k_out",
    "fv3_dense_forward",
    "fv3_dense_forward_f64in",
    "fv3_dense_forward_ex",
    "fv3_dense_set_trace",
    "fv3_regrid_coarsen",
    "fv3_regrid_coarsen_f64",
    "fv3_regrid_coarsen_f64d",
    "fv3_weighted_block_average",
    "fv3_weighted_block_average_f64",
    "fv3_hydrostatic_balance",
    "fv3_regrid_coarsen_edge",
    "fv3_regrid_coarsen_edge_f64",
    "fv3_interpolate_2d",
    "fv3_interpolate_levels",
    "fv3_pressure_midpoint_log",
    "fv3_column_integral",
    "fv3_area_weighted_sums",
    "fv3_area_weighted_sums_f64",
    "fv3_level_sums",
    "fv3_level_sums_f64",
    "fv3_level_sums_u8",
    "fv3_area_weighted_row_sums",
    "fv3_area_weighted_row_sums_f64",
    "fv3_level_row_sums_u8",
    "fv3_level_row_sums_f64",
    "fv3_fold_rows",
    "fv3_step_partials_f64",
    "fv3_fold_rows_repeat",
    "fv3_ml_epilogue",
    "fv3_ml_epilogue_ex",
    "fv3_tendency_columns",
    "fv3_range_mask",
    "fv3_time_blend",
    "fv3_classify_one_hot",
    "fv3_zc_infer_gscond_cloud",
    "fv3_zc_squash",
    "fv3_zc_zero_where",
    "fv3_zc_gscond_update",
    "fv3_zc_ice_water_flag",
    "fv3_zc_precpd_conservative",
    "fv3_zc_precip_simple",
    "fv3_standard_normalize",
    "fv3_standard_denormalize",
    "fv3_standard_normalize_f64",
    "fv3_standard_denormalize_f64",
    "fv3_member_reduce",
    "fv3_scale_levels",
    "fv3_adapter_apply",
    "fv3_derived_elementwise",
    "fv3_derived_columns",
    "fv3_host_copy",
    "fv3_host_alloc",
    "fv3_host_free",
    "fv3_host_arena_limit",
    "fv3_host_arena_cap",
    "fv3_host_memory_stats",
    "fv3_copy_to_host",
    "fv3_copy_2d",
    "fv3_center_rotate_winds",
    "fv3_sum_squares",
    "fv3_cos_zenith",
    "fv3_minmax_scores",
    "fv3_taper_columns",
)
ABI_VERSION = 11
# the remap arithmetic of fv3_mappm_ex / _multi and the fused coarsen entries
ARITH_EXACT = 0  # bit-identical to the reference build (mappm.f90 under flang)
ARITH_FAST = 1   # north_star's 1e-5 rel contract: reciprocal divisions, FMA, hardware MAX / MIN


def arith(exact: bool) -> int:
    return ARITH_EXACT if exact else ARITH_FAST

# fv3_dense_forward_ex precisions
DENSE_F32 = 0
DENSE_BF16X3 = 1
DENSE_BF16X6 = 2

# fv3_ml_epilogue_ex flags, fv3_tendency_columns modes
EPI_HAS_DQ1 = 1
EPI_HAS_DQ2 = 2
TEND_WIND = 0
TEND_MASS = 1

# fv3_member_reduce reductions; fv3_adapter_apply limits
REDUCE_MEAN = 0
REDUCE_MEDIAN = 1
ADAPTER_MAX_PREDS = 8
ADAPTER_MAX_TARGETS = 16

# fv3_zc_gscond_update modes
ZC_CLOUD_EMULATOR = 0
ZC_CLOUD_IDENTICAL = 1
ZC_CLOUD_VANISHES = 2
ZC_CLOUD_CLASS_ZERO = 3
ZC_CLOUD_CLASS_NOTEND = 4
ZC_PHASE_DEPENDENT = 5


class NativeLibraryError(RuntimeError):
    """The HIP extension is missing or unusable (no fallback exists)."""


class Layout(ctypes.Structure):
    _fields_ = [("ncol_blk", ctypes.c_int64), ("ld", ctypes.c_int64), ("blk_stride", ctypes.c_int64)]


class DenseDesc(ctypes.Structure):
    _fields_ = [
        ("n_in", ctypes.c_int),
        ("in_nz", ctypes.POINTER(ctypes.c_int)),
        ("in_clip", ctypes.POINTER(ctypes.c_int)),
        ("in_mean", ctypes.POINTER(ctypes.c_float)),
        ("in_sigma", ctypes.POINTER(ctypes.c_float)),
        ("epsilon", ctypes.c_float),
        ("width", ctypes.c_int),
        ("n_hidden", ctypes.c_int),
        ("hidden_kernel", ctypes.POINTER(ctypes.POINTER(ctypes.c_float))),
        ("hidden_bias", ctypes.POINTER(ctypes.POINTER(ctypes.c_float))),
        ("n_out", ctypes.c_int),
        ("out_nz", ctypes.POINTER(ctypes.c_int)),
        ("out_kernel", ctypes.POINTER(ctypes.POINTER(ctypes.c_float))),
        ("out_bias", ctypes.POINTER(ctypes.POINTER(ctypes.c_float))),
        ("out_mean", ctypes.POINTER(ctypes.c_float)),
        ("out_sigma", ctypes.POINTER(ctypes.c_float)),
        ("out_min", ctypes.POINTER(ctypes.c_float)),
        ("out_max", ctypes.POINTER(ctypes.c_float)),
        ("out_mask", ctypes.POINTER(ctypes.c_float)),
        ("in_log_eps", ctypes.POINTER(ctypes.c_float)),
        ("out_residual", ctypes.POINTER(ctypes.c_int)),
    ]


class EpilogueIO(ctypes.Structure):
    _fields_ = [
        ("dq1", ctypes.c_void_p),
        ("dq2", ctypes.c_void_p),
        ("sphum", ctypes.c_void_p),
        ("delp", ctypes.c_void_p),
        ("temperature", ctypes.c_void_p),
        ("physics_precip", ctypes.c_void_p),
        ("dq1_out", ctypes.c_void_p),
        ("dq2_out", ctypes.c_void_p),
        ("limiter_active", ctypes.c_void_p),
        ("temperature_out", ctypes.c_void_p),
        ("sphum_out", ctypes.c_void_p),
        ("column", ctypes.c_void_p),
        ("column_ld", ctypes.c_int64),
    ]


class AdapterTarget(ctypes.Structure):
    _fields_ = [
        ("preds", ctypes.c_void_p * 8),
        ("n_preds", ctypes.c_int),
        ("state", ctypes.c_void_p),
        ("out", ctypes.c_void_p),
        ("pred_f64", ctypes.c_uint),
        ("out_f64", ctypes.c_int),
    ]


class Field(ctypes.Structure):
    """fv3_field: a float32 / float64 [level][column] operand of fv3_derived_columns."""
    _fields_ = [
        ("data", ctypes.c_void_p),
        ("f64", ctypes.c_int),
        ("lay", Layout),
    ]


MAX_DIMS = 6

# the out-of-sample composite (fv3_minmax_scores / fv3_taper_columns)
NOV_MAX_VARS = 16
NOV_MAX_FIELDS = 16
TAPER_MASK = 0
TAPER_RAMP = 1
TAPER_DECAY = 2


class NovVar(ctypes.Structure):
    """fv3_nov_var: one input variable of the min-max detector, levels [z0, z0 + nfeat)."""
    _fields_ = [("data", ctypes.c_void_p), ("layout", Layout), ("data_f64", ctypes.c_int), ("z0", ctypes.c_int),
                ("nfeat", ctypes.c_int)]


class TaperField(ctypes.Structure):
    """fv3_taper_field: one base-model output and its tapered result."""
    _fields_ = [("inp", ctypes.c_void_p), ("in_layout", Layout), ("in_f64", ctypes.c_int), ("out", ctypes.c_void_p),
                ("out_layout", Layout), ("nz", ctypes.c_int)]


class Strided(ctypes.Structure):
    """fv3_strided: a float32 / float64 operand addressed by element strides over the dims
    of a result (0: broadcast)."""
    _fields_ = [
        ("data", ctypes.c_void_p),
        ("f64", ctypes.c_int),
        ("stride", ctypes.c_int64 * MAX_DIMS),
    ]


_lib = None
_lock = threading.Lock()

_P = ctypes.c_void_p
_I = ctypes.c_int
_I64 = ctypes.c_int64
_F = ctypes.c_float
_D = ctypes.c_double

_SIGNATURES = {
    "fv3_last_error": (ctypes.c_char_p, []),
    "fv3_abi_version": (_I, []),
    "fv3_build_kind": (ctypes.c_char_p, []),
    "fv3_mappm": (_I, [_P, _P, _P, _P, _I64, _I, _I, _I, _I, _F, _P]),
    "fv3_mappm_ex": (_I, [_P, Layout, _P, Layout, _P, Layout, _P, Layout, _I64, _I, _I, _I, _I, _F, _I, _P]),
    "fv3_mappm_multi": (_I, [_P, Layout, ctypes.POINTER(_P), ctypes.POINTER(Layout), _P, Layout, ctypes.POINTER(_P),
                             ctypes.POINTER(Layout), _I, _I64, _I, _I, _I, _I, _F, _I, _P]),
    "fv3_dense_create": (_I, [ctypes.POINTER(DenseDesc), ctypes.POINTER(_P)]),
    "fv3_dense_destroy": (_I, [_P]),
    "fv3_dense_set_trace": (_I, [_P, _P]),
    "fv3_dense_k_in": (_I, [_P]),
    "fv3_dense_k_out": (_I, [_P]),
    "fv3_dense_forward": (_I, [_P, ctypes.POINTER(_P), ctypes.POINTER(Layout), ctypes.POINTER(_P),
                               ctypes.POINTER(Layout), _I64, _P]),
    "fv3_dense_forward_f64in": (_I, [_P, ctypes.POINTER(_P), ctypes.POINTER(Layout), ctypes.POINTER(_P),
                               ctypes.POINTER(Layout), _I64, _P]),
    "fv3_dense_forward_ex": (_I, [_P, ctypes.POINTER(_P), ctypes.POINTER(Layout), ctypes.POINTER(_P),
                                  ctypes.POINTER(Layout), _I64, _I, _P]),
    "fv3_regrid_coarsen": (_I, [_P, _P, ctypes.POINTER(_P), ctypes.POINTER(_P), _I, _P, _I, _I, _I,
                                _I, _I, _I, _I, _D, _I, _P]),
    "fv3_regrid_coarsen_f64": (_I, [_P, _P, ctypes.POINTER(_P), ctypes.POINTER(_P), _I, _P, _I, _I, _I,
                                    _I, _I, _I, _I, _D, _I, _P]),
    "fv3_regrid_coarsen_f64d": (_I, [_P, _P, ctypes.POINTER(_P), ctypes.POINTER(_P), _I, _P, _I, _I, _I,
                                     _I, _I, _I, _I, _D, _I, _P]),
    "fv3_weighted_block_average": (_I, [ctypes.POINTER(_P), ctypes.POINTER(_P), _I, _P, _I, _I, _I, _I, _I, _P]),
    "fv3_weighted_block_average_f64": (_I, [ctypes.POINTER(_P), ctypes.POINTER(_P), _I, _P, _I, _I, _I, _I, _I,
                                            _P]),
    "fv3_hydrostatic_balance": (_I, [_P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _D, _P]),
    "fv3_regrid_coarsen_edge": (_I, [_P, _P, ctypes.POINTER(_P), ctypes.POINTER(_P), _I, _I, _I, _I, _I,
                                     _I, _I, _I, _I, _D, _I, _P]),
    "fv3_regrid_coarsen_edge_f64": (_I, [_P, _P, ctypes.POINTER(_P), ctypes.POINTER(_P), _I, _I, _I, _I, _I,
                                         _I, _I, _I, _I, _D, _I, _P]),
    "fv3_interpolate_2d": (_I, [_P, _I64, _P, _I64, _P, _I64, _P, _I64, _I64, _I, _I, _D, _P]),
    "fv3_interpolate_levels": (_I, [_P, _I64, _P, _I64, _I, _P, _I, _I, _P, _I64, _I64, _I, _D, _P]),
    "fv3_pressure_midpoint_log": (_I, [_P, _I, _I64, _P, _I64, _I64, _I, _D, _P]),
    "fv3_column_integral": (_I, [_P, Layout, _P, Layout, _P, _I64, _I, _D, _P]),
    "fv3_area_weighted_sums": (_I, [ctypes.POINTER(_P), _I, _P, _I64, _P, _P]),
    "fv3_area_weighted_sums_f64": (_I, [ctypes.POINTER(_P), _I, _P, _I64, _P, _P]),
    "fv3_level_sums": (_I, [_P, Layout, _I64, _I, _P, _P]),
    "fv3_level_sums_f64": (_I, [_P, Layout, _I64, _I, _P, _P]),
    "fv3_level_sums_u8": (_I, [_P, Layout, _I64, _I, _P, _P]),
    "fv3_area_weighted_row_sums": (_I, [ctypes.POINTER(_P), _I, _P, _I64, _I, _P, _I64, _P]),
    "fv3_area_weighted_row_sums_f64": (_I, [ctypes.POINTER(_P), _I, _P, _I64, _I, _P, _I64, _P]),
    "fv3_level_row_sums_u8": (_I, [_P, _I, _I64, _I, _I64, _P, _I64, _P]),
    "fv3_level_row_sums_f64": (_I, [_P, _I, _I64, _I, _I64, _P, _I64, _P]),
    "fv3_fold_rows": (_I, [_P, _I64, _I, _P, _P]),
    "fv3_step_partials_f64": (_I, [ctypes.POINTER(_P), _I, _P, _I64, _I, _P, _I64, _P, Layout, _I64, _I, _P, _P]),
    "fv3_fold_rows_repeat": (_I, [_P, _I64, _I, _I, _P, _P, _P]),
    "fv3_time_blend": (_I, [_P, _I, _P, _I, _P, _I64, _D, _P]),
    "fv3_range_mask": (_I, [_P, _P, _I64, _D, _D, _I, _I, _I, _P]),
    "fv3_classify_one_hot": (_I, [_P, _I, _I64, _P, _I, _I, _I, _P]),
    "fv3_zc_infer_gscond_cloud": (_I, [_P, _P, _P, _P, _I64, _I, _P]),
    "fv3_zc_squash": (_I, [_P, _P, _D, _P, _P, _I64, _I, _P]),
    "fv3_zc_zero_where": (_I, [_P, _P, _P, _I64, _I, _P]),
    "fv3_zc_gscond_update": (_I, [_I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I64, _I, _P]),
    "fv3_zc_ice_water_flag": (_I, [_P, _P, _D, _P, _I64, _I64, _I, _P]),
    "fv3_zc_precpd_conservative": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I64, _I, _P]),
    "fv3_zc_precip_simple": (_I, [_P, _P, _P, _P, _P, _P, _I, _I64, _I, _P]),
    "fv3_standard_normalize": (_I, [_P, _I, Layout, _P, _P, _I, _P, Layout, _I64, _I, _P]),
    "fv3_standard_denormalize": (_I, [_P, Layout, _P, _P, _I, _P, Layout, _I64, _I, _P]),
    "fv3_standard_normalize_f64": (_I, [_P, _I, Layout, _P, _P, _I, _P, Layout, _I64, _I, _P]),
    "fv3_standard_denormalize_f64": (_I, [_P, Layout, _P, _P, _I, _P, Layout, _I64, _I, _P]),
    "fv3_ml_epilogue": (_I, [ctypes.POINTER(EpilogueIO), Layout, _I64, _I, _I, _D, _I, _I, _P]),
    "fv3_ml_epilogue_ex": (_I, [ctypes.POINTER(EpilogueIO), Layout, _I64, _I, _I, _D, _I, _I, _I, _P]),
    "fv3_tendency_columns": (_I, [_P, _P, _P, _P, _P, _P, Layout, _I64, _I, _I, _I, _D, _P]),
    "fv3_member_reduce": (_I, [ctypes.POINTER(_P), _I, _I64, _I, _I, _P, _P]),
    "fv3_scale_levels": (_I, [_P, _I, Layout, _P, _I64, _I, _P, _P]),
    "fv3_adapter_apply": (_I, [ctypes.POINTER(AdapterTarget), _I, _I64, _I, _D, _I, _I, _I, _P]),
    "fv3_derived_elementwise": (_I, [_I, ctypes.POINTER(_P), ctypes.POINTER(_I), _I, _P, _I, _I64,
                                     ctypes.POINTER(_D), _I, _P]),
    "fv3_host_copy": (_I, [_P, _P, ctypes.c_size_t, _I, _P]),
    "fv3_host_alloc": (_I, [ctypes.c_size_t, ctypes.POINTER(_P)]),
    "fv3_host_free": (_I, [_P]),
    "fv3_host_arena_limit": (_I, [ctypes.c_size_t]),
    "fv3_host_arena_cap": (_I, [ctypes.c_size_t]),
    "fv3_host_memory_stats": (_I, [ctypes.POINTER(ctypes.c_uint64)]),
    "fv3_plan_create": (_I, [ctypes.POINTER(_P)]),
    "fv3_plan_destroy": (_I, [_P]),
    "fv3_plan_size": (_I, [_P]),
    "fv3_plan_run": (_I, [_P, _P]),
    "fv3_plan_add_dense_forward": (_I, [_P, _P, ctypes.POINTER(_P), ctypes.POINTER(Layout), ctypes.POINTER(_P),
                                        ctypes.POINTER(Layout), _I64, _I, _I]),
    "fv3_plan_add_ml_epilogue": (_I, [_P, ctypes.POINTER(EpilogueIO), Layout, _I64, _I, _I, _D, _I, _I, _I]),
    "fv3_plan_add_area_weighted_sums_f64": (_I, [_P, ctypes.POINTER(_P), _I, _P, _I64, _P]),
    "fv3_plan_add_area_weighted_row_sums_f64": (_I, [_P, ctypes.POINTER(_P), _I, _P, _I64, _I, _P, _I64]),
    "fv3_plan_add_level_sums_u8": (_I, [_P, _P, Layout, _I64, _I, _P]),
    "fv3_plan_add_fold_rows": (_I, [_P, _P, _I64, _I, _P]),
    "fv3_plan_add_step_partials_f64": (_I, [_P, ctypes.POINTER(_P), _I, _P, _I64, _I, _P, _I64, _P, Layout, _I64, _I,
                                            _P]),
    "fv3_plan_add_fold_rows_repeat": (_I, [_P, _P, _I64, _I, _I, _P, _P]),
    "fv3_plan_add_copy": (_I, [_P, _P, _P, ctypes.c_size_t]),
    "fv3_plan_add_repeat": (_I, [_P, _P, _P, ctypes.c_size_t, _I]),
    "fv3_copy_to_host": (_I, [_P, _P, ctypes.c_size_t, _P]),
    "fv3_copy_2d": (_I, [_P, ctypes.c_size_t, _P, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int,
                         _P]),
    "fv3_derived_columns": (_I, [_I, ctypes.POINTER(Field), _I, ctypes.POINTER(Field), _I, _I64, _I,
                                 ctypes.POINTER(_D), _I, _P]),
    "fv3_center_rotate_winds": (_I, [_I, ctypes.POINTER(_I64), Strided, _I64, Strided, _I64, ctypes.POINTER(Strided),
                                     _P, _I, _P, _I, _P]),
    "fv3_sum_squares": (_I, [ctypes.POINTER(_P), ctypes.POINTER(_I), _I, _I64, _P, _P]),
    "fv3_minmax_scores": (_I, [ctypes.POINTER(NovVar), _I, _P, _P, _I, _I, _I64, _P, _P]),
    "fv3_taper_columns": (_I, [_P, _I, _I64, _I, _D, _D, _P, ctypes.POINTER(TaperField), _I, _P]),
    "fv3_cos_zenith": (_I, [_I, ctypes.POINTER(_I64), Strided, _I, Strided, _I, ctypes.POINTER(_I64), _P, _I64, _P,
                            _P]),
}


def library_path() -> str:
    """The HIP library; FV3NET_AMD_LIB points at an alternative build (A/B of kernel
    variants in tools/), which must export the same ABI."""
    return os.environ.get("FV3NET_AMD_LIB", LIB)


def load():
    """Load (once) and return the ctypes library; raise if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        path = library_path()
        if not os.path.exists(path):
            raise NativeLibraryError(
                f"fv3net_amd HIP extension not built: {path} is missing "
                "(run `python -m fv3net_amd.build` or __graft_entry__.build()); "
                "there is no CPU fallback"
            )
        try:
            lib = ctypes.CDLL(path)
        except OSError as e:
            raise NativeLibraryError(f"cannot load {path}: {e}") from e
        for name, (res, args) in _SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.fv3_abi_version() != ABI_VERSION:
            raise NativeLibraryError("fv3net_amd ABI version mismatch: rebuild the extension")
        if path == LIB and lib.fv3_build_kind() != b"product":
            # experiment variants (results invalid by construction) load only when named
            # explicitly through FV3NET_AMD_LIB
            raise NativeLibraryError(f"{path} is not a product build: rebuild with fv3net_amd/build.py")
        _lib = lib
    return _lib


def variant(name: str):
    """A kernel-variant selector from the environment (A/B runs and the tests that pin every
    variant): ``os.environ[name]``, but only while ``FV3_VARIANTS=1``; otherwise None, so the
    product path is the same under any environment (the C side reads its selectors the
    same way, csrc/common.h ``variant_env``)."""
    if os.environ.get("FV3_VARIANTS") != "1":
        return None
    return os.environ.get(name)


def check(status: int, what: str = ""):
    """Map a C-ABI status to the reference's exception types."""
    if status == FV3_OK:
        return
    msg = load().fv3_last_error().decode(errors="replace")
    if what:
        msg = f"{what}: {msg}"
    if status == FV3_ERR_INVALID:
        raise ValueError(msg)
    if status == FV3_ERR_UNSUPPORTED:
        raise NotImplementedError(msg)
    raise RuntimeError(msg)


def layout(ncol_blk: int, ld: int, blk_stride: int = 0) -> Layout:
    return Layout(int(ncol_blk), int(ld), int(blk_stride))

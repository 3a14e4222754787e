"""ctypes binding of libgbm.so (include/gbm.h) — the same C ABI a Julia ``ccall`` binds.

The library is loaded from this package directory (built in-tree by ``__graft_entry__.build()``).
There is no fallback: if the HIP library is missing or no GPU is visible, calls raise.
"""
from __future__ import annotations

import ctypes
import os
import threading

import numpy as np

ABI_VERSION = 212  # GBM_VERSION in include/gbm.h
GBM_OK = 0
GBM_E_ARG = -1
GBM_E_NOTPD = -2
GBM_E_HIP = -3
GBM_E_RCCL = -4
GBM_E_OOM = -5
GBM_E_NODEV = -6
GBM_E_DATA = -7

LIB_PATH = os.environ.get("GBM_LIBGBM") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libgbm.so")

# Every symbol include/gbm.h declares (tests check the export table against this list).
EXPORTS = (
    "gbm_version", "gbm_last_error", "gbm_device_count", "gbm_device_allocations", "gbm_release_device_cache",
    "gbm_gblup_fit", "gbm_gblup_fit_reml", "gbm_gblup_fit_dosage_i8", "gbm_gblup_fit_synthetic", "gbm_grm", "gbm_grm_ploidy_aware", "gbm_colstats", "gbm_predict",
    "gbm_dev_npad", "gbm_dev_gdim", "gbm_dev_grm_workspace", "gbm_dev_solve_workspace",
    "gbm_dev_synth_genotypes", "gbm_dev_expand_dosage_i8", "gbm_dev_standardize", "gbm_dev_grm",
    "gbm_dev_grm_syrk", "gbm_dev_grm_reduce", "gbm_dev_grm_slices",
    "gbm_dev_gblup_solve", "gbm_dev_marker_effects",
    "gbm_dev_standardize_gather", "gbm_dev_gblup_terms",
    "gbm_session_create", "gbm_session_create_dosage_i8", "gbm_session_create_synthetic", "gbm_session_destroy", "gbm_session_gblup_fit",
    "gbm_session_predict", "gbm_session_reml_objective", "gbm_session_reml", "gbm_session_stats",
    "gbm_session_ridge_path", "gbm_session_ridge_lambda_max", "gbm_brr_fit",
    "gbm_dev_chol_prepare", "gbm_dev_chol_prepare_cols", "gbm_dev_chol_group_size", "gbm_dev_chol_group", "gbm_dev_chol_factor_diag",
    "gbm_dev_chol_strip_doubles", "gbm_dev_chol_strip_pack", "gbm_dev_chol_strip_unpack", "gbm_dev_chol_finish",
    "gbm_dev_grm_packed_size", "gbm_dev_grm_pack", "gbm_dev_grm_unpack",
    "gbm_debug_brr_stats", "gbm_debug_brr_shape", "gbm_debug_brr_trace", "gbm_debug_chol_flow_trace",
    "gbm_dev_synth_dosage_i8", "gbm_dev_standardize_i8", "gbm_dev_grm_accumulate", "gbm_dev_marker_effects_i8",
    "gbm_debug_oom_retries", "gbm_dev_chol_group_panels", "gbm_dev_chol_group_update", "gbm_dev_chol_strip_unpack_rows", "gbm_dev_chol_lower_copy",
    "gbm_dev_chol_area_doubles", "gbm_dev_chol_area_pack", "gbm_dev_chol_area_unpack",
    "gbm_dev_chol_group_update_cols", "gbm_dev_chol_group_update_tiles", "gbm_dev_grm_exact_workspace", "gbm_dev_grm_exact_i8",
    "gbm_gblup_fit_ex", "gbm_gblup_fit_reml_ex", "gbm_gblup_fit_dosage_i8_ex", "gbm_gblup_fit_synthetic_ex",
    "gbm_session_set_grm_mode", "gbm_session_grm_used", "gbm_debug_rccl_calls", "gbm_debug_xg_choose", "gbm_debug_chol_flow_order",
    "gbm_debug_chol_flow_order_check", "gbm_debug_chol_flow_order_size", "gbm_dev_grm_exact_status", "gbm_debug_set",
)

GBM_GRM_DEFAULT, GBM_GRM_FP64, GBM_GRM_EXACT, GBM_GRM_AUTO, GBM_GRM_DROPIN = -1, 0, 1, 2, 3
GRM_MODES = {None: GBM_GRM_DEFAULT, "default": GBM_GRM_DEFAULT, "fp64": GBM_GRM_FP64, "exact": GBM_GRM_EXACT,
             "auto": GBM_GRM_AUTO, "dropin": GBM_GRM_DROPIN}


def grm_mode(mode) -> int:
    """GBM_GRM_* of a Python/Julia-style mode name (None / "default", "fp64", "exact", "auto")."""
    if isinstance(mode, int) and mode in GRM_MODES.values():
        return mode
    try:
        return GRM_MODES[mode]
    except (KeyError, TypeError):
        raise ArgumentError(f"grm must be one of 'auto', 'exact', 'fp64', 'dropin' or None, got {mode!r}") from None


class ArgumentError(ValueError):
    """Mirrors Julia's ArgumentError thrown by the reference (e.g. src/prediction.jl:67-112)."""


class GBMError(RuntimeError):
    """Mirrors Julia's ErrorException (e.g. src/linear.jl:235-237, src/prediction.jl:125-127)."""


_lock = threading.Lock()
_lib = None

P = ctypes.c_void_p
I64 = ctypes.c_int64
I32 = ctypes.c_int
D = ctypes.c_double
U64 = ctypes.c_uint64


def _declare(lib):
    lib.gbm_version.restype = I32
    lib.gbm_version.argtypes = []
    lib.gbm_last_error.restype = ctypes.c_char_p
    lib.gbm_last_error.argtypes = []
    lib.gbm_device_count.restype = I32
    lib.gbm_device_count.argtypes = [ctypes.POINTER(I32)]
    lib.gbm_device_allocations.restype = I64
    lib.gbm_device_allocations.argtypes = []
    lib.gbm_release_device_cache.restype = I32
    lib.gbm_release_device_cache.argtypes = []
    lib.gbm_dev_chol_prepare.restype = I32
    lib.gbm_dev_chol_prepare.argtypes = [P, I64, I64, D, P, D, P, I64, I64, P, P, I64, P]
    lib.gbm_dev_chol_prepare_cols.restype = I32
    lib.gbm_dev_chol_prepare_cols.argtypes = [P, I64, I64, D, P, D, P, I64, I64, I32, I32, P, P, I64, P]
    lib.gbm_dev_chol_group_size.restype = I64
    lib.gbm_dev_chol_group_size.argtypes = [I64, I64]
    lib.gbm_dev_chol_group.restype = I32
    lib.gbm_dev_chol_group.argtypes = [P, I64, I64, I64, I32, I32, P, P, I64, P]
    for f in ("gbm_dev_chol_group_panels", "gbm_dev_chol_group_update"):
        getattr(lib, f).restype = I32
        getattr(lib, f).argtypes = [P, I64, I64, I64, I32, I32, P, P, I64, P]
    lib.gbm_dev_chol_group_update_cols.restype = I32
    lib.gbm_dev_chol_group_update_cols.argtypes = [P, I64, I64, I64, I32, I32, I64, I64, P, P, I64, P]
    lib.gbm_dev_chol_group_update_tiles.restype = I32
    lib.gbm_dev_chol_group_update_tiles.argtypes = [P, I64, I64, I64, I32, I32, I64, I64, I64, I64, P, P, I64, P]
    lib.gbm_dev_chol_area_doubles.restype = I64
    lib.gbm_dev_chol_area_doubles.argtypes = [I64, I64, I64, I32]
    lib.gbm_dev_chol_area_pack.restype = I32
    lib.gbm_dev_chol_area_pack.argtypes = [P, I64, I64, I64, I64, I32, I32, P, P]
    lib.gbm_dev_chol_area_unpack.restype = I32
    lib.gbm_dev_chol_area_unpack.argtypes = [P, I64, I64, I64, I64, I32, P, P]
    lib.gbm_dev_chol_strip_unpack_rows.restype = I32
    lib.gbm_dev_chol_strip_unpack_rows.argtypes = [P, I64, I64, I64, I64, I32, I32, P, P]
    lib.gbm_dev_chol_lower_copy.restype = I32
    lib.gbm_dev_chol_lower_copy.argtypes = [P, I64, I64, I64, I64, I32, I32, P]
    lib.gbm_dev_chol_factor_diag.restype = I32
    lib.gbm_dev_chol_factor_diag.argtypes = [P, I64, I64, I64, P, P, I64, P]
    lib.gbm_dev_chol_strip_doubles.restype = I64
    lib.gbm_dev_chol_strip_doubles.argtypes = [I64, I64, I64, I32]
    lib.gbm_dev_chol_strip_pack.restype = I32
    lib.gbm_dev_chol_strip_pack.argtypes = [P, I64, I64, I64, I64, I32, I32, P, P]
    lib.gbm_dev_chol_strip_unpack.restype = I32
    lib.gbm_dev_chol_strip_unpack.argtypes = [P, I64, I64, I64, I64, I32, P, P]
    lib.gbm_dev_chol_finish.restype = I32
    lib.gbm_dev_chol_finish.argtypes = [P, I64, I64, P, I64, I64, D, P, P, I64, P, P, P, I64, P]
    lib.gbm_gblup_fit.restype = I32
    lib.gbm_gblup_fit.argtypes = [P, I64, I64, I64, P, I64, I64, D, P, I32, P, P, P, P]
    lib.gbm_gblup_fit_reml.restype = I32
    lib.gbm_gblup_fit_reml.argtypes = [P, I64, I64, I64, P, I64, I64, P, I32, P, P, P, P, P, P, P]
    lib.gbm_gblup_fit_dosage_i8.restype = I32
    lib.gbm_gblup_fit_dosage_i8.argtypes = [P, I64, I64, I64, I32, P, I64, I64, D, P, I32, P, P, P, P]
    lib.gbm_gblup_fit_synthetic.restype = I32
    lib.gbm_gblup_fit_synthetic.argtypes = [U64, I64, I64, P, I64, I64, D, P, I32, P, P, P, P]
    lib.gbm_grm.restype = I32
    lib.gbm_grm.argtypes = [P, I64, I64, I64, P, I32, P, I64, P]
    lib.gbm_grm_ploidy_aware.restype = I32
    lib.gbm_grm_ploidy_aware.argtypes = [P, I64, I64, I64, I32, P, I32, P, I64, P]
    lib.gbm_colstats.restype = I32
    lib.gbm_colstats.argtypes = [P, I64, I64, I64, I32, P, P, P, P]
    lib.gbm_predict.restype = I32
    lib.gbm_predict.argtypes = [P, I64, I64, I64, P, I64, I64, I32, P, I64]
    for f in ("gbm_dev_npad", "gbm_dev_gdim"):
        getattr(lib, f).restype = I64
        getattr(lib, f).argtypes = [I64]
    for f in ("gbm_dev_grm_workspace", "gbm_dev_solve_workspace"):
        getattr(lib, f).restype = I64
        getattr(lib, f).argtypes = [I64, I64]
    lib.gbm_dev_synth_genotypes.restype = I32
    lib.gbm_dev_synth_genotypes.argtypes = [P, I64, I64, I64, U64, I64, P]
    lib.gbm_dev_expand_dosage_i8.restype = I32
    lib.gbm_dev_expand_dosage_i8.argtypes = [P, I64, I64, I64, I32, P, I64, P]
    lib.gbm_dev_standardize.restype = I32
    lib.gbm_dev_standardize.argtypes = [P, I64, I64, I64, P, I64, P, P, P, P, P]
    lib.gbm_dev_synth_dosage_i8.restype = I32
    lib.gbm_dev_synth_dosage_i8.argtypes = [P, I64, I64, I64, U64, I64, P]
    lib.gbm_dev_standardize_i8.restype = I32
    lib.gbm_dev_standardize_i8.argtypes = [P, I64, I64, I64, I32, P, I64, P, P, P, P, P]
    lib.gbm_dev_marker_effects_i8.restype = I32
    lib.gbm_dev_grm_exact_workspace.restype = I64
    lib.gbm_dev_grm_exact_workspace.argtypes = [I64, I64]
    lib.gbm_dev_grm_exact_i8.restype = I32
    lib.gbm_dev_grm_exact_i8.argtypes = [P, I64, I64, I64, I32, P, I64, P, P, P, P, I32, P, I64, P, P]
    lib.gbm_dev_marker_effects_i8.argtypes = [P, I64, I64, I64, I32, P, I64, I64, D, P, P, P, P, P, I64, P, P]
    for f in ("gbm_dev_grm", "gbm_dev_grm_syrk", "gbm_dev_grm_accumulate"):
        getattr(lib, f).restype = I32
        getattr(lib, f).argtypes = [P, I64, I64, I64, P, I64, P, I64, P]
    lib.gbm_dev_grm_reduce.restype = I32
    lib.gbm_dev_grm_reduce.argtypes = [I64, I64, P, I64, P, P]
    lib.gbm_dev_grm_slices.restype = I32
    lib.gbm_dev_grm_slices.argtypes = [I64, I64]
    lib.gbm_dev_gblup_solve.restype = I32
    lib.gbm_dev_gblup_solve.argtypes = [P, I64, I64, D, P, D, P, I64, I64, P, P, I64, P, P, P, I64, P]
    lib.gbm_dev_marker_effects.restype = I32
    lib.gbm_dev_marker_effects.argtypes = [P, I64, I64, I64, P, I64, I64, D, P, P, P, P, P, I64, P, P]
    lib.gbm_dev_standardize_gather.restype = I32
    lib.gbm_dev_standardize_gather.argtypes = [P, I64, I64, P, I64, P, I64, P, P, P, P, I32, P]
    lib.gbm_dev_gblup_terms.restype = I32
    lib.gbm_dev_gblup_terms.argtypes = [P, I64, I64, I64, P, P, P]
    lib.gbm_session_create.restype = I32
    lib.gbm_session_create.argtypes = [P, I64, I64, I64, I32, ctypes.POINTER(P)]
    lib.gbm_session_create_synthetic.restype = I32
    lib.gbm_session_create_synthetic.argtypes = [U64, I64, I64, I32, ctypes.POINTER(P)]
    lib.gbm_session_create_dosage_i8.restype = I32
    lib.gbm_session_create_dosage_i8.argtypes = [P, I64, I64, I64, I32, I32, ctypes.POINTER(P)]
    lib.gbm_session_destroy.restype = None
    lib.gbm_session_destroy.argtypes = [P]
    lib.gbm_session_gblup_fit.restype = I32
    lib.gbm_session_gblup_fit.argtypes = [P, P, I64, P, I64, I64, D, P, P, P, P]
    lib.gbm_session_predict.restype = I32
    lib.gbm_session_predict.argtypes = [P, P, I64, P, I64, I64, P, I64]
    lib.gbm_session_reml_objective.restype = I32
    lib.gbm_session_reml_objective.argtypes = [P, P, I64, P, P, P, I64, P]
    lib.gbm_session_reml.restype = I32
    lib.gbm_session_reml.argtypes = [P, P, I64, P, P, P, P, P]
    lib.gbm_session_ridge_path.restype = I32
    lib.gbm_session_ridge_path.argtypes = [P, P, I64, P, P, I64, P, P, I64, P]
    lib.gbm_session_ridge_lambda_max.restype = I32
    lib.gbm_session_ridge_lambda_max.argtypes = [P, P, I64, P, P]
    lib.gbm_dev_grm_packed_size.restype = I64
    lib.gbm_dev_grm_packed_size.argtypes = [I64]
    lib.gbm_dev_grm_pack.restype = I32
    lib.gbm_dev_grm_pack.argtypes = [P, I64, I64, P, P]
    lib.gbm_dev_grm_unpack.restype = I32
    lib.gbm_dev_grm_unpack.argtypes = [P, I64, P, I64, P]
    lib.gbm_brr_fit.restype = I32
    lib.gbm_brr_fit.argtypes = [P, I64, I64, I64, P, I64, I64, I64, D, D, U64, I32, P, P, P]
    lib.gbm_debug_oom_retries.restype = I32
    lib.gbm_debug_oom_retries.argtypes = [P, P]
    lib.gbm_session_stats.restype = I32
    lib.gbm_session_stats.argtypes = [P, P, P]
    lib.gbm_gblup_fit_ex.restype = I32
    lib.gbm_gblup_fit_ex.argtypes = [P, I64, I64, I64, P, I64, I64, D, P, I32, I32, P, P, P, P, P]
    lib.gbm_gblup_fit_reml_ex.restype = I32
    lib.gbm_gblup_fit_reml_ex.argtypes = [P, I64, I64, I64, P, I64, I64, P, I32, I32, P, P, P, P, P, P, P, P]
    lib.gbm_gblup_fit_dosage_i8_ex.restype = I32
    lib.gbm_gblup_fit_dosage_i8_ex.argtypes = [P, I64, I64, I64, I32, P, I64, I64, D, P, I32, I32, P, P, P, P, P]
    lib.gbm_gblup_fit_synthetic_ex.restype = I32
    lib.gbm_gblup_fit_synthetic_ex.argtypes = [U64, I64, I64, P, I64, I64, D, P, I32, I32, P, P, P, P, P]
    lib.gbm_session_set_grm_mode.restype = I32
    lib.gbm_session_set_grm_mode.argtypes = [P, I32]
    lib.gbm_session_grm_used.restype = I32
    lib.gbm_session_grm_used.argtypes = [P, P]
    lib.gbm_debug_rccl_calls.restype = I32
    lib.gbm_debug_rccl_calls.argtypes = [P, P]
    lib.gbm_debug_xg_choose.restype = I32
    lib.gbm_debug_xg_choose.argtypes = [D, D, P, P]
    lib.gbm_debug_chol_flow_order.restype = I64
    lib.gbm_debug_chol_flow_order.argtypes = [I32, P, I64]
    lib.gbm_debug_chol_flow_order_size.restype = I64
    lib.gbm_debug_chol_flow_order_size.argtypes = [I32]
    lib.gbm_debug_chol_flow_order_check.restype = I64
    lib.gbm_debug_chol_flow_order_check.argtypes = [I32, P, I64]
    lib.gbm_dev_grm_exact_status.restype = I32
    lib.gbm_dev_grm_exact_status.argtypes = [P, I64, I64, P]
    lib.gbm_debug_set.restype = I32
    lib.gbm_debug_set.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    return lib


def _bind_runtime_first():
    """One HIP runtime per process. PyTorch-ROCm bundles its own libamdhip64 (soname
    libamdhip64.so.7) and librccl (librccl.so.1); if torch is importable we load it first so
    that libgbm's NEEDED entries resolve to the already-loaded copies instead of mapping a
    second HIP/HSA runtime from /opt/rocm (two runtimes in one process cannot both own the GPU).
    Set GBM_NO_TORCH=1 to skip this in torch-free processes."""
    if os.environ.get("GBM_NO_TORCH") == "1":
        return
    try:
        import torch  # noqa: F401
    except ImportError:
        return


def load():
    """Load libgbm.so (once). Raises ImportError if the HIP library has not been built."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise ImportError(
                    f"libgbm.so not found at {LIB_PATH}: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
                    " (the GBLUP path has no CPU fallback)")
            _bind_runtime_first()
            _lib = _declare(ctypes.CDLL(LIB_PATH))
            v = _lib.gbm_version()
            if v != ABI_VERSION:
                raise ImportError(f"libgbm.so ABI version {v} != {ABI_VERSION}")
        return _lib


def debug_set(name: str, value=None):
    """Set (or with None clear) a GBM_* knob in libgbm and in os.environ alike. libgbm reads the environment
    once, at its first knob lookup, so a knob changed after the library has run goes through here (tests,
    timing tools); the os.environ copy serves the Python-level knobs (gbm.sharded) and child processes."""
    if value is None:
        os.environ.pop(name, None)
    else:
        os.environ[name] = str(value)
    check(load().gbm_debug_set(name.encode(), None if value is None else str(value).encode()), "gbm_debug_set")


def last_error() -> str:
    return load().gbm_last_error().decode("utf-8", "replace")


def check(rc: int, what: str):
    if rc == GBM_OK:
        return
    msg = f"{what}: {last_error()} (code {rc})"
    if rc == GBM_E_ARG:
        raise ArgumentError(msg)
    raise GBMError(msg)


def device_count() -> int:
    c = I32(0)
    check(load().gbm_device_count(ctypes.byref(c)), "gbm_device_count")
    return c.value


def ptr(a: np.ndarray):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


def devices_arg(devices):
    if devices is None:
        return None, 0
    arr = (ctypes.c_int * len(devices))(*devices)
    return arr, len(devices)

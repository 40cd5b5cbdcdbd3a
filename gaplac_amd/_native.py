"""ctypes binding of libgaplac_hip.so (the C-ABI in include/gaplac.h).

The product path has no fallback: if the HIP library is missing or fails to load this
module raises, and every logpdf call fails loudly.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_double, c_int, c_int32, c_int64, c_void_p

LIB_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib")
LIB_PATH = os.path.join(LIB_DIR, "libgaplac_hip.so")

SQEXP, OU, LINEAR, CAT, NOISE = 1, 2, 3, 4, 5
KIND_NAMES = {SQEXP: "SQEXP", OU: "OU", LINEAR: "LINEAR", CAT: "CAT", NOISE: "NOISE"}
MAX_TERMS = 16

E_ARG, E_KIND, E_PARAM, E_COL, E_NODEVICE, E_HIP, E_OOM, E_COMM = -1, -2, -3, -4, -5, -6, -7, -8

# Every symbol include/gaplac.h declares (checked by tests/test_abi.py).
EXPORTED = (
    "gaplac_abi_version",
    "gaplac_last_error",
    "gaplac_ctx_create",
    "gaplac_ctx_destroy",
    "gaplac_ctx_release",
    "gaplac_logpdf",
    "gaplac_logpdf_device",
    "gaplac_logpdf_batch",
    "gaplac_logpdf_grad",
    "gaplac_logpdf_grad_device",
    "gaplac_posterior_mean_var",
    "gaplac_rand",
    "gaplac_gram",
    "gaplac_gram_time",
    "gaplac_factor",
    "gaplac_set_profiling",
    "gaplac_get_stats",
    "gaplac_reset_stats",
    "gaplac_plan_check",
    "gaplac_plan_check_schedule",
    "gaplac_dist_create",
    "gaplac_dist_destroy",
    "gaplac_dist_last_error",
    "gaplac_dist_geometry",
    "gaplac_dist_set_panel_buffers",
    "gaplac_dist_begin",
    "gaplac_dist_factor",
    "gaplac_dist_panel",
    "gaplac_dist_comm_begin",
    "gaplac_dist_comm_end",
    "gaplac_dist_update",
    "gaplac_dist_finish",
    "gaplac_dist_local",
    "gaplac_dist_configure",
    "gaplac_dist_chunks",
    "gaplac_dist_panel_chunk",
    "gaplac_dist_comm_begin_chunk",
    "gaplac_dist_comm_end_chunk",
    "gaplac_dist_plan_check",
    "gaplac_dist_plan",
    "gaplac_dist_set_tail",
    "gaplac_dist_set_layout",
    "gaplac_dist_owner",
    "gaplac_dist_tail_geometry",
    "gaplac_dist_set_tail_buffer",
    "gaplac_dist_tail_segment",
    "gaplac_dist_tail_begin",
    "gaplac_dist_tail_end",
    "gaplac_dist_plan_check_tail",
    "gaplac_dist_plan_tail",
    "gaplac_dist_replay_enable",
    "gaplac_dist_replay_chunk",
    "gaplac_dist_replay_stamps",
    "gaplac_dist_replay_tail",
    "gaplac_dist_replay_info",
)


class Term(ctypes.Structure):
    _fields_ = [
        ("kind", c_int32),
        ("col", c_int32),
        ("param", c_double),
        ("group", c_int32),
        ("reserved", c_int32),
    ]


class Stats(ctypes.Structure):
    _fields_ = [
        ("evals", c_int64),
        ("syrk_launches", c_int64),
        ("syrk_ms", c_double),
        ("syrk_flops", c_double),
        ("gram_ms", c_double),
        ("gram_bytes", c_double),
        ("gram_launches", c_int64),
        ("panel_ms", c_double),
        ("trsm_ms", c_double),
        ("colupd_ms", c_double),
        ("total_ms", c_double),
        ("syrk_bytes", c_double),
        ("small_launches", c_int64),
        ("small_ms", c_double),
        ("grad_rows_ms", c_double),
        ("cinv_launches", c_int64),
        ("cinv_ms", c_double),
        ("contract_ms", c_double),
        ("tail_launches", c_int64),
        ("tail_ms", c_double),
        ("bulk_flops", c_double),
        ("bulk_launches", c_int64),
        ("bulk_union_ms", c_double),
    ]


_lib = None

_DP = POINTER(c_double)


def load() -> ctypes.CDLL:
    """Load the HIP library once; raise if it is absent (no CPU fallback exists)."""
    global _lib
    if _lib is not None:
        return _lib
    path = os.environ.get("GAPLAC_LIB_PATH", LIB_PATH)  # developer A/B builds
    if not os.path.exists(path):
        raise RuntimeError(
            f"libgaplac_hip.so not built ({path}); run `python -c 'import __graft_entry__ as g; g.build()'`"
        )
    lib = ctypes.CDLL(path)
    lib.gaplac_abi_version.restype = c_int
    lib.gaplac_last_error.restype = c_char_p
    lib.gaplac_last_error.argtypes = [c_void_p]
    lib.gaplac_ctx_create.argtypes = [c_int, POINTER(c_void_p)]
    lib.gaplac_ctx_destroy.argtypes = [c_void_p]
    lib.gaplac_ctx_release.argtypes = [c_void_p]
    common = [c_void_p, c_int64, c_int32, c_void_p, c_int64, c_int32, POINTER(Term), c_double, c_void_p]
    lib.gaplac_logpdf.argtypes = common + [_DP, _DP, _DP]
    lib.gaplac_logpdf_device.argtypes = common + [_DP, _DP, _DP]
    lib.gaplac_logpdf_batch.argtypes = [
        c_void_p, c_int32, c_int64, c_int32, c_void_p, c_int64, POINTER(c_int32), POINTER(Term),
        c_double, c_void_p, _DP, POINTER(c_int64),
    ]
    lib.gaplac_logpdf_grad.argtypes = common + [_DP, c_void_p, c_void_p, _DP]
    lib.gaplac_logpdf_grad_device.argtypes = common + [_DP, c_void_p, c_void_p, _DP]
    lib.gaplac_posterior_mean_var.argtypes = common + [c_int64, c_void_p, c_int64, c_void_p, c_void_p]
    lib.gaplac_rand.argtypes = common + [c_void_p]
    lib.gaplac_gram.argtypes = [
        c_void_p, c_int64, c_int32, c_void_p, c_int64, c_int32, POINTER(Term), c_double, c_void_p, c_int64,
    ]
    lib.gaplac_gram_time.argtypes = [
        c_void_p, c_int64, c_int32, c_void_p, c_int64, c_int32, POINTER(Term), c_double, c_void_p, c_int32,
        _DP, _DP,
    ]
    lib.gaplac_factor.argtypes = common + [c_void_p, c_int64, c_void_p]
    lib.gaplac_set_profiling.argtypes = [c_void_p, c_int]
    lib.gaplac_get_stats.argtypes = [c_void_p, POINTER(Stats)]
    lib.gaplac_reset_stats.argtypes = [c_void_p]
    _I32P, _I64P, _VPP = POINTER(c_int32), POINTER(c_int64), POINTER(c_void_p)
    lib.gaplac_plan_check.argtypes = [c_int64, c_int32, c_int64, c_int32, _I64P, _I64P, c_char_p, c_int64]
    lib.gaplac_plan_check_schedule.argtypes = [c_int64, c_int32, c_int32, c_int32, c_int32, _I64P, c_char_p, c_int64]
    lib.gaplac_dist_create.argtypes = [c_int, c_int, c_int, c_int, _VPP]
    lib.gaplac_dist_destroy.argtypes = [c_void_p]
    lib.gaplac_dist_last_error.argtypes = [c_void_p]
    lib.gaplac_dist_geometry.argtypes = [c_void_p, c_int64, _I64P, _I32P, _I32P, _I32P, _I64P]
    lib.gaplac_dist_set_panel_buffers.argtypes = [c_void_p, c_void_p, c_void_p, c_int64]
    lib.gaplac_dist_begin.argtypes = common + [c_int, _I32P]
    lib.gaplac_dist_factor.argtypes = [c_void_p, c_int32]
    lib.gaplac_dist_panel.argtypes = [c_void_p, c_int32, _VPP, _I64P, _I32P]
    lib.gaplac_dist_comm_begin.argtypes = [c_void_p, c_int32, _VPP]
    lib.gaplac_dist_comm_end.argtypes = [c_void_p, c_int32]
    lib.gaplac_dist_update.argtypes = [c_void_p, c_int32]
    lib.gaplac_dist_finish.argtypes = [c_void_p, _DP, _DP, _I64P]
    lib.gaplac_dist_local.argtypes = [c_void_p, c_void_p, c_int64]
    lib.gaplac_dist_configure.argtypes = [c_void_p, c_int32, c_int32, c_int32, c_int32, c_int32]
    lib.gaplac_dist_chunks.argtypes = [c_void_p, c_int32, _I32P]
    lib.gaplac_dist_panel_chunk.argtypes = [c_void_p, c_int32, c_int32, _VPP, _I64P, _I32P]
    lib.gaplac_dist_comm_begin_chunk.argtypes = [c_void_p, c_int32, c_int32, _VPP]
    lib.gaplac_dist_comm_end_chunk.argtypes = [c_void_p, c_int32, c_int32]
    lib.gaplac_dist_plan_check.argtypes = [c_int32, c_int32, c_int32, c_int32, _I64P, c_char_p, c_int64]
    lib.gaplac_dist_plan.argtypes = [c_int32, c_int32, c_int32, c_int32, _I32P, c_int64, _I64P]
    lib.gaplac_dist_set_tail.argtypes = [c_void_p, c_int32, c_int32]
    lib.gaplac_dist_set_layout.argtypes = [c_void_p, c_int32]
    lib.gaplac_dist_owner.argtypes = [c_void_p, c_int32, _I32P]
    lib.gaplac_dist_tail_geometry.argtypes = [c_void_p, c_int64, _I32P, _I64P, _I32P]
    lib.gaplac_dist_set_tail_buffer.argtypes = [c_void_p, c_void_p, c_int64]
    lib.gaplac_dist_tail_segment.argtypes = [c_void_p, c_int32, _VPP, _I64P, _I32P]
    lib.gaplac_dist_tail_begin.argtypes = [c_void_p, _VPP]
    lib.gaplac_dist_tail_end.argtypes = [c_void_p]
    lib.gaplac_dist_plan_check_tail.argtypes = [c_int32, c_int32, c_int32, c_int32, c_int32, _I64P, c_char_p, c_int64]
    lib.gaplac_dist_plan_tail.argtypes = [c_int32, c_int32, c_int32, c_int32, c_int32, _I32P, c_int64, _I64P]
    lib.gaplac_dist_replay_enable.argtypes = [c_void_p, c_int64]
    lib.gaplac_dist_replay_chunk.argtypes = [c_void_p, c_void_p, c_int32, c_int32, c_int64, c_int64, c_int64,
                                             c_int64, c_int64]
    lib.gaplac_dist_replay_stamps.argtypes = [c_void_p, c_void_p, c_int64]
    lib.gaplac_dist_replay_tail.argtypes = [c_void_p, c_void_p, c_int32, c_int64, c_double, c_int64, c_int64]
    lib.gaplac_dist_replay_info.argtypes = [c_void_p, c_int32, c_int32, _I64P, _I32P, _I32P]
    for name in EXPORTED:
        getattr(lib, name).restype = getattr(lib, name).restype or c_int
    lib.gaplac_last_error.restype = c_char_p
    lib.gaplac_dist_last_error.restype = c_char_p
    _lib = lib
    return lib


def term_array(terms) -> "ctypes.Array[Term]":
    """terms: iterable of (kind, col, param, group)."""
    terms = list(terms)
    arr = (Term * max(1, len(terms)))()
    for i, (kind, col, param, group) in enumerate(terms):
        arr[i] = Term(int(kind), int(col), float(param), int(group), 0)
    return arr

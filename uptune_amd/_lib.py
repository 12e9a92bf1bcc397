"""ctypes binding of libuthot.so (include/uthot.h).

The product path has no CPU fallback: if the shared library is missing or
cannot be loaded, importing this module's `lib()` raises.  Structures mirror
the C header field for field.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("UTHOT_LIB", os.path.join(_HERE, "libuthot.so"))

UT_FLOAT, UT_INT, UT_LOGINT, UT_POW2, UT_BOOL, UT_ENUM, UT_PERM = range(7)
UT_ACQ_EI, UT_ACQ_UCB = 0, 1
UT_RED_SUM, UT_RED_MAX, UT_RED_MIN = 0, 1, 2
UT_COMM_ID_BYTES = 128
# permutation crossover operators (op3_cross_*, manipulator.py:1179-1353)
UT_X_NONE, UT_X_OX1, UT_X_OX3, UT_X_PX, UT_X_CX, UT_X_PMX = range(6)
CROSSOVERS = {"op3_cross_OX1": UT_X_OX1, "op3_cross_OX3": UT_X_OX3, "op3_cross_PX": UT_X_PX,
              "op3_cross_CX": UT_X_CX, "op3_cross_PMX": UT_X_PMX}

ERRORS = {
    -1: "UT_EINVAL", -2: "UT_EHIP", -3: "UT_ENOSPACE", -4: "UT_EUNSUPPORTED", -5: "UT_ENOTPD", -6: "UT_ENOMEM", -7: "UT_ECOMM",
}


class ParamDesc(C.Structure):
    _fields_ = [
        ("kind", C.c_int32), ("sort_rank", C.c_int32),
        ("lo", C.c_double), ("hi", C.c_double),
        ("u_lo", C.c_double), ("u_hi", C.c_double), ("u_span", C.c_double),
        ("n_options", C.c_int64),
        ("name", C.c_char_p), ("name_len", C.c_int32),
        ("lut_count", C.c_int32), ("lut_host", C.c_void_p),
        ("vtab_count", C.c_int32), ("pad", C.c_int32), ("vtab_host", C.c_void_p),
        ("perm_repr_host", C.c_void_p), ("perm_repr_off_host", C.c_void_p),
    ]


class TreeNode(C.Structure):
    _fields_ = [("feature", C.c_int32), ("left", C.c_int32), ("right", C.c_int32), ("default_left", C.c_int32),
                ("threshold", C.c_double), ("value", C.c_double)]


UT_SPLIT_LE, UT_SPLIT_LT = 0, 1


class DeParams(C.Structure):
    _fields_ = [("cr", C.c_double), ("n_cross", C.c_int32), ("information_sharing", C.c_int32),
                ("best", C.c_void_p)]


class PruneStats(C.Structure):
    _fields_ = [("survivors", C.c_int64), ("bound_rows", C.c_int32), ("dense", C.c_int32), ("threshold", C.c_double)]


class PsoParams(C.Structure):
    _fields_ = [("omega", C.c_double), ("phi_l", C.c_double), ("phi_g", C.c_double), ("sigma", C.c_double),
                ("alias_pbest", C.c_int32), ("enum_mode", C.c_int32), ("crossover", C.c_int32),
                ("pad", C.c_int32)]


class GaParams(C.Structure):
    _fields_ = [("mutation_rate", C.c_double), ("sigma", C.c_double), ("crossover_rate", C.c_double),
                ("crossover_strength", C.c_double), ("must_mutate_count", C.c_int32), ("normal", C.c_int32),
                ("max_retries", C.c_int32), ("op", C.c_int32), ("crossover", C.c_int32), ("pad", C.c_int32)]


class GpHyper(C.Structure):
    _fields_ = [("sigma_f2", C.c_double), ("sigma_n2", C.c_double), ("jitter", C.c_double),
                ("lengthscale_host", C.c_void_p)]


class Acq(C.Structure):
    _fields_ = [("kind", C.c_int32), ("pad", C.c_int32), ("xi", C.c_double), ("kappa", C.c_double)]


class RoundOut(C.Structure):
    _fields_ = [("topk_idx", C.c_void_p), ("topk_score", C.c_void_p), ("topk_digest", C.c_void_p),
                ("topk_values", C.c_void_p)]


P = C.c_void_p
I32, I64, U32, U64, D = C.c_int32, C.c_int64, C.c_uint32, C.c_uint64, C.c_double

# name -> (restype, argtypes); every symbol declared in include/uthot.h
SIGNATURES = {
    "ut_version": (C.c_int, []),
    "ut_device_bytes": (C.c_int, [I32, C.POINTER(I64)]),
    "ut_ctx_create": (C.c_int, [C.c_int, U64, C.POINTER(P)]),
    "ut_ctx_destroy": (C.c_int, [P]),
    "ut_last_error": (C.c_char_p, [P]),
    "ut_set_stream": (C.c_int, [P, P]),
    "ut_sync": (C.c_int, [P]),
    "ut_space_define": (C.c_int, [P, I32, C.POINTER(ParamDesc), I32]),
    "ut_space_info": (C.c_int, [P, C.POINTER(I64), C.POINTER(I64), C.POINTER(I32)]),
    "ut_space_columns": (C.c_int, [P, C.POINTER(I32)]),
    "ut_population_init": (C.c_int, [P, I64, U32]),
    "ut_population_set": (C.c_int, [P, I64, P, I64]),
    "ut_population_get": (C.c_int, [P, P, I64]),
    "ut_population_replace": (C.c_int, [P, P, I64, P, I64]),
    "ut_population_select": (C.c_int, [P, I32]),
    "ut_score_round_de_pruned": (C.c_int, [P, C.POINTER(DeParams), C.POINTER(Acq), U32, I64, I64, I32, I32,
                                           C.POINTER(RoundOut), C.POINTER(PruneStats)]),
    "ut_gp_topk_pruned": (C.c_int, [P, P, I64, I64, C.POINTER(Acq), P, I64, I32, I32, P, P, C.POINTER(PruneStats)]),
    "ut_hash_de": (C.c_int, [P, P, I64, I64, I64, P]),
    "ut_hash_parent": (C.c_int, [P, P, I64, I64, P, P]),
    "ut_propose_de": (C.c_int, [P, C.POINTER(DeParams), U32, I64, I64, P, I64]),
    "ut_pso_reset": (C.c_int, [P]),
    "ut_propose_pso": (C.c_int, [P, C.POINTER(PsoParams), P, U32, I64, I64, P, P, I64]),
    "ut_pso_commit": (C.c_int, [P, P, P, I64, I64, I64]),
    "ut_pso_update_best": (C.c_int, [P, P, I64, P, I64]),
    "ut_propose_ga": (C.c_int, [P, C.POINTER(GaParams), P, P, U32, I64, I64, P, I64, P]),
    "ut_encode_features": (C.c_int, [P, P, I64, I64, P, I64]),
    "ut_hash": (C.c_int, [P, P, I64, I64, P]),
    "ut_history_reset": (C.c_int, [P, I64]),
    "ut_history_add": (C.c_int, [P, P, I64]),
    "ut_history_add_host": (C.c_int, [P, P, I64]),
    "ut_dedup": (C.c_int, [P, P, I64, P]),
    "ut_gp_fit": (C.c_int, [P, P, P, I32, I32, C.POINTER(GpHyper)]),
    "ut_gp_fit_async": (C.c_int, [P, P, P, I32, I32, C.POINTER(GpHyper)]),
    "ut_gp_set_fit_append": (C.c_int, [P, I32]),
    "ut_gp_last_fit_kind": (C.c_int, [P, C.POINTER(I32)]),
    "ut_forest_set": (C.c_int, [P, I32, P, I64, P, I32, D, D, D]),
    "ut_forest_predict": (C.c_int, [P, P, I64, I64, I32, P, D, P, P]),
    "ut_gp_score": (C.c_int, [P, P, I64, I64, C.POINTER(Acq), P, P, P, P]),
    "ut_gp_score_values": (C.c_int, [P, P, I64, I64, C.POINTER(Acq), P, P, P, P]),
    "ut_gp_set_precision": (C.c_int, [P, I32]),
    "ut_gp_set_i8_tol": (C.c_int, [P, C.c_double]),
    "ut_gp_set_prune_pass": (C.c_int, [P, C.c_int32]),
    "ut_gp_i8_stats": (C.c_int, [P, C.POINTER(C.c_int64), C.POINTER(C.c_double)]),
    "ut_gp_i8_bounds": (C.c_int, [P, P, P]),
    "ut_gp_fit_status": (C.c_int, [P, C.POINTER(I32)]),
    "ut_gp_join_fit": (C.c_int, [P]),
    "ut_gp_stats": (C.c_int, [P, C.POINTER(D), C.POINTER(D), C.POINTER(D)]),
    "ut_gp_kstar_mode": (C.c_int, [P, C.POINTER(I32)]),
    "ut_topk": (C.c_int, [P, P, P, I64, I64, I32, P, P]),
    "ut_score_round_ga": (C.c_int, [P, C.POINTER(GaParams), C.c_void_p, C.c_void_p, C.POINTER(Acq), U32, I64, I64,
                                    I32, C.POINTER(RoundOut)]),
    "ut_score_round_de": (C.c_int, [P, C.POINTER(DeParams), C.POINTER(Acq), U32, I64, I64, I32,
                                    C.POINTER(RoundOut)]),
    "ut_round_buffers": (C.c_int, [P, C.POINTER(P), C.POINTER(P), C.POINTER(P), C.POINTER(P), C.POINTER(P),
                                   C.POINTER(P), C.POINTER(P), C.POINTER(I64)]),
    "ut_comm_unique_id": (C.c_int, [P]),
    "ut_comm_init": (C.c_int, [P, I32, I32, P]),
    "ut_comm_destroy": (C.c_int, [P]),
    "ut_comm_info": (C.c_int, [P, C.POINTER(I32), C.POINTER(I32)]),
    "ut_comm_allgather_topk": (C.c_int, [P, I32, P, P, P, P, I64, I32, P, P, P, P, I64]),
    "ut_topk_merge": (C.c_int, [P, I64, I32, P, P, P, P, I64, I32, P, P, P, P, I64]),
    "ut_comm_bcast_results": (C.c_int, [P, I32, I64, P, P, I64, C.POINTER(I64)]),
    "ut_comm_bcast": (C.c_int, [P, P, I64, I32]),
    "ut_comm_allreduce_f64": (C.c_int, [P, P, I64, I32]),
    "ut_comm_barrier": (C.c_int, [P]),
    "ut_debug_fail_alloc": (C.c_int, [P, I32]),
    "ut_set_timing": (C.c_int, [P, I32]),
    "ut_stage_time": (C.c_int, [P, C.c_char_p, C.POINTER(D)]),
}

_lock = threading.Lock()
_lib = None


class UthotError(RuntimeError):
    pass


def lib() -> C.CDLL:
    """Load libuthot.so once; raise (never fall back) when it is unavailable."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise UthotError(
                    f"{LIB_PATH} not found: build it with `python -m uptune_amd.build` "
                    "(the uptune_amd device path has no CPU fallback)")
            handle = C.CDLL(LIB_PATH)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(handle, name)
                fn.restype = res
                fn.argtypes = args
            _lib = handle
        return _lib


def check(ctx, rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().ut_last_error(ctx).decode(errors="replace") if ctx else ""
        raise UthotError(f"{what} failed: {ERRORS.get(rc, rc)}: {msg}")

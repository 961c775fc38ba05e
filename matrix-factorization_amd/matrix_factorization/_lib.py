"""ctypes binding of libmf_hip.so (the C ABI declared in include/mf_hip.h).

The shared library is built in-tree (``make -C matrix-factorization_amd/csrc``
or ``__graft_entry__.build()``).  There is no fallback: if the library is
missing or fails to load, every entry point raises ``MFLibraryError``.
"""

from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MF_HIP_LIB", os.path.join(_HERE, "libmf_hip.so"))

MF_F32, MF_F64 = 0, 1
MF_LINEAR, MF_SIGMOID, MF_RBF = 0, 1, 2
MF_FLAG_XCD_SWIZZLE = 1
MF_FLAG_NT_USER = 2
MF_FLAG_NT_ITEM = 4
MF_FLAG_XCD_CLAIM = 8
MF_FLAG_PERSISTENT = 16
MF_FLAG_DEEP_PIPE = 32
MF_FLAG_NO_COOP = 64
MF_FLAG_NARROW = 128
MF_FLAG_L2_HANDOFF = 256
MF_FLAG_NO_EARLY_POLL = 512
MF_FLAG_STREAM = 1024
MF_FLAG_PREPARE = 2048
MF_FLAG_CLASSES_SHIFT = 24       # bits 24..27: user-range classes - 1
MF_STRATA_MAX_CLASSES = 4
MF_ERR_CAPACITY = 3
MF_DELTA_TAKE, MF_DELTA_APPLY = 0, 1
KERNEL_CODES = {"linear": MF_LINEAR, "sigmoid": MF_SIGMOID, "rbf": MF_RBF}

_P = ctypes.c_void_p
_I32 = ctypes.c_int32
_I64 = ctypes.c_int64
_F64 = ctypes.c_double
_PD = ctypes.c_void_p          # double[2] timing output (nullable)

# name -> (restype, argtypes); mirrors include/mf_hip.h one to one
SIGNATURES = {
    "mf_last_error": (ctypes.c_char_p, []),
    "mf_abi_version": (ctypes.c_int, []),
    "mf_max_factors": (ctypes.c_int, []),
    "mf_sgd_epoch": (ctypes.c_int, [
        _P, _P, _P, _I64, _P, _P, _I32, _P, _I32,    # ids, ratings, n, order, offs, nb, seq, nseq
        _F64, _P, _P, _P, _P,                         # mu, bu, bi, P, Q
        _I32, _I32, _I32,                             # n_users, n_items, k
        _I32, _I32, _F64, _F64, _F64, _F64, _F64,     # kernel dtype gamma lr reg min max
        _I32, _I32, _I32, _P, ctypes.c_size_t,        # upd_u upd_i flags ws ws_bytes
        _P, _PD]),                                    # stream kernel_ms
    "mf_sgd_workspace_bytes": (ctypes.c_size_t, [_I32]),
    "mf_sgd_epoch_strata": (ctypes.c_int, [
        _P, _P, _P, _I64, _I32,                       # ids, ratings, n_positions, n_blocks
        _P, _P, _P, _I32, _I32, _I32,                 # plan: bounds, block steps, slots, max sizes
        _P, _I32, ctypes.c_uint32,                    # strata_seq, n_seq, seed
        _F64, _P, _P, _P, _P,                         # mu, bu, bi, P, Q
        _I32, _I32, _I32,                             # n_users, n_items, k
        _I32, _I32, _F64, _F64, _F64, _F64, _F64,     # kernel dtype gamma lr reg min max
        _I32, _I32, _I32,                             # upd_u upd_i flags
        _P, ctypes.c_size_t, _P, _PD]),               # ws ws_bytes stream kernel_ms
    "mf_sgd_epoch_strata_delta": (ctypes.c_int, [
        _P, _P, _P, _I64, _I32, _P, _P, _P, _I32, _I32, _I32, _P, _I32, ctypes.c_uint32,
        _F64, _P, _P, _P, _P, _I32, _I32, _I32, _I32, _I32, _F64, _F64, _F64, _F64, _F64,
        _I32, _I32, _I32, _P, ctypes.c_size_t,
        _P, _P, _P, _PD]),                            # item delta, bias delta, stream, ms
    "mf_strata_workspace_bytes": (ctypes.c_size_t, [_I32, _I32]),
    "mf_strata_status": (ctypes.c_int, [_P, _I32, _P]),
    "mf_strata_lds_bytes": (ctypes.c_size_t, [_I32, _I32, _I32, _I32]),
    "mf_strata_lds_limit": (ctypes.c_int32, []),
    "mf_strata_slots": (ctypes.c_int32, [_I32, _I32]),
    "mf_strata_slots_waves": (ctypes.c_int32, [_I32, _I32, _I32]),
    "mf_sse_workspace_bytes": (ctypes.c_size_t, [_I64]),
    "mf_sse": (ctypes.c_int, [
        _P, _P, _P, _I64, _F64, _P, _P, _P, _P, _I32, _I32, _I32, _I32, _I32, _F64,
        _F64, _F64, _P, _I32, _P, _P, _P]),
    "mf_sse_capped": (ctypes.c_int, [
        _P, _P, _P, _I64, _F64, _P, _P, _P, _P, _I32, _I32, _I32, _I32, _I32, _F64,
        _F64, _F64, _P, _I32, _P, _I32, _P, _P]),
    "mf_predict": (ctypes.c_int, [
        _P, _P, _I64, _F64, _P, _P, _P, _P, _I32, _I32, _I32, _F64, _F64,
        _F64, _I32, _P, _P]),
    "mf_topk_workspace_bytes": (ctypes.c_size_t, [_I32, _I32, _I32]),
    "mf_topk": (ctypes.c_int, [
        _P, _I32, _F64, _P, _P, _P, _P, _I32, _I32, _I32, _I32, _F64, _F64,
        _F64, _P, _P, _I32, _P, _P, _P, _P]),
    "mf_topk_mm_supported": (_I32, [_I32, _I32, _I32, _I32]),
    "mf_topk_mm_workspace_bytes": (ctypes.c_size_t, [_I32, _I32]),
    "mf_topk_mm": (ctypes.c_int, [
        _P, _I32, _F64, _P, _P, _P, _P, _I32, _I32, _I32, _I32, _P, _P, _I32, _P, _P,
        _P, _P, _P]),
    "mf_bias_sgd_epoch": (ctypes.c_int, [
        _P, _P, _P, _I64, _P, _P, _I32, _P, _I32, _F64, _P, _P, _I32, _F64, _F64,
        _I32, _I32, _P]),
    "mf_bias_sse": (ctypes.c_int, [
        _P, _P, _P, _I64, _F64, _P, _P, _I32, _P, _P, _P]),
    "mf_bias_als_epoch": (ctypes.c_int, [
        _P, _P, _P, _F64, _P, _P, _I32, _I32, _P, _P, _P, _P, _I32, _F64, _P]),
    "mf_bias_predict": (ctypes.c_int, [
        _P, _P, _I64, _F64, _P, _P, _I32, _F64, _F64, _I32, _P, _P]),
    "mf_als_sweep": (ctypes.c_int, [
        _P, _P, _P, _I32, _F64, _P, _P, _P, _P, _I32, _I32, _F64, _P]),
    "mf_als_max_factors": (ctypes.c_int32, []),
    "mf_als_sweep_probe": (ctypes.c_int, [
        _P, _P, _P, _I32, _F64, _P, _P, _P, _P, _I32, _I32, _F64, _P, _P]),
    "mf_replica_delta": (ctypes.c_int, [_P, _P, _I64, _I32, _I32, _P]),
    "mf_replica_apply": (ctypes.c_int, [_P, _P, _I64, _I32, _F64, _P]),
    "mf_warmup": (ctypes.c_int, [ctypes.c_int32, _P]),
    "mf_permute_rows": (ctypes.c_int, [_I32, _P, _P, _P, _P, _P, _I32, _P]),
    "mf_sched_levels": (ctypes.c_int, [
        _P, _P, _I64, _P, _I32, _I32, _I32, _I32, _P, _P, _I64, _P]),
    "mf_sched_levels_chunked": (ctypes.c_int, [
        _P, _P, _I64, _P, _I32, _I32, _I32, _I32, _I32, _P, _P, _I64, _P]),
    "mf_sched_color": (ctypes.c_int, [
        _P, _P, _I64, _I32, _I32, _P, _P, _I64, _P]),
    "mf_sched_slices": (ctypes.c_int, [_P, _P, _I64, _I32, _I32, _I32, _P, _P]),
    "mf_sched_tiles": (ctypes.c_int, [_P, _P, _I64, _I32, _I32, _I32, _I32, _P, _P]),
    "mf_strata_plan_build": (ctypes.c_int, [
        _P, _P, _I64, _I32, _I32, _I32, _P, _P, _I32, _P]),
    "mf_strata_plan_build_classes": (ctypes.c_int, [
        _P, _P, _I64, _I32, _I32, _I32, _I32, _P, _P, _I32, _P]),
    "mf_strata_plan_build_pick": (ctypes.c_int, [
        _P, _P, _I64, _I32, _I32, _I32, _I32, _P, _P, _P, _P, _I32, ctypes.c_double, _P, _P]),
    "mf_strata_plan_positions": (_I64, [_P]),
    "mf_strata_plan_fetch": (ctypes.c_int, [_P, _P, _P]),
    "mf_strata_plan_free": (None, [_P]),
    "mf_strata_set_probe": (ctypes.c_int, [_P]),
    "mf_strata_inject_fail": (ctypes.c_int, [_I32]),
    "mf_legacy_shuffle": (ctypes.c_int, [_P, _P, _P, _I64]),
    "mf_legacy_shuffle_i32": (ctypes.c_int, [_P, _P, _P, _I64]),
    "mf_legacy_permutation": (ctypes.c_int, [_P, _P, _P, _I64]),
    "mf_legacy_shuffle_draws": (ctypes.c_int, [_P, _P, _I64, _P]),
    "mf_legacy_apply_swaps_i32": (ctypes.c_int, [_P, _I64, _I64, _P]),
    "mf_shuffle_swaps_workspace_bytes": (ctypes.c_size_t, [_I64]),
    "mf_shuffle_swaps_device": (ctypes.c_int, [_P, _I64, _I64, _P, _P, _P, _P, _P]),
    "mf_pairs_duplicated": (ctypes.c_int, [_P, _P, _I64, _P]),
    "mf_factorize": (ctypes.c_int, [_P, _I64, _P, _P, _P]),
    "mf_id_range": (ctypes.c_int, [_P, _I64, _P, _P]),
    "mf_first_appearance": (ctypes.c_int, [_P, _I64, _I64, _P, _I64, _P, _P, _P]),
    "mf_gather": (ctypes.c_int, [_P, _I64, _I32, _P, _I64, _P]),
    "mf_gather_i32": (ctypes.c_int, [_P, _I64, _I32, _P, _I64, _P]),
    "mf_ids_to_i32": (ctypes.c_int, [_P, _I64, _I64, _P]),
    "mf_f64_to_f32": (ctypes.c_int, [_P, _I64, _P]),
    "mf_fingerprint": (ctypes.c_uint64, [_P, _I64]),
}


class MFLibraryError(RuntimeError):
    """libmf_hip.so is missing, failed to load, or returned an error."""


_lock = threading.Lock()
_lib = None


def load() -> ctypes.CDLL:
    """Load libmf_hip.so once; raise MFLibraryError if it is unavailable."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise MFLibraryError(
                    f"{LIB_PATH} not found: build it with "
                    "`make -C matrix-factorization_amd/csrc` (hipcc, gfx950)")
            try:
                lib = ctypes.CDLL(LIB_PATH)
            except OSError as e:  # pragma: no cover - environment specific
                raise MFLibraryError(f"cannot load {LIB_PATH}: {e}") from e
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = args
            _lib = lib
    return _lib


def last_error() -> str:
    msg = load().mf_last_error()
    return msg.decode() if msg else ""


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise MFLibraryError(f"{what} failed (code {rc}): {last_error()}")


def call(name: str, *args) -> int:
    """Call an entry point and raise on a non-zero status."""
    rc = getattr(load(), name)(*args)
    check(rc, name)
    return rc

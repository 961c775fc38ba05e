"""Host helpers of fit()'s preprocessing at 10^8 rows (mf_prep.cpp).

``RecommenderBase._preprocess_data`` (recommender_base.py:120-141 of the
reference) and the per-epoch row shuffle of ``_sgd``
(kernel_matrix_factorization.py:371) cost seconds to a minute at C3 scale in
pandas / NumPy, against ~12 ms per GPU epoch.  Each helper here returns what
the pandas / NumPy call it replaces returns, and draws from NumPy's global
legacy RandomState exactly as that call does (tests/test_prep.py compares
them on the same seeds).
"""

from __future__ import annotations

import ctypes

import numpy as np

from . import _lib

_MAX_N = (1 << 32) + 1       # NumPy's 32-bit random_interval branch


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def legacy_shuffle_(a: np.ndarray) -> None:
    """``np.random.shuffle(a)`` for a 1-D contiguous 8- or 4-byte array, in
    place, advancing the global RandomState exactly as NumPy does (the swap
    targets depend on len(a) only, so the element size changes nothing but
    the bytes moved)."""
    if a.ndim != 1 or a.dtype.itemsize not in (4, 8) or not a.flags.c_contiguous \
            or not a.flags.writeable or len(a) > _MAX_N or a.dtype.hasobject:
        np.random.shuffle(a)
        return
    st = np.random.get_state()
    if st[0] != "MT19937":                       # pragma: no cover - legacy is MT19937
        np.random.shuffle(a)
        return
    key = np.ascontiguousarray(st[1], dtype=np.uint32).copy()
    pos = ctypes.c_int32(int(st[2]))
    if a.dtype.itemsize == 8:
        _lib.call("mf_legacy_shuffle", _ptr(key), ctypes.addressof(pos),
                  _ptr(a.view(np.int64)), len(a))
    else:
        _lib.call("mf_legacy_shuffle_i32", _ptr(key), ctypes.addressof(pos),
                  _ptr(a.view(np.int32)), len(a))
    np.random.set_state(("MT19937", key, pos.value, st[3], st[4]))


def legacy_permutation(n: int) -> np.ndarray:
    """``np.random.permutation(n)`` (int64), same draws."""
    st = np.random.get_state()
    if n > _MAX_N or st[0] != "MT19937":        # pragma: no cover - NumPy's own path
        return np.random.permutation(n).astype(np.int64)
    perm = np.empty(n, np.int64)
    key = np.ascontiguousarray(st[1], dtype=np.uint32).copy()
    pos = ctypes.c_int32(int(st[2]))
    _lib.call("mf_legacy_permutation", _ptr(key), ctypes.addressof(pos), _ptr(perm), n)
    np.random.set_state(("MT19937", key, pos.value, st[3], st[4]))
    return perm


def legacy_shuffle_draws(n: int, targets: np.ndarray) -> None:
    """The draws of ``np.random.shuffle`` of n elements, without the swaps:
    ``targets[d]`` (uint32 bits, d = 0 .. n-2) = the position swapped with
    n-1-d; the global RandomState is advanced exactly as by the shuffle."""
    st = np.random.get_state()
    if st[0] != "MT19937" or n > _MAX_N:         # pragma: no cover - legacy is MT19937
        raise ValueError("legacy_shuffle_draws: MT19937 and n <= 2^32 + 1 only")
    if n > 1 and (targets.dtype.itemsize != 4 or not targets.flags.c_contiguous
                  or len(targets) < n - 1):
        raise ValueError("targets must be a contiguous 4-byte array of n - 1 entries")
    key = np.ascontiguousarray(st[1], dtype=np.uint32).copy()
    pos = ctypes.c_int32(int(st[2]))
    _lib.call("mf_legacy_shuffle_draws", _ptr(key), ctypes.addressof(pos), n,
              _ptr(targets) if n > 1 else None)
    np.random.set_state(("MT19937", key, pos.value, st[3], st[4]))


def apply_swaps_i32(targets: np.ndarray, n: int, d_begin: int, data: np.ndarray) -> None:
    """Swaps d_begin .. n-2 of a shuffle drawn by legacy_shuffle_draws,
    applied in order to the int32 array ``data`` -- the first n - d_begin
    elements of the shuffled array, all those swaps touch."""
    if data.dtype != np.int32 or not data.flags.c_contiguous or len(data) < n - d_begin:
        raise ValueError("data must be a contiguous int32 array of n - d_begin entries")
    _lib.call("mf_legacy_apply_swaps_i32", _ptr(targets) if n > 1 else None, n, d_begin,
              _ptr(data))


def as_int64_ids(col: np.ndarray):
    """The id column as int64 (a view or a widening copy) when its values can
    be hashed as 64-bit integers with equality preserved, else None."""
    col = np.asarray(col)
    if col.ndim != 1 or col.dtype.kind not in "iu":
        return None
    if col.dtype.itemsize == 8:
        return np.ascontiguousarray(col).view(np.int64)
    return col.astype(np.int64)


def pairs_duplicated(a: np.ndarray, b: np.ndarray) -> bool:
    """``DataFrame({a, b}).duplicated().sum() != 0`` for int64 id columns."""
    a = np.ascontiguousarray(a, dtype=np.int64)
    b = np.ascontiguousarray(b, dtype=np.int64)
    if len(a) != len(b):
        raise ValueError("id columns differ in length")
    flag = ctypes.c_int32(0)
    _lib.call("mf_pairs_duplicated", _ptr(a), _ptr(b), len(a), ctypes.addressof(flag))
    return bool(flag.value)


def factorize(vals: np.ndarray):
    """``pd.factorize(vals, sort=False)`` for an int64 column: (codes int64,
    uniques int64 in first-appearance order)."""
    vals = np.ascontiguousarray(vals, dtype=np.int64)
    codes = np.empty(len(vals), np.int64)
    uniques = np.empty(len(vals), np.int64)
    nu = ctypes.c_int64(0)
    _lib.call("mf_factorize", _ptr(vals), len(vals), _ptr(codes), _ptr(uniques),
              ctypes.addressof(nu))
    return codes, uniques[: nu.value].copy()


# ids spanning at most n + this many values are their own dense ids
DIRECT_SPAN_SLACK = 1 << 20


def dense_ids(vals: np.ndarray):
    """Dense ids of an UNSHUFFLED int64 column for ``factorize_shuffled``:
    (dense, base, n_dense, uniques) -- the column itself and its minimum when
    its values span at most len + DIRECT_SPAN_SLACK integers, else
    ``factorize``'s codes and uniques.  Needs no permutation, so fit() runs it
    while the permutation is drawn."""
    vals = np.ascontiguousarray(vals, dtype=np.int64)
    if len(vals) == 0:
        return vals, 0, 0, np.empty(0, np.int64)
    lo, hi = ctypes.c_int64(0), ctypes.c_int64(0)
    _lib.call("mf_id_range", _ptr(vals), len(vals), ctypes.addressof(lo), ctypes.addressof(hi))
    span = int(hi.value) - int(lo.value) + 1
    if span <= min(len(vals) + DIRECT_SPAN_SLACK, (1 << 32) - 1):
        return vals, int(lo.value), span, None
    codes, uniq = factorize(vals)
    return codes, 0, len(uniq), uniq


def factorize_shuffled(dense, perm: np.ndarray):
    """``pd.factorize(vals[perm], sort=False)`` from ``dense_ids(vals)``:
    (codes int64, uniques int64 in first-appearance order of the shuffled
    column)."""
    d, base, nd, uniq = dense
    perm = np.ascontiguousarray(perm, dtype=np.int64)
    if len(perm) != len(d):
        raise ValueError("permutation and column differ in length")
    codes = np.empty(len(perm), np.int64)
    order = np.empty(max(nd, 1), np.int64)
    nu = ctypes.c_int64(0)
    if len(perm):
        _lib.call("mf_first_appearance", _ptr(d), base, nd, _ptr(perm), len(perm),
                  _ptr(codes), _ptr(order), ctypes.addressof(nu))
    order = order[: nu.value]
    return codes, (order + base if uniq is None else uniq[order])


def gather(src: np.ndarray, idx: np.ndarray) -> np.ndarray:
    """``src[idx]`` for a 1-D array of 4- or 8-byte elements (threaded);
    int32 indices are used as they are (mf_gather_i32), others as int64."""
    src = np.ascontiguousarray(src)
    i32 = isinstance(idx, np.ndarray) and idx.dtype == np.int32
    idx = np.ascontiguousarray(idx, dtype=np.int32 if i32 else np.int64)
    if src.ndim != 1 or src.dtype.itemsize not in (4, 8) or src.dtype.hasobject:
        return src[idx]
    dst = np.empty(len(idx), src.dtype)
    _lib.call("mf_gather_i32" if i32 else "mf_gather", _ptr(src), len(src), src.dtype.itemsize,
              _ptr(idx), len(idx), _ptr(dst))
    return dst


def ids_to_i32(ids: np.ndarray, bound: int) -> np.ndarray:
    """int64 ids -> int32, each checked against [0, bound) (threaded;
    MFLibraryError if one is outside)."""
    ids = np.ascontiguousarray(ids, dtype=np.int64)
    out = np.empty(len(ids), np.int32)
    _lib.call("mf_ids_to_i32", _ptr(ids), len(ids), int(bound), _ptr(out))
    return out


def f64_to_f32(x: np.ndarray) -> np.ndarray:
    """float64 -> float32 (threaded; NumPy's round-to-nearest cast)."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    out = np.empty(len(x), np.float32)
    _lib.call("mf_f64_to_f32", _ptr(x), len(x), _ptr(out))
    return out

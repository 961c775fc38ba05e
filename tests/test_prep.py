"""fit() preprocessing on the native path (mf_prep.cpp, host only) against the
pandas / NumPy calls it replaces (recommender_base.py:120-141 and
kernel_matrix_factorization.py:371 of the reference): same outputs, same
draws from NumPy's global RandomState, same errors.  CPU only."""

import numpy as np
import pandas as pd
import pytest

from matrix_factorization import _lib, _prep
from matrix_factorization import recommender_base as rb
from matrix_factorization import KernelMF


def _state_equal(s1, s2):
    return (s1[0] == s2[0] and np.array_equal(s1[1], s2[1]) and s1[2] == s2[2]
            and s1[3] == s2[3] and s1[4] == s2[4])


@pytest.mark.parametrize("n", [0, 1, 2, 3, 5, 64, 65, 1000, 70_001, 1_000_003])
def test_legacy_permutation_is_numpys(n):
    for seed in (0, 11):
        np.random.seed(seed)
        a = np.random.permutation(n)
        s1 = np.random.get_state()
        np.random.seed(seed)
        b = _prep.legacy_permutation(n)
        s2 = np.random.get_state()
        assert np.array_equal(a, b)
        assert _state_equal(s1, s2)


def test_legacy_shuffle_mid_stream():
    # a pending Gaussian and an MT position inside the 624-word block
    for draws in (0, 1, 623, 624, 625, 5000):
        np.random.seed(7)
        np.random.randint(0, 10, draws)
        np.random.normal()
        st = np.random.get_state()
        a = np.arange(123_457, dtype=np.int64) * 3
        np.random.shuffle(a)
        x1 = np.random.rand(3)
        np.random.set_state(st)
        b = np.arange(123_457, dtype=np.int64) * 3
        _prep.legacy_shuffle_(b)
        x2 = np.random.rand(3)
        assert np.array_equal(a, b) and np.array_equal(x1, x2), draws


@pytest.mark.parametrize("simd", [None, "0"])
@pytest.mark.parametrize("threads", [None, "2"])
@pytest.mark.parametrize("dtype,n,draws", [(np.int32, 5_000_000, 0), (np.int32, 4_194_305, 623),
                                           (np.int64, 4_500_001, 624), (np.int32, 6_000_011, 5)])
def test_large_shuffle_is_numpys(dtype, n, draws, threads, simd, monkeypatch):
    """Millions of elements (the prefetch ring wraps many times, the MT state
    crosses thousands of 624-word blocks): the same permutation and the same
    RandomState afterwards as np.random.shuffle, from any MT position -- on
    one thread (the default) and on the two-thread form (draws / swaps,
    MF_SHUFFLE_THREADS=2), with the AVX-512 draws where the host has them
    and with the scalar draws (MF_SHUFFLE_SIMD=0)."""
    if simd is None:
        monkeypatch.delenv("MF_SHUFFLE_SIMD", raising=False)
    else:
        monkeypatch.setenv("MF_SHUFFLE_SIMD", simd)
    if threads is None:
        monkeypatch.delenv("MF_SHUFFLE_THREADS", raising=False)
    else:
        monkeypatch.setenv("MF_SHUFFLE_THREADS", threads)
    np.random.seed(19)
    np.random.randint(0, 10, draws)
    st = np.random.get_state()
    a = np.arange(n, dtype=dtype)
    np.random.shuffle(a)
    x1 = np.random.rand(3)
    np.random.set_state(st)
    b = np.arange(n, dtype=dtype)
    _prep.legacy_shuffle_(b)
    x2 = np.random.rand(3)
    assert np.array_equal(a, b) and np.array_equal(x1, x2)


@pytest.mark.parametrize("threads", [None, "2"])
def test_large_permutation_is_numpys(threads, monkeypatch):
    """np.random.permutation(n) at 5M (fit()'s X.sample(frac=1) draw), both
    shuffle forms: the same permutation and RandomState afterwards."""
    if threads is None:
        monkeypatch.delenv("MF_SHUFFLE_THREADS", raising=False)
    else:
        monkeypatch.setenv("MF_SHUFFLE_THREADS", threads)
    np.random.seed(23)
    a = np.random.permutation(5_000_003)
    x1 = np.random.rand(3)
    np.random.seed(23)
    b = _prep.legacy_permutation(5_000_003)
    x2 = np.random.rand(3)
    assert np.array_equal(a, b) and np.array_equal(x1, x2)


def test_legacy_shuffle_falls_back_for_other_layouts():
    np.random.seed(3)
    a = np.arange(1000, dtype=np.int32)
    np.random.shuffle(a)
    np.random.seed(3)
    b = np.arange(1000, dtype=np.int32)
    _prep.legacy_shuffle_(b)
    assert np.array_equal(a, b)


def test_legacy_shuffle_rejects_bad_state():
    key = np.zeros(624, np.uint32)
    import ctypes
    pos = ctypes.c_int32(625)
    a = np.arange(10, dtype=np.int64)
    with pytest.raises(_lib.MFLibraryError):
        _lib.call("mf_legacy_shuffle", key.ctypes.data, ctypes.addressof(pos), a.ctypes.data, 10)


@pytest.mark.parametrize("n,hi", [(0, 5), (1, 5), (10, 3), (5000, 40), (200_000, 10**15),
                                  (300_000, 2**62), (1_000_000, 700)])
def test_factorize_is_pandas(n, hi):
    rs = np.random.RandomState(n % 1000)
    v = rs.randint(-hi, hi, n).astype(np.int64)
    c, u = _prep.factorize(v)
    c2, u2 = pd.factorize(v, sort=False)
    assert np.array_equal(c, c2) and np.array_equal(u, u2)


@pytest.mark.parametrize("n,lo,hi", [(0, 0, 5), (1, 7, 8), (10, -3, 3), (5000, 0, 40),
                                     (200_000, -10**15, 10**15), (300_000, 0, 2**62),
                                     (1_000_000, 1000, 1700), (400_000, 0, 2_000_000)])
def test_factorize_shuffled_is_pandas(n, lo, hi):
    """dense ids of the unshuffled column (direct range or hashed) +
    first appearance in perm order == pd.factorize(v[perm])."""
    rs = np.random.RandomState(n % 997)
    v = rs.randint(lo, hi, n).astype(np.int64)
    perm = rs.permutation(n).astype(np.int64)
    dn = _prep.dense_ids(v)
    direct = dn[3] is None
    assert direct == (n > 0 and hi - lo <= n + _prep.DIRECT_SPAN_SLACK)
    c, u = _prep.factorize_shuffled(dn, perm)
    c2, u2 = pd.factorize(v[perm], sort=False)
    assert np.array_equal(c, c2) and np.array_equal(u, u2)


def test_first_appearance_rejects_bad_permutation():
    v = np.arange(10, dtype=np.int64)
    with pytest.raises(_lib.MFLibraryError):
        _prep.factorize_shuffled(_prep.dense_ids(v), np.full(10, 10, np.int64))


@pytest.mark.parametrize("n", [0, 1, 2, 1000, 300_000])
def test_pairs_duplicated_is_pandas(n):
    rs = np.random.RandomState(n)
    side = max(2, int(np.sqrt(n)) * 3)
    a = rs.randint(0, side, n)
    b = rs.randint(0, side, n)
    want = bool(pd.DataFrame({"a": a, "b": b}).duplicated().sum() != 0)
    assert _prep.pairs_duplicated(a, b) == want
    k = np.unique(a.astype(np.int64) * side + b)
    rs.shuffle(k)
    assert not _prep.pairs_duplicated(k // side, k % side)
    if len(k) > 1:                                # one duplicate at the far end
        k2 = np.concatenate([k, k[:1]])
        assert _prep.pairs_duplicated(k2 // side, k2 % side)
    # (a, b) and (b, a) are different pairs
    assert not _prep.pairs_duplicated(np.array([1, 2]), np.array([2, 1]))


@pytest.mark.parametrize("idx_dtype", [np.int64, np.int32])
def test_gather_and_bounds(idx_dtype):
    """mf_gather (int64 indices) and mf_gather_i32 (int32 indices: the
    relabelled plans' host ids): src[idx], out-of-range indices refused."""
    rs = np.random.RandomState(0)
    for dt in (np.float32, np.float64, np.int32, np.int64):
        src = rs.randint(0, 1000, 100_000).astype(dt)
        idx = rs.randint(0, len(src), 250_000).astype(idx_dtype)
        assert np.array_equal(_prep.gather(src, idx), src[idx])
    for bad in ([0, 10], [-1, 0]):
        with pytest.raises(_lib.MFLibraryError):
            _prep.gather(np.zeros(10, np.float32), np.array(bad, idx_dtype))


def test_native_narrowing_is_numpys():
    """The engine's inputs narrowed on the host threads (_make_engine at
    10^8 rows): int64 ids -> int32 with the [0, bound) check, float64
    ratings -> float32 as NumPy casts them (NaN, inf, overflow included)."""
    rs = np.random.RandomState(4)
    ids = rs.randint(0, 70_000, 2_000_003).astype(np.int64)
    assert np.array_equal(_prep.ids_to_i32(ids, 70_000), ids.astype(np.int32))
    for bad in (69_999, ):
        with pytest.raises(_lib.MFLibraryError):
            _prep.ids_to_i32(ids, bad)
    neg = ids.copy()
    neg[1_234_567] = -1
    with pytest.raises(_lib.MFLibraryError):
        _prep.ids_to_i32(neg, 70_000)
    x = rs.normal(0, 1e3, 2_000_001)
    x[[3, 4, 5, 6]] = [np.nan, np.inf, -1e300, 3.4028235677973366e38]
    with np.errstate(over="ignore"):
        want = x.astype(np.float32)
    assert np.array_equal(_prep.f64_to_f32(x), want, equal_nan=True)


def _frame(n, dtype, seed, index=None):
    rs = np.random.RandomState(seed)
    nu, ni = 3000, 700
    keys = rs.choice(nu * ni, n, replace=False)
    if np.dtype(dtype).kind == "i":
        u = (keys // ni * 7 - 5000).astype(dtype)
    elif np.dtype(dtype).itemsize == 8:           # ids above 2^63
        u = (keys // ni).astype(np.uint64) + np.uint64(2**63)
    else:
        u = (keys // ni + 7).astype(dtype)
    i = (keys % ni * 13 + 1).astype(dtype)
    X = pd.DataFrame({"user_id": u, "item_id": i, "extra": 1.0}, index=index)
    y = pd.Series(rs.randint(1, 6, n).astype(np.float64), index=X.index)
    return X, y


def _run(model, X, y, typ, fast, monkeypatch, seed):
    monkeypatch.setattr(rb, "FAST_PREP_MIN_ROWS", 0 if fast else 1 << 62)
    np.random.seed(seed)
    out = model._preprocess_data(X, y, type=typ)
    return out, np.random.get_state()


@pytest.mark.parametrize("dtype", [np.int32, np.int64, np.uint32, np.uint64])
@pytest.mark.parametrize("index", ["range", "offset", "labels"])
def test_fit_preprocess_native_equals_pandas(dtype, index, monkeypatch):
    n = 20_000
    idx = {"range": None, "offset": pd.RangeIndex(5, 5 + 3 * n, 3),
           "labels": pd.Index(np.random.RandomState(1).permutation(n) * 2 + 1)}[index]
    X, y = _frame(n, dtype, 4, idx)
    ma, mb = KernelMF(), KernelMF()
    a, sa = _run(ma, X, y, "fit", True, monkeypatch, 21)
    b, sb = _run(mb, X, y, "fit", False, monkeypatch, 21)
    assert _state_equal(sa, sb)
    assert list(a.columns) == list(b.columns)
    assert a.index.equals(b.index)
    for c in ("user_id", "item_id", "rating"):
        assert a[c].dtype == b[c].dtype and np.array_equal(a[c].to_numpy(), b[c].to_numpy())
    assert (ma.n_users, ma.n_items) == (mb.n_users, mb.n_items)
    assert list(ma.user_id_map.items()) == list(mb.user_id_map.items())
    assert list(ma.item_id_map.items()) == list(mb.item_id_map.items())
    # the reference's own construction: unique() of the shuffled frame
    np.random.seed(21)
    Xs = X.loc[:, ["user_id", "item_id"]].sample(frac=1, replace=False)
    assert list(ma.user_id_map) == list(Xs["user_id"].unique())
    assert list(ma.item_id_map) == list(Xs["item_id"].unique())


@pytest.mark.parametrize("fast", [True, False])
def test_duplicates_raise(fast, monkeypatch):
    X, y = _frame(5000, np.int64, 2)
    X.iloc[4000, :2] = X.iloc[17, :2].to_numpy()
    st = np.random.get_state()
    with pytest.raises(ValueError, match="Duplicate"):
        _run(KernelMF(), X, y, "fit", fast, monkeypatch, 0)
    # the check fails before X.sample's draw: the RNG is where seed(0) left it
    after = np.random.get_state()
    np.random.seed(0)
    assert _state_equal(after, np.random.get_state())
    np.random.set_state(st)


@pytest.mark.parametrize("ykind", ["permuted_index", "int_series", "array", "partial_index"])
def test_fit_preprocess_rating_alignment(ykind, monkeypatch):
    """X["rating"] = y aligns a Series on X's index (and takes an array as
    it stands): the native path, which reads y in place, gives the frame
    the pandas path gives for each form of y."""
    n = 12_000
    X, y = _frame(n, np.int64, 6, pd.Index(np.arange(n) * 3 + 2))
    rs = np.random.RandomState(9)
    if ykind == "permuted_index":
        y = y.iloc[rs.permutation(n)]
    elif ykind == "int_series":
        y = y.astype(np.int64)
    elif ykind == "array":
        y = y.to_numpy()
    else:
        y = y.iloc[: n - 100].copy()
        y.index = y.index + 1                      # some labels missing: NaN ratings
    ma, mb = KernelMF(), KernelMF()
    a, sa = _run(ma, X, y, "fit", True, monkeypatch, 4)
    b, sb = _run(mb, X, y, "fit", False, monkeypatch, 4)
    assert _state_equal(sa, sb) and a.index.equals(b.index)
    for c in ("user_id", "item_id", "rating"):
        assert a[c].dtype == b[c].dtype
        assert np.array_equal(a[c].to_numpy(), b[c].to_numpy(), equal_nan=True)


def test_update_preprocess_native_equals_pandas(monkeypatch):
    X, y = _frame(8000, np.int64, 5)
    ma, mb = KernelMF(), KernelMF()
    _run(ma, X.iloc[:6000], y.iloc[:6000], "fit", True, monkeypatch, 1)
    _run(mb, X.iloc[:6000], y.iloc[:6000], "fit", False, monkeypatch, 1)
    Xn, yn = X.iloc[5000:], y.iloc[5000:]
    (a, ka, na), sa = _run(ma, Xn, yn, "update", True, monkeypatch, 2)
    (b, kb, nb), sb = _run(mb, Xn, yn, "update", False, monkeypatch, 2)
    assert _state_equal(sa, sb) and a.equals(b) and ka == kb and na == nb
    assert list(ma.user_id_map.items()) == list(mb.user_id_map.items())

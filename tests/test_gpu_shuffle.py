"""The exact schedule's per-epoch np.random.shuffle with its swaps on the GPU
(engine.ExactShuffler: host draws, mf_shuffle_swaps_device's reservation
rounds, the last swaps on the host): the same permutation and the same
RandomState afterwards as NumPy, call after call (the device keeps the
order it made) and from an order it did not make; and an exact-schedule
fit gives the same parameters with the GPU swaps as with the host shuffle."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,rounds", [(5_000_003, None), (4_194_305, None), (4_500_007, "1"),
                                      (4_500_007, "2")])
def test_gpu_shuffle_is_numpys(n, rounds, monkeypatch):
    """Also with one or two reservation rounds (MF_SHUFFLE_GPU_ROUNDS), so
    that the in-order one-thread fixup takes thousands of stragglers."""
    import torch

    if rounds is None:
        monkeypatch.delenv("MF_SHUFFLE_GPU_ROUNDS", raising=False)
    else:
        monkeypatch.setenv("MF_SHUFFLE_GPU_ROUNDS", rounds)

    from matrix_factorization.engine import ExactShuffler

    sh = ExactShuffler(n, torch.device("cuda:0"))
    np.random.seed(11)
    np.random.randint(0, 9, 3)
    st = np.random.get_state()
    want = np.arange(n, dtype=np.int32)
    wants = []
    for _ in range(3):
        np.random.shuffle(want)
        wants.append(want.copy())
    x_ref = np.random.rand(2)
    np.random.set_state(st)
    got = np.arange(n, dtype=np.int32)
    for e in range(3):
        src = got
        got = sh.shuffle_from(src)
        assert got is not src
        assert np.array_equal(got, wants[e]), f"shuffle {e} differs"
    assert np.array_equal(np.random.rand(2), x_ref)
    # an order it did not make (uploaded), and src left alone
    np.random.set_state(st)
    other = np.random.RandomState(5).permutation(n).astype(np.int32)
    keep = other.copy()
    np.random.set_state(st)
    ref = other.copy()
    np.random.shuffle(ref)
    np.random.set_state(st)
    out = sh.shuffle_from(other)
    assert np.array_equal(other, keep)
    assert np.array_equal(out, ref)


def test_exact_fit_gpu_swaps_equal_host_shuffle(monkeypatch):
    from matrix_factorization.engine import EXACT_GPU_SHUFFLE_MIN, SGDEngine, fit_epochs

    nu, ni, k = 60000, 8000, 16
    n = EXACT_GPU_SHUFFLE_MIN + 12345
    rs = np.random.RandomState(2)
    keys = rs.choice(nu * ni, n, replace=False)
    u = (keys // ni).astype(np.int32)
    i = (keys % ni).astype(np.int32)
    r = rs.randint(1, 6, n).astype(np.float64)
    P0 = rs.normal(0, 0.1, (nu, k))
    Q0 = rs.normal(0, 0.1, (ni, k))
    out = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("MF_EXACT_GPU_SHUFFLE", mode)
        eng = SGDEngine(u, i, r, nu, ni, k, "linear", "float64", "cuda:0",
                        global_mean=float(r.mean()), min_rating=1, max_rating=5)
        eng.load_params(P0, Q0, np.zeros(nu), np.zeros(ni))
        np.random.seed(21)
        rmse = fit_epochs(eng, 3, "exact", 0.01, 0.02)
        out[mode] = (eng.params_numpy(), rmse, np.random.rand(2))
        assert (getattr(eng, "_exact_shuffler", None) is not None) == (mode == "1")
    (pa, ra, xa), (pb, rb, xb) = out["1"], out["0"]
    for a, b in zip(pa, pb):
        assert np.array_equal(a, b)
    assert ra == rb
    assert np.array_equal(xa, xb)


def test_device_permutation_is_numpys():
    """fit()'s X.sample(frac=1) draw at 10^8 rows (legacy_permutation_device:
    the swaps on the GPU): np.random.permutation's result and RandomState."""
    import torch

    from matrix_factorization.engine import legacy_permutation_device

    n = 5_000_011
    np.random.seed(8)
    want = np.random.permutation(n)
    x_ref = np.random.rand(2)
    np.random.seed(8)
    got = legacy_permutation_device(n, torch.device("cuda:0"))
    assert got.dtype == np.int64
    assert np.array_equal(got, want)
    assert np.array_equal(np.random.rand(2), x_ref)

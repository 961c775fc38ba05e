"""The training-RMSE pass (mf_sse, _calculate_rmse kernel_matrix_factorization.py:
240-317) in its kernel variants: k_sse_lean (the default: biases loaded once
per chunk), its round-5 form with a bias load per rating (variant 12),
k_sse_owned (user rows owned per run; variant 6),
k_sse_pipe (the same walk software-pipelined, pieces of 8 or 4 ratings) and
k_sse_stream.  Per rating the arithmetic is identical; the FP64 sums differ
only in accumulation order (the grid follows each kernel's occupancy), so
they agree to 1e-12 relative, and with the FP64 oracle to 1e-9 relative
(FP32 products and dot-product order)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("k,nu,ni,nnz", [(64, 20000, 4000, 600000), (64, 300, 5000, 200000),
                                         (20, 5000, 3000, 300000)])      # row tails
def test_sse_variants_agree(k, nu, ni, nnz, monkeypatch):
    import oracle
    from matrix_factorization.engine import SGDEngine

    rs = np.random.RandomState(k + nu)
    keys = rs.choice(nu * ni, nnz, replace=False)
    u = (keys // ni).astype(np.int32)
    i = (keys % ni).astype(np.int32)
    r = rs.randint(1, 6, nnz).astype(np.float32)
    P = rs.normal(0, 0.3, (nu, k)).astype(np.float32)
    Q = rs.normal(0, 0.3, (ni, k)).astype(np.float32)
    bu = rs.normal(0, 0.1, nu).astype(np.float32)
    bi = rs.normal(0, 0.1, ni).astype(np.float32)
    eng = SGDEngine(u, i, r, nu, ni, k, "linear", "float32", "cuda:0",
                    global_mean=float(r.mean()), min_rating=1, max_rating=5)
    eng.load_params(P, Q, bu, bi)
    got = {}
    for slot, var in enumerate(("0", "4", "5", "1", "6", "12")):
        monkeypatch.setenv("MF_SSE_VARIANT", var)
        eng.sse_async(slot)
        got[var] = eng.sse_values(slot + 1)[slot]
    monkeypatch.delenv("MF_SSE_VARIANT")
    for v in got.values():
        assert abs(v - got["0"]) <= 1e-12 * got["0"], got
    ref = oracle.sse(u, i, r.astype(np.float64), eng.global_mean, bu.astype(np.float64),
                     bi.astype(np.float64), P.astype(np.float64), Q.astype(np.float64))
    for v in got.values():
        assert abs(v - ref) <= 1e-9 * ref, (got, ref)


@pytest.mark.parametrize("tiles", ["1,8", "4,16", "8,16", "2,32", "16,8"])
def test_device_eval_order_equals_host(tiles, monkeypatch):
    """The evaluation order computed on the GPU (engine._eval_order_device:
    stable sort by tile and user) is mf_sched_tiles' host order exactly."""
    from matrix_factorization.engine import SGDEngine, sched_tiles

    rs = np.random.RandomState(11)
    nu, ni, nnz = 30000, 7000, 900000
    keys = rs.choice(nu * ni, nnz, replace=False)
    u = (keys // ni).astype(np.int32)
    i = (keys % ni).astype(np.int32)
    r = rs.randint(1, 6, nnz).astype(np.float64)
    monkeypatch.setenv("MF_SSE_TILES", tiles)
    eng = SGDEngine(u, i, r, nu, ni, 16, "linear", "float64", "cuda:0")
    c, s = (int(x) for x in tiles.split(","))
    order, offs = eng._eval_order_device(c, s)
    hs, ho = sched_tiles(u, i, nu, ni, c, s)
    assert np.array_equal(order.cpu().numpy(), hs) and np.array_equal(offs, ho)
    assert np.array_equal(eng.eu.cpu().numpy(), u[hs])


@pytest.mark.parametrize("dtype,k", [("float64", 64), ("float32", 64), ("float64", 20)])
@pytest.mark.parametrize("tiles", ["4,16", "1,16", "8,8"])
def test_phased_tile_pass_agrees(dtype, k, tiles, monkeypatch):
    """The FP64 pass over tiles walked in phases by a resident grid
    (k_sse_phased) and the dispatch-ordered walk of the same tiles give the
    default pass's SSE up to FP64 summation order (1e-12 relative) and the
    oracle's to 1e-9."""
    import oracle
    from matrix_factorization.engine import SGDEngine

    rs = np.random.RandomState(k + 5)
    nu, ni, nnz = 20000, 4000, 600000
    keys = rs.choice(nu * ni, nnz, replace=False)
    u = (keys // ni).astype(np.int32)
    i = (keys % ni).astype(np.int32)
    r = rs.randint(1, 6, nnz).astype(dtype)
    P = rs.normal(0, 0.3, (nu, k)).astype(dtype)
    Q = rs.normal(0, 0.3, (ni, k)).astype(dtype)
    bu = rs.normal(0, 0.1, nu).astype(dtype)
    bi = rs.normal(0, 0.1, ni).astype(dtype)
    monkeypatch.delenv("MF_SSE_TILES", raising=False)
    eng = SGDEngine(u, i, r, nu, ni, k, "linear", dtype, "cuda:0",
                    global_mean=float(r.mean()), min_rating=1, max_rating=5)
    eng.load_params(P, Q, bu, bi)
    eng.sse_async(0)
    base = eng.sse_values(1)[0]
    monkeypatch.setenv("MF_SSE_TILES", tiles)
    eng._build_eval()
    got = []
    for slot, ph in enumerate(("1", "0")):
        monkeypatch.setenv("MF_SSE_PHASED", ph)
        eng.sse_async(slot)
        got.append(eng.sse_values(slot + 1)[slot])
    for v in got:
        assert abs(v - base) <= 1e-12 * base, (got, base)
    ref = oracle.sse(u, i, r.astype(np.float64), eng.global_mean, bu.astype(np.float64),
                     bi.astype(np.float64), P.astype(np.float64), Q.astype(np.float64))
    assert abs(base - ref) <= 1e-9 * ref

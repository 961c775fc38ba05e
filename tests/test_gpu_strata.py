"""GPU parity of the stratified sweep (schedule='strata', mf_strata.hpp).

A strata epoch applies the ratings in one sequential order (strata in the
given order, blocks of a stratum in any order, steps of a block from the
seeded rotation); StrataPlan.serial_order lists it.  The GPU result must equal
the oracle's sequential sweep over that order:
  FP64 parameters: max |diff| <= 1e-11 * max(1, |value|), RMSE <= 1e-12
  FP32 state vs FP64 oracle: RMSE <= 1e-5 (the north-star bar)
Every block holds several ratings per user on the user's slot, often in
consecutive steps, so both the prefetched user rows (read before the previous
step's stores) and the forwarding of a just-updated row are exercised.
"""

import numpy as np
import pandas as pd
import pytest

pytestmark = pytest.mark.gpu


def _close(a, b, tol):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    assert a.shape == b.shape
    scale = max(1.0, float(np.max(np.abs(b)))) if b.size else 1.0
    err = float(np.max(np.abs(a - b))) if a.size else 0.0
    assert err <= tol * scale, f"max |diff| {err:.3e} > {tol:.0e} * {scale:.3g}"


def _synthetic(seed, n_users, n_items, nnz):
    rs = np.random.RandomState(seed)
    keys = rs.choice(n_users * n_items, nnz, replace=False)
    u = (keys // n_items).astype(np.int32)
    i = (keys % n_items).astype(np.int32)
    r = rs.randint(1, 6, nnz).astype(np.float64)
    return u, i, r


def _engine(u, i, r, nu, ni, k, kernel, dtype, P, Q, bu, bi):
    from matrix_factorization.engine import SGDEngine

    eng = SGDEngine(u, i, r, nu, ni, k, kernel, dtype, "cuda:0", gamma=1.0 / max(k, 1),
                    min_rating=1.0, max_rating=5.0, global_mean=float(r.mean()))
    eng.load_params(P, Q, bu, bi)
    return eng


# FP64 LDS image per block: items/B * (k+1) * 8 B + users/B * 8 B <= 160 KiB
@pytest.mark.parametrize("kernel,k,B", [("linear", 64, 4), ("sigmoid", 32, 3), ("rbf", 16, 5),
                                        ("linear", 100, 8), ("sigmoid", 7, 2), ("linear", 8, 1)])
def test_strata_epochs_equal_serialized_oracle(kernel, k, B):
    import oracle

    nu, ni, nnz = 3000, 800, 120000
    u, i, r = _synthetic(11, nu, ni, nnz)
    rs = np.random.RandomState(12)
    P = rs.normal(0, 0.1, (nu, k)); Q = rs.normal(0, 0.1, (ni, k))
    bu = np.zeros(nu); bi = np.zeros(ni)
    eng = _engine(u, i, r, nu, ni, k, kernel, "float64", P, Q, bu, bi)
    plan = eng.prepare_strata(n_blocks=B)
    assert plan.B == B
    mu = eng.global_mean
    hyp = dict(kernel=kernel, gamma=eng.gamma, min_rating=1.0, max_rating=5.0)
    P2, Q2, bu2, bi2 = P.copy(), Q.copy(), bu.copy(), bi.copy()
    for ep in range(2):
        seq = rs.permutation(B).astype(np.int32)
        seed = int(rs.randint(0, 2**31 - 1))
        eng.epoch_strata(seq, seed, lr=0.01, reg=0.02)
        order = plan.serial_order(seq, seed)
        assert np.array_equal(np.sort(order), np.arange(nnz))
        oracle.sgd_pass(eng.u_host, eng.i_host, eng.r_host, mu, bu2, bi2, P2, Q2,
                        lr=0.01, reg=0.02, order=order, **hyp)
    eng.sse_async(0)
    Pg, Qg, bug, big = eng.params_numpy()
    _close(Pg, P2, 1e-11)
    _close(Qg, Q2, 1e-11)
    _close(bug, bu2, 1e-11)
    _close(big, bi2, 1e-11)
    ro = oracle.rmse(eng.u_host, eng.i_host, eng.r_host, mu, bu2, bi2, P2, Q2, **hyp)
    assert abs(eng.rmse_values(1)[0] - ro) < 1e-12


def test_strata_partial_epoch_and_frozen_items():
    """A prefix of the strata is a partial epoch; update_item=False leaves the
    item rows and biases bit-identical (update_users, :234)."""
    import oracle

    nu, ni, nnz, k = 2000, 600, 60000, 64
    u, i, r = _synthetic(21, nu, ni, nnz)
    rs = np.random.RandomState(22)
    P = rs.normal(0, 0.1, (nu, k)); Q = rs.normal(0, 0.1, (ni, k))
    bu = rs.normal(0, 0.1, nu); bi = rs.normal(0, 0.1, ni)
    eng = _engine(u, i, r, nu, ni, k, "linear", "float64", P, Q, bu, bi)
    plan = eng.prepare_strata(n_blocks=6)
    seq = np.array([4, 1, 5], np.int32)
    eng.epoch_strata(seq, 7, lr=0.02, reg=0.05, update_item=False)
    Pg, Qg, bug, big = eng.params_numpy()
    assert np.array_equal(Qg, Q) and np.array_equal(big, bi)
    P2, Q2, bu2, bi2 = P.copy(), Q.copy(), bu.copy(), bi.copy()
    oracle.sgd_pass(eng.u_host, eng.i_host, eng.r_host, eng.global_mean, bu2, bi2, P2, Q2,
                    kernel="linear", lr=0.02, reg=0.05, order=plan.serial_order(seq, 7),
                    update_item=False, min_rating=1.0, max_rating=5.0)
    _close(Pg, P2, 1e-11)
    _close(bug, bu2, 1e-11)


def test_strata_float32_large_slab_rmse_within_1e5():
    """FP32 at rank 64 with ~500-item slabs (≈130 KB of LDS per workgroup)."""
    import oracle

    nu, ni, nnz, k = 3000, 2000, 150000, 64
    u, i, r = _synthetic(31, nu, ni, nnz)
    rs = np.random.RandomState(32)
    P = rs.normal(0, 0.1, (nu, k)); Q = rs.normal(0, 0.1, (ni, k))
    eng = _engine(u, i, r, nu, ni, k, "linear", "float32", P, Q, np.zeros(nu), np.zeros(ni))
    plan = eng.prepare_strata(n_blocks=4)
    assert plan.max_items >= 450
    P2, Q2 = P.copy(), Q.copy()
    bu2, bi2 = np.zeros(nu), np.zeros(ni)
    for ep in range(3):
        seq = rs.permutation(4).astype(np.int32)
        eng.epoch_strata(seq, ep + 100, lr=0.01, reg=0.02)
        eng.sse_async(ep)
        oracle.sgd_pass(eng.u_host, eng.i_host, eng.r_host, eng.global_mean, bu2, bi2, P2, Q2,
                        lr=0.01, reg=0.02, order=plan.serial_order(seq, ep + 100),
                        min_rating=1.0, max_rating=5.0)
    ro = oracle.rmse(eng.u_host, eng.i_host, eng.r_host, eng.global_mean, bu2, bi2, P2, Q2,
                     min_rating=1.0, max_rating=5.0)
    assert abs(eng.rmse_values(3)[2] - ro) < 1e-5


def test_kernelmf_strata_fit_converges():
    import matrix_factorization as mf

    u, i, r = _synthetic(41, 4000, 1000, 200000)
    X = pd.DataFrame({"user_id": u, "item_id": i})
    hp = dict(n_factors=32, n_epochs=6, lr=0.01, reg=0.02, min_rating=1, max_rating=5,
              verbose=0)
    np.random.seed(5)
    ms = mf.KernelMF(dtype="float32", schedule="strata", **hp).fit(X, pd.Series(r))
    np.random.seed(5)
    me = mf.KernelMF(dtype="float32", schedule="exact", **hp).fit(X, pd.Series(r))
    assert np.all(np.diff(ms.train_rmse) < 0)
    # a different (valid) visit order: same trajectory to within SGD noise
    assert abs(ms.train_rmse[-1] - me.train_rmse[-1]) < 2e-3
    pred = ms.predict(X.iloc[:100])
    assert len(pred) == 100 and np.all(np.isfinite(pred))


@pytest.mark.parametrize("dtype,B", [("float64", 6), ("float32", 16)])
def test_persistent_epoch_equals_per_stratum_launches(dtype, B):
    """MF_FLAG_PERSISTENT (one launch per epoch, item slabs resident, neighbour
    waits) applies the same sequential order as one launch per stratum: the
    parameters are bit-identical."""
    nu, ni, nnz, k = 3000, 1200, 150000, 64
    u, i, r = _synthetic(51, nu, ni, nnz)
    rs = np.random.RandomState(52)
    P = rs.normal(0, 0.1, (nu, k)); Q = rs.normal(0, 0.1, (ni, k))
    bu = rs.normal(0, 0.1, nu); bi = rs.normal(0, 0.1, ni)
    out = []
    for persistent in (True, False):
        eng = _engine(u, i, r, nu, ni, k, "linear", dtype, P, Q, bu, bi)
        eng.prepare_strata(n_blocks=B)
        for ep in range(3):
            seq = np.random.RandomState(ep).permutation(B).astype(np.int32)
            eng.epoch_strata(seq, 1000 + ep, lr=0.01, reg=0.02, persistent=persistent)
        eng.check_strata()
        out.append(eng.params_numpy())
    for a, b in zip(*out):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("dtype,B,kernel,k,nu,ni,waves", [
    ("float64", 6, "linear", 64, 3000, 1200, None),
    ("float32", 16, "linear", 64, 3000, 1200, None),
    ("float32", 8, "sigmoid", 32, 3000, 1200, None),
    ("float32", 6, "linear", 64, 200, 2000, None),   # ~80 ratings per user per block:
    ("float32", 8, "sigmoid", 32, 3000, 1200, 8),    # rows forwarded from t-1 and t-2
    ("float32", 6, "linear", 64, 200, 2000, 8),
    ("float32", 8, "sigmoid", 20, 3000, 1200, 8),    # row tails (k < GS * V * W)
])
def test_deep_pipe_equals_per_stratum_launches(dtype, B, kernel, k, nu, ni, waves):
    """MF_FLAG_DEEP_PIPE (user rows gathered two steps ahead, forwarded from
    either of the two previous steps of the slot) keeps the sequential order:
    bit-identical to one launch per stratum, user-only epochs included."""
    nnz = 150000 if nu > 1000 else 100000
    u, i, r = _synthetic(61, nu, ni, nnz)
    rs = np.random.RandomState(62)
    P = rs.normal(0, 0.1, (nu, k)); Q = rs.normal(0, 0.1, (ni, k))
    bu = rs.normal(0, 0.1, nu); bi = rs.normal(0, 0.1, ni)
    out = []
    for deep in (True, None):
        eng = _engine(u, i, r, nu, ni, k, kernel, dtype, P, Q, bu, bi)
        eng.prepare_strata(n_blocks=B, waves=waves)
        eng.strata_deep_pipe = deep
        for ep in range(3):
            seq = np.random.RandomState(ep).permutation(B).astype(np.int32)
            eng.epoch_strata(seq, 2000 + ep, lr=0.01, reg=0.02, update_item=ep != 2,
                             persistent=deep is True)
        eng.check_strata()
        out.append(eng.params_numpy())
    for a, b in zip(*out):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("kernel,k,waves,dtype", [
    ("sigmoid", 32, 8, "float32"), ("linear", 64, 8, "float32"), ("rbf", 16, 8, "float32"),
    ("sigmoid", 32, 4, "float32"), ("linear", 16, 4, "float32"),
    ("sigmoid", 32, 8, "float64"), ("linear", 20, 8, "float64")])
def test_eight_wave_kernels(kernel, k, waves, dtype):
    """The 8-wave strata kernels (plans of half the slots; rows of one vector
    per lane: FP32 k <= 64, FP64 k <= 32) and their narrow 4-wave form (FP32:
    the same plan, lane groups half as wide, MF_FLAG_NARROW): the persistent
    epoch is bit-identical to per-stratum launches, and both are the oracle's
    sequential sweep in the plan's serial order (FP32 vs FP64: train RMSE
    within 1e-5; FP64: parameters within 1e-11)."""
    import oracle

    nu, ni, nnz = 3000, 800, 120000
    u, i, r = _synthetic(71, nu, ni, nnz)
    rs = np.random.RandomState(72)
    P = rs.normal(0, 0.1, (nu, k)); Q = rs.normal(0, 0.1, (ni, k))
    bu = rs.normal(0, 0.1, nu); bi = rs.normal(0, 0.1, ni)
    out = []
    for persistent in (True, False):
        eng = _engine(u, i, r, nu, ni, k, kernel, dtype, P, Q, bu, bi)
        plan = eng.prepare_strata(n_blocks=6, waves=waves)
        from matrix_factorization.engine import strata_slots
        assert plan.NS == strata_slots(k, eng.dcode, waves) == strata_slots(k, eng.dcode) // 2
        assert plan.narrow == (waves == 4)
        orders = []
        for ep in range(2):
            seq = np.random.RandomState(ep).permutation(6).astype(np.int32)
            _, n_launch = eng.epoch_strata(seq, 3000 + ep, lr=0.01, reg=0.02, timing=True,
                                           persistent=persistent)
            assert n_launch == (1 if persistent else 6)
            orders.append(plan.serial_order(seq, 3000 + ep))
        eng.check_strata()
        eng.sse_async(0)
        out.append(eng.params_numpy() + (eng.rmse_values(1)[0],))
    for a, b in zip(out[0][:4], out[1][:4]):
        assert np.array_equal(a, b)
    P2, Q2, bu2, bi2 = P.copy(), Q.copy(), bu.copy(), bi.copy()
    hyp = dict(kernel=kernel, gamma=1.0 / k, min_rating=1.0, max_rating=5.0)
    for order in orders:
        oracle.sgd_pass(eng.u_host, eng.i_host, eng.r_host.astype(np.float64), eng.global_mean,
                        bu2, bi2, P2, Q2, lr=0.01, reg=0.02, order=order, **hyp)
    ro = oracle.rmse(eng.u_host, eng.i_host, eng.r_host.astype(np.float64), eng.global_mean,
                     bu2, bi2, P2, Q2, **hyp)
    assert abs(out[0][4] - ro) < (1e-12 if dtype == "float64" else 1e-5)
    if dtype == "float64":
        for g, o in zip(out[0][:4], (P2, Q2, bu2, bi2)):
            _close(g, o, 1e-11)


def test_auto_waves_picks_lower_cost():
    """prepare_strata(waves=None) keeps the 16-wave plan when it fills >= 70 %
    of its slots, else the plan with the lower steps x waves (the per-CU
    VALU issue that bounds item-degree-bound plans)."""
    from matrix_factorization.engine import strata_slots

    nu, ni, k, B = 20000, 400, 32, 4
    u, i, r = _synthetic(81, nu, ni, 200000)
    rs = np.random.RandomState(82)
    P, Q = rs.normal(0, 0.1, (nu, k)), rs.normal(0, 0.1, (ni, k))
    plans = {}
    for wv in (16, 8, None):
        eng = _engine(u, i, r, nu, ni, k, "sigmoid", "float32", P, Q, np.zeros(nu), np.zeros(ni))
        plans[wv] = eng.prepare_strata(n_blocks=B, waves=wv)
    cost = {wv: int(plans[wv].bstep[-1]) * wv for wv in (16, 8)}
    fill16 = len(u) / plans[16].n_positions
    expect = 16 if fill16 >= 0.7 else min(cost, key=cost.get)
    assert plans[None].NS == strata_slots(k, eng.dcode, expect), (fill16, cost)
    seq = np.random.RandomState(0).permutation(B).astype(np.int32)
    eng.epoch_strata(seq, 5, 0.01, 0.02)
    eng.check_strata()


@pytest.mark.parametrize("dtype,kernel,k,P,B,waves", [
    ("float64", "linear", 64, 2, 4, None),
    ("float64", "sigmoid", 32, 3, 3, None),
    ("float32", "linear", 64, 2, 6, 8),
    ("float64", "rbf", 16, 2, 5, None),
])
def test_item_phases_equal_serialized_oracle(dtype, kernel, k, P, B, waves):
    """PhasedStrata: the items cut into P ranges, each a whole strata plan run
    as its own persistent launch.  The epoch equals the oracle's sweep in
    plan.serial_order (phase 0's order, then phase 1's, ...), persistent and
    per-stratum launches are bit-identical, and the delta-out form leaves Q /
    b_i untouched with the same update in the deltas."""
    import torch

    import oracle
    from matrix_factorization.engine import PhasedStrata

    nu, ni, nnz = 3000, 900, 120000
    u, i, r = _synthetic(31 + P, nu, ni, nnz)
    rs = np.random.RandomState(32)
    P0 = rs.normal(0, 0.1, (nu, k)); Q0 = rs.normal(0, 0.1, (ni, k))
    bu0 = rs.normal(0, 0.1, nu); bi0 = rs.normal(0, 0.1, ni)
    eps = [(rs.permutation(B).astype(np.int32), int(rs.randint(0, 2**31 - 1))) for _ in range(2)]
    out = []
    for persistent in (True, False):
        eng = _engine(u, i, r, nu, ni, k, kernel, dtype, P0, Q0, bu0, bi0)
        plan = eng.prepare_strata(n_blocks=B, waves=waves, phases=P)
        assert isinstance(plan, PhasedStrata) and len(plan.phases) == P and plan.B == B
        for seq, seed in eps:
            ms = eng.epoch_strata(seq, seed, lr=0.01, reg=0.02, persistent=persistent,
                                  timing=True)
            assert ms[1] == (P if persistent else P * B)
        eng.check_strata()
        out.append(eng.params_numpy())
    for a, b in zip(*out):
        assert np.array_equal(a, b)
    hyp = dict(kernel=kernel, gamma=eng.gamma, min_rating=1.0, max_rating=5.0)
    P2, Q2, bu2, bi2 = P0.copy(), Q0.copy(), bu0.copy(), bi0.copy()
    for seq, seed in eps:
        order = plan.serial_order(seq, seed)
        assert np.array_equal(np.sort(order), np.arange(nnz))
        oracle.sgd_pass(eng.u_host, eng.i_host, eng.r_host.astype(np.float64), eng.global_mean,
                        bu2, bi2, P2, Q2, lr=0.01, reg=0.02, order=order, **hyp)
    tol = 1e-11 if dtype == "float64" else 1e-4
    for g, o in zip(out[0], (P2, Q2, bu2, bi2)):
        _close(g, o, tol)
    # delta-out: the replica stays, the deltas carry the epoch's item update
    eng = _engine(u, i, r, nu, ni, k, kernel, dtype, P0, Q0, bu0, bi0)
    eng.prepare_strata(n_blocks=B, waves=waves, phases=P)
    dq = torch.zeros_like(eng.Q)
    dbi = torch.zeros_like(eng.bi)
    seq, seed = eps[0]
    eng.epoch_strata(seq, seed, lr=0.01, reg=0.02, delta=(dq, dbi))
    eng.check_strata()
    Pd, Qd, bud, bid = eng.params_numpy()
    assert np.array_equal(Qd, Q0.astype(eng.ndt)) and np.array_equal(bid, bi0.astype(eng.ndt))
    ref = _engine(u, i, r, nu, ni, k, kernel, dtype, P0, Q0, bu0, bi0)
    ref.prepare_strata(n_blocks=B, waves=waves, phases=P)
    ref.epoch_strata(seq, seed, lr=0.01, reg=0.02)
    Pr, Qr, bur, bir = ref.params_numpy()
    assert np.array_equal(Pd, Pr)
    _close(Qd + dq.cpu().numpy(), Qr, 1e-12 if dtype == "float64" else 1e-6)
    if kernel != "rbf":
        _close(bid + dbi.cpu().numpy(), bir, 1e-12 if dtype == "float64" else 1e-6)


def test_item_phases_chosen_when_slabs_exceed_lds():
    """prepare_strata() picks item phases when the item rows cannot be spread
    over one workgroup per CU (FP64 rank 128 over 60K items: 62 MB of rows,
    236 KiB per workgroup at B = 256 > 160 KiB of LDS), and the phased
    persistent epoch equals its per-stratum launches."""
    from matrix_factorization.engine import PhasedStrata, stratum_order

    nu, ni, nnz, k = 4000, 60000, 200000, 128
    u, i, r = _synthetic(41, nu, ni, nnz)
    rs = np.random.RandomState(42)
    P0 = rs.normal(0, 0.1, (nu, k)); Q0 = rs.normal(0, 0.1, (ni, k))
    eng = _engine(u, i, r, nu, ni, k, "linear", "float64", P0, Q0, np.zeros(nu), np.zeros(ni))
    plan = eng.prepare_strata()
    assert isinstance(plan, PhasedStrata), "60K items of FP64 rank 128 (62 MB) need phases"
    assert plan.B <= eng._cus()
    seq = stratum_order(rs, plan)
    ms = eng.epoch_strata(seq, 5, lr=0.01, reg=0.02, timing=True)
    assert ms[1] == len(plan.phases)                # persistent: one launch per phase
    eng.check_strata()
    got = eng.params_numpy()
    eng2 = _engine(u, i, r, nu, ni, k, "linear", "float64", P0, Q0, np.zeros(nu), np.zeros(ni))
    eng2.prepare_strata(n_blocks=plan.B, phases=len(plan.phases))
    eng2.epoch_strata(seq, 5, lr=0.01, reg=0.02, persistent=False)
    for a, b in zip(got, eng2.params_numpy()):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("kernel,k,B,waves", [("sigmoid", 32, 32, 8), ("linear", 64, 64, None),
                                              ("linear", 32, 16, None)])
def test_l2_handoff_equals_per_stratum_launches(kernel, k, B, waves, monkeypatch):
    """MF_FLAG_L2_HANDOFF (MF_STRATA_L2=1 with the XCD-class stratum order):
    inside a class the user rows are stored plainly and handed over through
    the XCD's L2, with an L2 write-back before every hand-off to another XCD.
    Same sequential order, so the parameters are bit-identical to one launch
    per stratum; the kernel published every workgroup's XCC id for the
    launch (the workspace tail), i.e. the launcher did turn it on."""
    import torch

    from matrix_factorization.engine import stratum_order

    nu, ni, nnz = 4000, 2000, 300000
    u, i, r = _synthetic(71, nu, ni, nnz)
    rs = np.random.RandomState(72)
    P = rs.normal(0, 0.1, (nu, k)); Q = rs.normal(0, 0.1, (ni, k))
    bu = rs.normal(0, 0.1, nu); bi = rs.normal(0, 0.1, ni)
    monkeypatch.setenv("MF_STRATA_L2", "1")
    out = []
    for persistent in (True, False):
        eng = _engine(u, i, r, nu, ni, k, kernel, "float32", P, Q, bu, bi)
        eng.prepare_strata(n_blocks=B, waves=waves)
        for ep in range(3):
            seq = stratum_order(np.random.RandomState(ep), B, "xcd")
            eng.epoch_strata(seq, 3000 + ep, lr=0.01, reg=0.02, persistent=persistent)
            if persistent and ep == 0:
                # first launch on a freshly zeroed workspace: its tag is 1
                # (base 0 + 1), never the 0 of an unpublished entry
                torch.cuda.synchronize()
                ws = eng._strata_ws.cpu().numpy().view(np.int32)
                assert np.all(ws[B + 1: 2 * B + 1] >> 4 == 1)
        eng.check_strata()
        if persistent:
            torch.cuda.synchronize()
            ws = eng._strata_ws.cpu().numpy().view(np.int32)
            tags = ws[B + 1: 2 * B + 1]
            assert np.all(tags >> 4 == tags[0] >> 4) and tags[0] >> 4 > 0
            assert len(set((tags & 0xF).tolist())) == 8
        out.append(eng.params_numpy())
    for a, b in zip(*out):
        assert np.array_equal(a, b)


def test_contiguous_rows_allocation():
    """P from 16 MiB up lives in hipDeviceMallocContiguous memory wrapped by
    torch (engine._contiguous_empty): torch's storage keeps the block alive
    (its deleter holds a reference beside the tensor attribute), the memory
    reads and writes as a tensor, and the engine's P uses it at C3-like size."""
    import sys

    import torch

    from matrix_factorization.engine import SGDEngine, _contiguous_empty

    t = _contiguous_empty((5000, 1000), torch.float32, torch.device("cuda:0"))
    assert t is not None
    assert sys.getrefcount(t._mf_block) >= 3       # attribute + torch's deleter + argument
    t.fill_(3.0)
    assert float(t.sum()) == 3.0 * 5e6
    nu, k = 70000, 64                               # 17.9 MB of rows
    u = np.arange(1000, dtype=np.int32) % nu
    i = np.arange(1000, dtype=np.int32) % 50
    eng = SGDEngine(u, i, np.ones(1000), nu, 50, k, "linear", "float32", "cuda:0",
                    min_rating=1.0, max_rating=5.0, global_mean=1.0)
    P = np.random.RandomState(0).normal(0, 0.1, (nu, k)).astype(np.float32)
    eng.load_params(P, np.zeros((50, k), np.float32), np.zeros(nu), np.zeros(50))
    assert hasattr(eng.P, "_mf_block")
    assert np.array_equal(eng.P.cpu().numpy(), P)


@pytest.mark.parametrize("dtype,kernel,k,B,C,waves,phases", [
    ("float64", "linear", 64, 4, 2, None, None),
    ("float64", "sigmoid", 32, 3, 3, None, None),
    ("float32", "linear", 64, 16, 4, None, None),
    ("float32", "sigmoid", 32, 8, 2, 8, None),       # 8 waves, rows two steps ahead
    ("float64", "linear", 64, 4, 2, None, 2),        # item phases
    ("float64", "rbf", 16, 5, 2, None, None),
])
def test_user_range_classes(dtype, kernel, k, B, C, waves, phases):
    """C user-range classes (C*B user ranges, C*B strata; the persistent
    kernel waits for the holder C positions back, so every hand-off has C - 1
    blocks of slack): the persistent epoch is bit-identical to one launch per
    stratum, the result is the oracle's sweep in plan.serial_order, and an
    order that does not cycle through the classes runs per stratum (the
    launcher refuses the persistent form) with the same bits as that order's
    per-stratum launches."""
    import oracle
    from matrix_factorization.engine import stratum_order

    nu, ni, nnz = 3000, 900, 120000
    u, i, r = _synthetic(91, nu, ni, nnz)
    rs = np.random.RandomState(92)
    P0 = rs.normal(0, 0.1, (nu, k)); Q0 = rs.normal(0, 0.1, (ni, k))
    bu0 = rs.normal(0, 0.1, nu); bi0 = rs.normal(0, 0.1, ni)
    out = []
    n_ph = phases or 1
    for persistent in (True, False):
        eng = _engine(u, i, r, nu, ni, k, kernel, dtype, P0, Q0, bu0, bi0)
        plan = eng.prepare_strata(n_blocks=B, waves=waves, phases=phases, classes=C)
        assert plan.classes == C and plan.n_strata == C * B
        eps = []
        for ep in range(3):
            seq = stratum_order(np.random.RandomState(ep), plan)
            ms = eng.epoch_strata(seq, 4000 + ep, lr=0.01, reg=0.02, persistent=persistent,
                                  timing=True)
            assert ms[1] == (n_ph if persistent else n_ph * C * B)
            eps.append((seq, 4000 + ep))
        eng.check_strata()
        out.append(eng.params_numpy())
    for a, b in zip(*out):
        assert np.array_equal(a, b)
    hyp = dict(kernel=kernel, gamma=1.0 / k, min_rating=1.0, max_rating=5.0)
    P2, Q2, bu2, bi2 = P0.copy(), Q0.copy(), bu0.copy(), bi0.copy()
    for seq, seed in eps:
        order = eng.serial_order(seq, seed)        # the plan the epoch picked
        assert np.array_equal(np.sort(order), np.arange(nnz))
        oracle.sgd_pass(eng.u_host, eng.i_host, eng.r_host.astype(np.float64), eng.global_mean,
                        bu2, bi2, P2, Q2, lr=0.01, reg=0.02, order=order, **hyp)
    tol = 1e-11 if dtype == "float64" else 1e-4
    for g, o in zip(out[0], (P2, Q2, bu2, bi2)):
        _close(g, o, tol)
    # classes not dealt round-robin (all of class 0 first): per-stratum launches
    bad = np.concatenate([np.arange(c, C * B, C) for c in range(C)]).astype(np.int32)
    res = []
    for persistent in (True, False):
        eng = _engine(u, i, r, nu, ni, k, kernel, dtype, P0, Q0, bu0, bi0)
        eng.prepare_strata(n_blocks=B, waves=waves, phases=phases, classes=C)
        ms = eng.epoch_strata(bad, 7, lr=0.01, reg=0.02, persistent=persistent, timing=True)
        assert ms[1] == n_ph * C * B
        res.append(eng.params_numpy())
    for a, b in zip(*res):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("dtype,phases,K", [("float64", None, 2), ("float32", None, 3),
                                           ("float64", 2, 2)])
def test_regrouped_plans(dtype, phases, K):
    """Relabelled plans (engine.strata_regroup): every epoch's seed picks one
    of K plans of the same B and classes over relabelled users / items; the
    parameters are gathered into its labelling and back, so after each epoch
    they are the oracle's sweep in the picked plan's serial order
    (engine.serial_order), with persistent == per-stratum bits, and the
    auto rule gives the linear kernel's multi-class plans 2."""
    import oracle
    from matrix_factorization.engine import stratum_order

    nu, ni, nnz, k, B, C = 2000, 700, 90000, 32, 5, 4
    u, i, r = _synthetic(93, nu, ni, nnz)
    rs = np.random.RandomState(94)
    P0 = rs.normal(0, 0.1, (nu, k)); Q0 = rs.normal(0, 0.1, (ni, k))
    bu0 = rs.normal(0, 0.1, nu); bi0 = rs.normal(0, 0.1, ni)
    seeds = [5001, 5002, 5003, 5004, 5005, 5006]
    out = []
    for persistent in (True, False):
        eng = _engine(u, i, r, nu, ni, k, "linear", dtype, P0, Q0, bu0, bi0)
        eng.strata_regroup = K
        plan = eng.prepare_strata(n_blocks=B, phases=phases, classes=C)
        assert len(eng._regroups) == K - 1
        picks = {eng._regroup_pick(sd) for sd in seeds}
        assert len(picks) > 1                      # the seeds exercise a regrouping
        eps = []
        for ep, sd in enumerate(seeds):
            seq = stratum_order(np.random.RandomState(ep), plan)
            eng.epoch_strata(seq, sd, lr=0.01, reg=0.02, persistent=persistent)
            eps.append((seq, sd))
        eng.check_strata()
        out.append(eng.params_numpy())
    for a, b in zip(*out):
        assert np.array_equal(a, b)
    P2, Q2, bu2, bi2 = P0.copy(), Q0.copy(), bu0.copy(), bi0.copy()
    for seq, sd in eps:
        order = eng.serial_order(seq, sd)
        assert np.array_equal(np.sort(order), np.arange(nnz))
        oracle.sgd_pass(eng.u_host, eng.i_host, eng.r_host.astype(np.float64), eng.global_mean,
                        bu2, bi2, P2, Q2, lr=0.01, reg=0.02, order=order, kernel="linear",
                        gamma=1.0 / k, min_rating=1.0, max_rating=5.0)
    tol = 1e-11 if dtype == "float64" else 1e-4
    for g, o in zip(out[0], (P2, Q2, bu2, bi2)):
        _close(g, o, tol)
    # the automatic rule: 2 plans for the linear kernel's multi-class plans, 1 otherwise
    e2 = _engine(u, i, r, nu, ni, k, "linear", dtype, P0, Q0, bu0, bi0)
    e2.prepare_strata(n_blocks=B, classes=C)
    assert len(e2._regroups) == 1
    e3 = _engine(u, i, r, nu, ni, k, "linear", dtype, P0, Q0, bu0, bi0)
    e3.prepare_strata(n_blocks=B, classes=1)
    assert len(e3._regroups) == 0
    # the env override sets the count of the engine's plans, not of its
    # regroupings' (which never regroup themselves)
    import os
    os.environ["MF_STRATA_REGROUP"] = "3"
    try:
        e4 = _engine(u, i, r, nu, ni, k, "linear", dtype, P0, Q0, bu0, bi0)
        e4.prepare_strata(n_blocks=B, classes=C)
    finally:
        del os.environ["MF_STRATA_REGROUP"]
    assert len(e4._regroups) == 2 and all(not e._regroups for e, _, _ in e4._regroups)


@pytest.mark.parametrize("dtype,kernel,k,B,C,waves,phases,nu,ni,nnz", [
    ("float64", "linear", 64, 4, 2, None, None, 3000, 900, 120000),
    ("float32", "linear", 64, 16, 4, 8, None, 3000, 900, 120000),
    ("float32", "sigmoid", 32, 8, 2, 8, None, 3000, 900, 120000),
    ("float64", "rbf", 16, 5, 3, None, None, 3000, 900, 120000),
    ("float64", "linear", 64, 4, 2, None, 2, 3000, 900, 120000),   # item phases
    ("float32", "linear", 64, 16, 4, 8, None, 4000, 1500, 3000),   # empty / 1-3 step blocks
    ("float64", "sigmoid", 32, 6, 4, None, None, 5000, 600, 60000),
])
def test_stream_equals_per_stratum_launches(dtype, kernel, k, B, C, waves, phases, nu, ni, nnz,
                                            monkeypatch):
    """The stream form of the multi-class persistent sweep (MF_FLAG_STREAM:
    one software pipeline through every position of the launch, the next
    block's triples and rows loaded while the current block's last steps
    apply, the bias slices double-buffered) applies the same sequential order:
    bit-identical to one launch per stratum over 3 epochs, and the oracle's
    sweep in plan.serial_order -- blocks of every length, empty ones and ones
    shorter than the 4-step lookahead included."""
    import oracle
    from matrix_factorization.engine import stratum_order

    monkeypatch.setenv("MF_STRATA_DEEP", "1")
    u, i, r = _synthetic(95, nu, ni, nnz)
    rs = np.random.RandomState(96)
    P0 = rs.normal(0, 0.1, (nu, k)); Q0 = rs.normal(0, 0.1, (ni, k))
    bu0 = rs.normal(0, 0.1, nu); bi0 = rs.normal(0, 0.1, ni)
    out = []
    n_ph = phases or 1
    for stream in (True, False):
        monkeypatch.setenv("MF_STRATA_STREAM", "1" if stream else "0")
        eng = _engine(u, i, r, nu, ni, k, kernel, dtype, P0, Q0, bu0, bi0)
        eng.strata_regroup = 1
        plan = eng.prepare_strata(n_blocks=B, waves=waves, phases=phases, classes=C)
        eps = []
        for ep in range(3):
            seq = stratum_order(np.random.RandomState(ep), plan)
            ms = eng.epoch_strata(seq, 6000 + ep, lr=0.01, reg=0.02, persistent=stream,
                                  timing=True)
            assert ms[1] == (n_ph if stream else n_ph * C * B)
            eps.append((seq, 6000 + ep))
        eng.check_strata()
        out.append(eng.params_numpy())
    if nnz < 10000:
        steps = np.diff(plan.bstep) if hasattr(plan, "bstep") else None
        assert steps is None or (steps.min() == 0 and (steps < 4).mean() > 0.5)
    for a, b in zip(*out):
        assert np.array_equal(a, b)
    hyp = dict(kernel=kernel, gamma=1.0 / k, min_rating=1.0, max_rating=5.0)
    P2, Q2, bu2, bi2 = P0.copy(), Q0.copy(), bu0.copy(), bi0.copy()
    for seq, seed in eps:
        order = eng.serial_order(seq, seed)
        oracle.sgd_pass(eng.u_host, eng.i_host, eng.r_host.astype(np.float64), eng.global_mean,
                        bu2, bi2, P2, Q2, lr=0.01, reg=0.02, order=order, **hyp)
    tol = 1e-11 if dtype == "float64" else 1e-4
    for g, o in zip(out[0], (P2, Q2, bu2, bi2)):
        _close(g, o, tol)

"""GPU parity of the factor ALS (mf_als_sweep, ALSMF) against the FP64 oracle
restatement (oracle.als_half_sweep, pinned in tests/test_als_oracle.py).

The GPU forms the Gramian in f32 on MFMA and eliminates in f32; the oracle
solves in f64 from the same f32-rounded inputs.  Bars (stated per test):
  parameters   max |diff| <= 2e-4 * max(1, |value|)   (f32 solve of systems
               with condition numbers up to ~1e3 here)
  train RMSE   |diff| <= 1e-5                          (the north-star bar)
"""

import numpy as np
import pandas as pd
import pytest

pytestmark = pytest.mark.gpu


def _data(seed, nu, ni, nnz, heavy=()):
    rs = np.random.RandomState(seed)
    keys = set(rs.choice(nu * ni, nnz, replace=False).tolist())
    for user, deg in heavy:                    # users with several LDS chunks
        keys.update((user * ni + rs.choice(ni, deg, replace=False)).tolist())
    keys = np.array(sorted(keys))
    rs.shuffle(keys)
    u = (keys // ni).astype(np.int32)
    i = (keys % ni).astype(np.int32)
    r = rs.randint(1, 6, len(keys)).astype(np.float64)
    return u, i, r


def _close(a, b, tol):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    err = np.max(np.abs(a - b) / np.maximum(1.0, np.abs(b)))
    assert err <= tol, f"max rel diff {err:.3e} > {tol:.0e}"
    return err


@pytest.mark.parametrize("k", [8, 20, 32, 64, 100, 128])
def test_half_sweeps_match_oracle(k):
    import oracle
    from matrix_factorization.engine import FactorALS, SGDEngine

    nu, ni = 400, 260
    u, i, r = _data(k, nu - 1, ni, 14000, heavy=[(0, 250), (3, 130), (7, 65)])
    # user nu-1 has no ratings: its parameters must be left as they are
    rs = np.random.RandomState(100 + k)
    P = rs.normal(0, 0.3, (nu, k)).astype(np.float32)
    Q = rs.normal(0, 0.3, (ni, k)).astype(np.float32)
    bu = rs.normal(0, 0.1, nu).astype(np.float32)
    bi = rs.normal(0, 0.1, ni).astype(np.float32)
    mu, reg = float(r.mean()), 0.1
    eng = SGDEngine(u, i, r, nu, ni, k, "linear", "float32", "cuda:0", global_mean=mu,
                    min_rating=1, max_rating=5)
    eng.load_params(P, Q, bu, bi)
    als = FactorALS(eng)
    als.sweep_users(reg)
    Pg, Qg, bug, big = eng.params_numpy()
    bu_o, P_o = oracle.als_half_sweep(u, i, r, np.float32(mu), bi, Q, nu, reg)
    assert np.array_equal(Pg[nu - 1], P[nu - 1].astype(np.float64))
    assert bug[nu - 1] == np.float64(bu[nu - 1])
    _close(Pg[: nu - 1], P_o[: nu - 1], 2e-4)
    _close(bug[: nu - 1], bu_o[: nu - 1], 2e-4)
    assert np.array_equal(Qg, Q.astype(np.float64))          # item side untouched
    # item half-sweep from the GPU's user side
    als.sweep_items(reg)
    _, Qg2, _, big2 = eng.params_numpy()
    bi_o, Q_o = oracle.als_half_sweep(i, u, r, np.float32(mu), bug, Pg, ni, reg)
    _close(Qg2, Q_o, 2e-4)
    _close(big2, bi_o, 2e-4)


def test_alsmf_fit_matches_oracle():
    import oracle
    from matrix_factorization import ALSMF

    u, i, r = _data(5, 500, 300, 20000)
    X = pd.DataFrame({"user_id": u, "item_id": i})
    hp = dict(n_factors=48, n_epochs=4, reg=0.05, min_rating=1, max_rating=5, verbose=0)
    np.random.seed(9)
    m = ALSMF(**hp).fit(X, pd.Series(r))
    # oracle: same preprocessing / RNG order as KernelMF.fit
    np.random.seed(9)
    Xp, uids, iids = oracle.preprocess_fit(X, pd.Series(r))
    mu = Xp["rating"].mean()
    P0 = np.random.normal(0, 0.1, (len(uids), 48)).astype(np.float32)
    Q0 = np.random.normal(0, 0.1, (len(iids), 48)).astype(np.float32)
    arr = Xp.to_numpy(np.float64)
    uu, ii, rr = arr[:, 0].astype(np.int32), arr[:, 1].astype(np.int32), arr[:, 2]
    bu, bi = np.zeros(len(uids)), np.zeros(len(iids))
    P, Q = P0.astype(np.float64), Q0.astype(np.float64)
    rm = []
    for _ in range(4):
        bu, bi, P, Q = oracle.als_epoch(uu, ii, rr, np.float32(mu), bu, bi, P, Q, 0.05)
        rm.append(oracle.linear_rmse(uu, ii, rr, mu, bu, bi, P, Q))
    assert np.max(np.abs(np.array(m.train_rmse) - np.array(rm))) < 1e-5
    assert all(b < a for a, b in zip(m.train_rmse, m.train_rmse[1:]))
    pred = np.asarray(m.predict(X.iloc[:200], bound_ratings=False))
    ui = np.array([m.user_id_map[x] for x in X["user_id"].iloc[:200]])
    ij = np.array([m.item_id_map[x] for x in X["item_id"].iloc[:200]])
    po = ((mu + bi[ij]) + bu[ui]) + np.einsum("nk,nk->n", P[ui], Q[ij])
    assert np.max(np.abs(pred - po)) < 1e-3


def test_alsmf_update_users_keeps_absent_users():
    from matrix_factorization import ALSMF

    u, i, r = _data(6, 300, 200, 9000)
    X = pd.DataFrame({"user_id": u, "item_id": i})
    np.random.seed(1)
    m = ALSMF(n_factors=16, n_epochs=2, reg=0.1, verbose=0).fit(X, pd.Series(r))
    Q, bi = m.item_features.copy(), m.item_biases.copy()
    P = m.user_features.copy()
    sel = X["user_id"].isin([3, 4])
    Xn = X[sel].copy()
    Xn.loc[Xn["user_id"] == 4, "user_id"] = 10_000          # a new user
    m.update_users(Xn, pd.Series(r[sel.to_numpy()], index=Xn.index), n_epochs=1)
    assert np.array_equal(m.item_features, Q) and np.array_equal(m.item_biases, bi)
    others = [m.user_id_map[x] for x in m.user_id_map if x not in (3, 10_000)]
    assert np.array_equal(m.user_features[others], P[others])
    assert m.user_features.shape[0] == P.shape[0] + 1
    for user in (3, 10_000):
        assert np.all(np.isfinite(m.user_features[m.user_id_map[user]]))

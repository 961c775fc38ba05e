"""The factor-ALS restatement (oracle.als_half_sweep / als_epoch), CPU only.

BASELINE config 5 has no reference counterpart.  The restatement extends the
reference's bias ALS (baseline_model.py:283-362) to the latent factors, so
it is pinned two ways:
  * with n_factors = 0 it must reproduce the reference's BaselineModel ALS
    fixture (tests/golden/baseline_als.npz, generated from the reference's
    own source) -- same update, same order, same RMSE;
  * with n_factors > 0 every half-sweep must be the exact minimiser of the
    regularised least-squares objective it states (zero gradient, and no
    perturbation lowers the objective).
"""

import numpy as np
import pandas as pd

import oracle
from conftest import golden_hp, load_golden


def test_k0_is_the_reference_bias_als():
    d = load_golden("baseline_als")
    hp = golden_hp(d)
    X = pd.DataFrame({"user_id": d["user_id"], "item_id": d["item_id"]})
    np.random.seed(int(d["seed"]))
    Xp, uids, iids = oracle.preprocess_fit(X, pd.Series(d["rating"]))
    mu = Xp["rating"].mean()
    arr = Xp.to_numpy(np.float64)
    u, i, r = arr[:, 0].astype(np.int32), arr[:, 1].astype(np.int32), arr[:, 2].copy()
    bu, bi = np.zeros(len(uids)), np.zeros(len(iids))
    P, Q = np.zeros((len(uids), 0)), np.zeros((len(iids), 0))
    rm = []
    for _ in range(hp["n_epochs"]):
        bu, bi, P, Q = oracle.als_epoch(u, i, r, mu, bu, bi, P, Q, hp["reg"])
        rm.append(oracle.linear_rmse(u, i, r, mu, bu, bi, P, Q))
    # summation order (BLAS vs sequential) is the only difference
    assert np.max(np.abs(bu - d["user_biases"])) < 1e-12
    assert np.max(np.abs(bi - d["item_biases"])) < 1e-12
    assert np.max(np.abs(np.array(rm) - d["train_rmse"])) < 1e-12


def _objective(x, Y, t, reg):
    res = t - Y @ x
    return float(res @ res + reg * (x @ x))


def test_half_sweep_is_the_regularised_least_squares_minimiser():
    rs = np.random.RandomState(3)
    nu, ni, n, k, reg = 60, 40, 900, 12, 0.3
    keys = rs.choice(nu * ni, n, replace=False)
    u, i = (keys // ni).astype(np.int32), (keys % ni).astype(np.int32)
    r = rs.randint(1, 6, n).astype(np.float64)
    mu = r.mean()
    bi = rs.normal(0, 0.2, ni)
    Q = rs.normal(0, 0.3, (ni, k))
    bu, P = oracle.als_half_sweep(u, i, r, mu, bi, Q, nu, reg)
    for e in range(nu):
        m = u == e
        Y = np.hstack([Q[i[m]], np.ones((m.sum(), 1))])
        t = (r[m] - mu) - bi[i[m]]
        x = np.concatenate([P[e], [bu[e]]])
        grad = -2 * Y.T @ (t - Y @ x) + 2 * reg * x
        assert np.max(np.abs(grad)) < 1e-9
        f0 = _objective(x, Y, t, reg)
        for _ in range(3):
            assert _objective(x + 1e-3 * rs.normal(size=k + 1), Y, t, reg) > f0


def test_als_epochs_lower_the_training_error():
    rs = np.random.RandomState(4)
    nu, ni, n, k, reg = 80, 50, 1500, 8, 0.5
    keys = rs.choice(nu * ni, n, replace=False)
    u, i = (keys // ni).astype(np.int32), (keys % ni).astype(np.int32)
    r = rs.randint(1, 6, n).astype(np.float64)
    mu = r.mean()
    bu, bi = np.zeros(nu), np.zeros(ni)
    P, Q = rs.normal(0, 0.1, (nu, k)), rs.normal(0, 0.1, (ni, k))
    rm = [oracle.linear_rmse(u, i, r, mu, bu, bi, P, Q)]
    for _ in range(4):
        bu, bi, P, Q = oracle.als_epoch(u, i, r, mu, bu, bi, P, Q, reg)
        rm.append(oracle.linear_rmse(u, i, r, mu, bu, bi, P, Q))
    assert all(b < a for a, b in zip(rm, rm[1:]))

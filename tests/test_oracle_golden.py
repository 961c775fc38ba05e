"""The CPU oracle is pinned against the reference's own outputs.

tests/golden/*.npz were produced by running the reference source
(tests/golden/make_golden.py).  The oracle restates the algorithm in C/FP64;
differences come only from dot-product summation order (BLAS ddot vs
sequential), i.e. ULP-level.
"""

import numpy as np
import pandas as pd
import pytest

import oracle
from conftest import golden_hp, load_golden

CASES = ["tiny_linear", "tiny_sigmoid", "tiny_rbf", "tiny_defaults", "mid_k100",
         "mid_sigmoid_k32", "c1_linear"]


def _rel(a, b):
    return float(np.max(np.abs(a - b)) / max(1.0, np.max(np.abs(b))))


@pytest.mark.parametrize("name", CASES)
def test_oracle_fit_matches_reference(name):
    d = load_golden(name)
    hp = golden_hp(d)
    hp.pop("verbose", None)
    X = pd.DataFrame({"user_id": d["user_id"], "item_id": d["item_id"]})
    np.random.seed(int(d["seed"]))
    o = oracle.oracle_kernel_fit(X, pd.Series(d["rating"]), **hp)
    assert (o["user_ids"] == d["user_ids"]).all()
    assert (o["item_ids"] == d["item_ids"]).all()
    assert o["global_mean"] == d["global_mean"]
    for key in ("user_features", "item_features", "user_biases", "item_biases"):
        assert _rel(o[key], d[key]) < 1e-13, key
    assert np.max(np.abs(o["train_rmse"] - d["train_rmse"])) < 1e-13
    # predictions on the reference's test pairs
    uidx = pd.Index(o["user_ids"]).get_indexer(d["test_user"])
    iidx = pd.Index(o["item_ids"]).get_indexer(d["test_item"])
    kw = dict(kernel=hp.get("kernel", "linear"), gamma=o["gamma"],
              min_rating=hp.get("min_rating", 0), max_rating=hp.get("max_rating", 5))
    pb = oracle.predict(uidx, iidx, o["global_mean"], o["user_biases"], o["item_biases"],
                        o["user_features"], o["item_features"], bound=True, **kw)
    pu = oracle.predict(uidx, iidx, o["global_mean"], o["user_biases"], o["item_biases"],
                        o["user_features"], o["item_features"], bound=False, **kw)
    assert _rel(pb, d["pred_bound"]) < 1e-13
    assert _rel(pu, d["pred_unbound"]) < 1e-13


@pytest.mark.parametrize("method", ["sgd", "als"])
def test_oracle_bias_model_matches_reference(method):
    d = load_golden(f"baseline_{method}")
    hp = golden_hp(d)
    X = pd.DataFrame({"user_id": d["user_id"], "item_id": d["item_id"]})
    np.random.seed(int(d["seed"]))
    Xp, uids, iids = oracle.preprocess_fit(X, pd.Series(d["rating"]))
    mu = Xp["rating"].mean()
    arr = Xp.to_numpy(np.float64)
    u, i, r = arr[:, 0].astype(np.int32), arr[:, 1].astype(np.int32), arr[:, 2].copy()
    bu, bi = np.zeros(len(uids)), np.zeros(len(iids))
    rm = []
    if method == "sgd":
        order = np.arange(len(u), dtype=np.int64)
        for _ in range(hp["n_epochs"]):
            np.random.shuffle(order)
            oracle.bias_sgd_pass(u, i, r, mu, bu, bi, hp["lr"], hp["reg"], order=order)
            rm.append(np.sqrt(oracle.bias_sse(u, i, r, mu, bu, bi) / len(u)))
    else:
        uc = np.bincount(u, minlength=len(uids)).astype(np.float64)
        ic = np.bincount(i, minlength=len(iids)).astype(np.float64)
        for _ in range(hp["n_epochs"]):
            oracle.bias_als_epoch(u, i, r, mu, bu, bi, uc, ic, hp["reg"])
            rm.append(np.sqrt(oracle.bias_sse(u, i, r, mu, bu, bi) / len(u)))
    # no dot product: bit-identical
    assert np.array_equal(bu, d["user_biases"])
    assert np.array_equal(bi, d["item_biases"])
    assert np.max(np.abs(np.array(rm) - d["train_rmse"])) < 1e-14


def test_golden_fixture_inventory():
    """Fixtures cover every kernel, the update path and both bias methods."""
    kernels = set()
    for name in CASES:
        kernels.add(golden_hp(load_golden(name)).get("kernel", "linear"))
    assert kernels == {"linear", "sigmoid", "rbf"}
    for name in ("update_users", "baseline_sgd", "baseline_als"):
        assert load_golden(name)["user_biases"].size > 0

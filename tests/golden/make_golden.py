"""Generate golden vectors from the REFERENCE implementation (this container only).

Run:  python tests/golden/make_golden.py  [--only NAME]

The reference (SHEEPididoo/matrix-factorization, mounted read-only at
/root/reference) is numba-JIT code.  numba is not importable in this image
(system Python has no numba; /opt/conda's numba 0.54.1 fails to initialise
against its numpy), so the reference is executed as plain Python: a throw-away
``numba`` module whose ``njit`` is the identity decorator is written to a
temporary directory that is put on sys.path ahead of /root/reference.  No
reference source is copied, modified or committed; only the input/output
vectors below are.

Semantic deltas of the pure-Python reference vs numba:
  * the per-epoch ``np.random.shuffle`` draws from NumPy's global legacy
    RandomState (numba would use its own os.urandom-seeded MT state) -- this
    is what makes the fixtures reproducible;
  * ``np.dot`` / ``np.sum`` summation order is NumPy's (BLAS ddot / pairwise),
    so parity against these vectors is stated with an FP64 tolerance.

Each fixture stores the external-id inputs, the seed and hyper-parameters, and
the reference outputs (features, biases, train_rmse, id maps, predictions,
recommend() top lists).  The generator never runs on the GPU box.
"""

from __future__ import annotations

import argparse
import contextlib
import io
import os
import sys
import tempfile
import warnings

import numpy as np
import pandas as pd

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"


def _import_reference():
    shim = tempfile.mkdtemp(prefix="nbshim_")
    os.makedirs(os.path.join(shim, "numba"))
    with open(os.path.join(shim, "numba", "__init__.py"), "w") as f:
        f.write(
            "def njit(*a, **k):\n"
            "    if a and callable(a[0]) and not k:\n"
            "        return a[0]\n"
            "    return lambda f: f\n"
        )
    sys.path[:0] = [shim, REF]
    import matrix_factorization as ref  # noqa: E402  (the reference package)

    assert os.path.realpath(ref.__file__).startswith(REF), ref.__file__
    return ref


# ----------------------------------------------------------------- data
def synth_ratings(seed, n_users, n_items, nnz, rank=4, user_base=1,
                  item_base=1):
    """Unique (user,item) pairs with a low-rank signal, ratings 1..5."""
    rs = np.random.RandomState(seed)
    keys = np.empty(0, np.int64)
    while len(keys) < nnz:
        need = nnz - len(keys)
        uu = rs.randint(0, n_users, size=2 * need)
        ii = rs.randint(0, n_items, size=2 * need)
        cand = uu.astype(np.int64) * n_items + ii
        keys = np.concatenate([keys, cand])
        _, first = np.unique(keys, return_index=True)
        keys = keys[np.sort(first)][:nnz]
    u = (keys // n_items).astype(np.int64)
    i = (keys % n_items).astype(np.int64)
    U = rs.normal(0, 0.6, (n_users, rank))
    V = rs.normal(0, 0.6, (n_items, rank))
    raw = 3.5 + (U[u] * V[i]).sum(1) + rs.normal(0, 0.7, nnz)
    r = np.clip(np.rint(raw), 1, 5).astype(np.float64)
    return pd.DataFrame({"user_id": u + user_base, "item_id": i + item_base,
                         "rating": r})


def _test_pairs(df, seed, n, n_unknown_users=3, n_unknown_items=3):
    rs = np.random.RandomState(seed)
    users = df["user_id"].unique()
    items = df["item_id"].unique()
    tu = rs.choice(users, n)
    ti = rs.choice(items, n)
    tu[:n_unknown_users] = -999 - np.arange(n_unknown_users)     # unknown users
    ti[n_unknown_users:n_unknown_users + n_unknown_items] = -777  # unknown items
    return pd.DataFrame({"user_id": tu, "item_id": ti})


# ----------------------------------------------------------------- cases
def kernel_case(ref, name, df, seed, hp, n_test=200, rec_users=(), out=None):
    X = df[["user_id", "item_id"]]
    y = df["rating"]
    np.random.seed(seed)
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        m = ref.KernelMF(**hp).fit(X, y)
    T = _test_pairs(df, seed + 1, n_test)
    pb = np.asarray(m.predict(T, bound_ratings=True), np.float64)
    poss = np.asarray(m.predictions_possible, bool)
    pu = np.asarray(m.predict(T, bound_ratings=False), np.float64)
    recs_items, recs_pred = [], []
    for j, user in enumerate(rec_users):
        known = df.loc[df.user_id == user, "item_id"].to_numpy()
        known = known[: len(known) // 2] if j % 2 == 0 else None
        rec = m.recommend(user=user, amount=10, items_known=known)
        recs_items.append(rec["item_id"].to_numpy(np.int64))
        recs_pred.append(rec["rating_pred"].to_numpy(np.float64))
    d = dict(
        user_id=df["user_id"].to_numpy(np.int64),
        item_id=df["item_id"].to_numpy(np.int64),
        rating=df["rating"].to_numpy(np.float64),
        seed=np.int64(seed),
        hp_json=np.array(repr(hp)),
        user_ids=np.asarray(list(m.user_id_map.keys()), np.int64),
        item_ids=np.asarray(list(m.item_id_map.keys()), np.int64),
        global_mean=np.float64(m.global_mean),
        user_biases=np.array(m.user_biases, np.float64, copy=True),
        item_biases=np.array(m.item_biases, np.float64, copy=True),
        user_features=np.array(m.user_features, np.float64, copy=True),
        item_features=np.array(m.item_features, np.float64, copy=True),
        train_rmse=np.asarray(m.train_rmse, np.float64),
        gamma=np.float64(m.gamma),
        test_user=T["user_id"].to_numpy(np.int64),
        test_item=T["item_id"].to_numpy(np.int64),
        pred_bound=pb,
        pred_unbound=pu,
        pred_possible=poss,
        rec_users=np.asarray(rec_users, np.int64),
        rec_items=np.asarray(recs_items, np.int64).reshape(len(rec_users), -1),
        rec_pred=np.asarray(recs_pred, np.float64).reshape(len(rec_users), -1),
        stdout=np.array(buf.getvalue()),
    )
    if out is not None:
        out.update(d)
    return m, d


def case_update(ref, name):
    """fit -> update_users (kernel_matrix_factorization.py:165-237)."""
    df = synth_ratings(11, 60, 45, 900)
    seed = 5
    np.random.seed(seed)
    (Xi, yi, Xu, yu, Xt, yt) = ref.train_update_test_split(df, frac_new_users=0.25)
    hp = dict(n_factors=6, n_epochs=4, lr=0.02, reg=0.05, min_rating=1,
              max_rating=5, verbose=0)
    m = ref.KernelMF(**hp).fit(Xi, yi)
    P_fit = np.asarray(m.user_features).copy()
    Q_fit = np.asarray(m.item_features).copy()
    # also re-submit some ratings of a known user to exercise known_users
    known_user = Xi["user_id"].iloc[0]
    extra = Xi[Xi.user_id == known_user].iloc[:3]
    Xu2 = pd.concat([Xu, extra])
    yu2 = pd.concat([yu, yi.loc[extra.index]])
    m.update_users(Xu2, yu2, lr=0.03, n_epochs=5, verbose=0)
    pred = np.asarray(m.predict(Xt), np.float64)
    return dict(
        user_id=df["user_id"].to_numpy(np.int64),
        item_id=df["item_id"].to_numpy(np.int64),
        rating=df["rating"].to_numpy(np.float64),
        seed=np.int64(seed), hp_json=np.array(repr(hp)),
        split_train_index=Xi.index.to_numpy(np.int64),
        split_update_index=Xu.index.to_numpy(np.int64),
        split_test_index=Xt.index.to_numpy(np.int64),
        known_user=np.int64(known_user),
        extra_index=extra.index.to_numpy(np.int64),
        fit_user_features=P_fit, fit_item_features=Q_fit,
        user_ids=np.asarray(list(m.user_id_map.keys()), np.int64),
        user_id_vals=np.asarray(list(m.user_id_map.values()), np.int64),
        item_ids=np.asarray(list(m.item_id_map.keys()), np.int64),
        n_users=np.int64(m.n_users),
        global_mean=np.float64(m.global_mean),
        user_biases=np.array(m.user_biases, np.float64, copy=True),
        item_biases=np.array(m.item_biases, np.float64, copy=True),
        user_features=np.array(m.user_features, np.float64, copy=True),
        item_features=np.array(m.item_features, np.float64, copy=True),
        train_rmse=np.asarray(m.train_rmse, np.float64),
        pred_test=pred,
    )


def case_baseline(ref, method):
    df = synth_ratings(21, 40, 30, 500)
    seed = 9
    np.random.seed(seed)
    hp = dict(method=method, n_epochs=6, lr=0.02, reg=0.1 if method == "sgd"
              else 2.0, min_rating=1, max_rating=5, verbose=0)
    m = ref.BaselineModel(**hp).fit(df[["user_id", "item_id"]], df["rating"])
    T = _test_pairs(df, 99, 100)
    pred = np.asarray(m.predict(T), np.float64)
    poss = np.asarray(m.predictions_possible, bool)
    out = dict(
        user_id=df["user_id"].to_numpy(np.int64),
        item_id=df["item_id"].to_numpy(np.int64),
        rating=df["rating"].to_numpy(np.float64),
        seed=np.int64(seed), hp_json=np.array(repr(hp)),
        user_ids=np.asarray(list(m.user_id_map.keys()), np.int64),
        item_ids=np.asarray(list(m.item_id_map.keys()), np.int64),
        global_mean=np.float64(m.global_mean),
        user_biases=np.array(m.user_biases, np.float64, copy=True),
        item_biases=np.array(m.item_biases, np.float64, copy=True),
        train_rmse=np.asarray(m.train_rmse, np.float64),
        test_user=T["user_id"].to_numpy(np.int64),
        test_item=T["item_id"].to_numpy(np.int64),
        pred=pred, pred_possible=poss,
    )
    if method == "sgd":
        # update_users for the bias model (baseline_model.py:136-180)
        Xn = pd.DataFrame({"user_id": [1000, 1000, 1001, 1],
                           "item_id": df["item_id"].unique()[:4]})
        yn = pd.Series([5.0, 4.0, 1.0, 3.0])
        np.random.seed(seed + 1)
        m.update_users(Xn, yn, lr=0.05, n_epochs=3)
        out.update(upd_user=Xn["user_id"].to_numpy(np.int64),
                   upd_item=Xn["item_id"].to_numpy(np.int64),
                   upd_rating=yn.to_numpy(np.float64),
                   upd_user_biases=np.array(m.user_biases, np.float64, copy=True),
                   upd_train_rmse=np.asarray(m.train_rmse, np.float64))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default=None)
    args = ap.parse_args()
    warnings.simplefilter("ignore", FutureWarning)
    ref = _import_reference()
    want = lambda n: args.only in (None, n)  # noqa: E731

    small = synth_ratings(1, 50, 40, 600)
    cases = {}
    if want("tiny_linear"):
        _, cases["tiny_linear"] = kernel_case(
            ref, "tiny_linear", small, 3,
            dict(n_factors=8, n_epochs=5, kernel="linear", lr=0.01, reg=0.02,
                 min_rating=1, max_rating=5, verbose=1),
            rec_users=(1, 2, 17))
    if want("tiny_sigmoid"):
        _, cases["tiny_sigmoid"] = kernel_case(
            ref, "tiny_sigmoid", small, 4,
            dict(n_factors=8, n_epochs=5, kernel="sigmoid", lr=0.05, reg=0.02,
                 min_rating=1, max_rating=5, verbose=0),
            rec_users=(1, 5))
    if want("tiny_rbf"):
        _, cases["tiny_rbf"] = kernel_case(
            ref, "tiny_rbf", small, 5,
            dict(n_factors=8, n_epochs=5, kernel="rbf", lr=0.5, reg=0.02,
                 min_rating=1, max_rating=5, verbose=0),
            rec_users=(3,))
    if want("tiny_defaults"):
        # reference defaults: reg=1, min_rating=0, max_rating=5, k odd
        _, cases["tiny_defaults"] = kernel_case(
            ref, "tiny_defaults", small, 6,
            dict(n_factors=5, n_epochs=3, verbose=0), rec_users=(7,))
    if want("mid_k100"):
        df = synth_ratings(2, 120, 90, 2500)
        _, cases["mid_k100"] = kernel_case(
            ref, "mid_k100", df, 8,
            dict(n_factors=100, n_epochs=2, kernel="linear", lr=0.001,
                 reg=0.005, min_rating=1, max_rating=5, verbose=0),
            rec_users=(1, 2))
    if want("mid_sigmoid_k32"):
        df = synth_ratings(3, 400, 300, 12000)
        _, cases["mid_sigmoid_k32"] = kernel_case(
            ref, "mid_sigmoid_k32", df, 12,
            dict(n_factors=32, n_epochs=2, kernel="sigmoid", lr=0.01,
                 reg=0.02, min_rating=1, max_rating=5, verbose=0),
            rec_users=(1,))
    if want("c1_linear"):
        df = synth_ratings(20261015, 943, 1682, 80000)
        _, cases["c1_linear"] = kernel_case(
            ref, "c1_linear", df, 7,
            dict(n_factors=16, n_epochs=20, kernel="linear", lr=0.01,
                 reg=0.02, min_rating=1, max_rating=5, verbose=0),
            n_test=2000, rec_users=(1, 100, 200, 943))
    if want("update_users"):
        cases["update_users"] = case_update(ref, "update_users")
    if want("baseline_sgd"):
        cases["baseline_sgd"] = case_baseline(ref, "sgd")
    if want("baseline_als"):
        cases["baseline_als"] = case_baseline(ref, "als")

    for name, d in cases.items():
        path = os.path.join(HERE, f"{name}.npz")
        np.savez_compressed(path, **d)
        print(f"wrote {path} ({os.path.getsize(path)} B)")


if __name__ == "__main__":
    main()

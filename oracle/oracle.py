"""CPU oracle for the KernelMF SGD path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of
``bench.py`` may import this module, and only as the checker or as the
reported CPU baseline.  The product package never imports it.

It is a restatement of the reference algorithm:

* ``libmf_oracle.so`` (``mf_oracle.c``): the numba epoch bodies of
  ``kernel_matrix_factorization.py:240-541`` / ``kernels.py:1-327`` and
  ``baseline_model.py:183-362`` in FP64, sequential, reference operation order.
* ``preprocess_fit`` / ``oracle_kernel_fit``: the host side of
  ``KernelMF.fit`` (``kernel_matrix_factorization.py:81-128``) and
  ``RecommenderBase._preprocess_data`` (``recommender_base.py:97-173``),
  drawing from NumPy's legacy global RandomState in the reference's order:
  ``X.sample(frac=1)`` -> ``normal(P)`` -> ``normal(Q)`` -> per-epoch
  ``np.random.shuffle``.

Pinned against tests/golden/*.npz, which were generated from the reference's
own source (see tests/golden/make_golden.py and DESIGN.md section 3).
"""

from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np
import pandas as pd

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "_build", "libmf_oracle.so")

KERNELS = {"linear": 0, "sigmoid": 1, "rbf": 2}

_lib = None


def build() -> str:
    """Compile libmf_oracle.so with gcc (no-op when up to date)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _SO


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(_SO) or os.path.getmtime(_SO) < os.path.getmtime(
            os.path.join(_HERE, "mf_oracle.c")
        ):
            build()
        L = ctypes.CDLL(_SO)
        P = ctypes.c_void_p
        i32, i64, f64 = ctypes.c_int32, ctypes.c_int64, ctypes.c_double
        L.oracle_sgd_pass.argtypes = [P, P, P, i64, P, f64, P, P, P, P, i32,
                                      i32, f64, f64, f64, f64, f64, i32, i32]
        L.oracle_sgd_pass.restype = ctypes.c_int
        L.oracle_sse.argtypes = [P, P, P, i64, f64, P, P, P, P, i32, i32,
                                 f64, f64, f64]
        L.oracle_sse.restype = f64
        L.oracle_predict.argtypes = [P, P, i64, f64, P, P, P, P, i32, i32, f64,
                                     f64, f64, i32, P, P]
        L.oracle_predict.restype = None
        L.oracle_bias_sgd_pass.argtypes = [P, P, P, i64, P, f64, P, P, f64,
                                           f64, i32, i32]
        L.oracle_bias_sgd_pass.restype = ctypes.c_int
        L.oracle_bias_sse.argtypes = [P, P, P, i64, f64, P, P]
        L.oracle_bias_sse.restype = f64
        L.oracle_bias_als_epoch.argtypes = [P, P, P, i64, f64, P, P, P, P, i32,
                                            i32, f64]
        L.oracle_bias_als_epoch.restype = ctypes.c_int
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _c(a, dt):
    a = np.ascontiguousarray(a, dtype=dt)
    return a


# ---------------------------------------------------------------- passes
def sgd_pass(u, i, r, mu, bu, bi, P, Q, kernel="linear", gamma=0.0, lr=0.01,
             reg=0.02, min_rating=0.0, max_rating=5.0, order=None,
             update_user=True, update_item=True):
    """One sequential sweep over ``order`` (rating indices; default all
    ratings in row order); mutates bu, bi, P, Q (float64, C-contiguous)."""
    for a in (bu, bi, P, Q):
        assert a.dtype == np.float64 and a.flags.c_contiguous
    u = _c(u, np.int32); i = _c(i, np.int32); r = _c(r, np.float64)
    order = None if order is None else _c(order, np.int64)
    k = P.shape[1] if P.ndim == 2 else 0
    steps = len(u) if order is None else len(order)
    lib().oracle_sgd_pass(_p(u), _p(i), _p(r), steps, _p(order), float(mu),
                          _p(bu), _p(bi), _p(P), _p(Q), k, KERNELS[kernel],
                          float(gamma), float(lr), float(reg),
                          float(min_rating), float(max_rating - min_rating),
                          int(update_user), int(update_item))


def sse(u, i, r, mu, bu, bi, P, Q, kernel="linear", gamma=0.0, min_rating=0.0,
        max_rating=5.0) -> float:
    u = _c(u, np.int32); i = _c(i, np.int32); r = _c(r, np.float64)
    k = P.shape[1]
    return lib().oracle_sse(_p(u), _p(i), _p(r), len(u), float(mu), _p(bu),
                            _p(bi), _p(P), _p(Q), k, KERNELS[kernel],
                            float(gamma), float(min_rating),
                            float(max_rating - min_rating))


def rmse(*args, **kw) -> float:
    n = len(args[0])
    return float(np.sqrt(sse(*args, **kw) / n)) if n else float("nan")


def predict(u, i, mu, bu, bi, P, Q, kernel="linear", gamma=0.0,
            min_rating=0.0, max_rating=5.0, bound=True) -> np.ndarray:
    u = _c(u, np.int32); i = _c(i, np.int32)
    k = P.shape[1]
    out = np.empty(len(u), np.float64)
    zeros = np.zeros(max(k, 1), np.float64)
    lib().oracle_predict(_p(u), _p(i), len(u), float(mu), _p(bu), _p(bi),
                         _p(P), _p(Q), k, KERNELS[kernel], float(gamma),
                         float(min_rating), float(max_rating), int(bound),
                         _p(out), _p(zeros))
    return out


def bias_sgd_pass(u, i, r, mu, bu, bi, lr, reg, order=None, update_user=True,
                  update_item=True):
    u = _c(u, np.int32); i = _c(i, np.int32); r = _c(r, np.float64)
    order = None if order is None else _c(order, np.int64)
    steps = len(u) if order is None else len(order)
    lib().oracle_bias_sgd_pass(_p(u), _p(i), _p(r), steps, _p(order),
                               float(mu), _p(bu), _p(bi), float(lr),
                               float(reg), int(update_user), int(update_item))


def bias_sse(u, i, r, mu, bu, bi) -> float:
    u = _c(u, np.int32); i = _c(i, np.int32); r = _c(r, np.float64)
    return lib().oracle_bias_sse(_p(u), _p(i), _p(r), len(u), float(mu),
                                 _p(bu), _p(bi))


def bias_als_epoch(u, i, r, mu, bu, bi, ucnt, icnt, reg):
    u = _c(u, np.int32); i = _c(i, np.int32); r = _c(r, np.float64)
    lib().oracle_bias_als_epoch(_p(u), _p(i), _p(r), len(u), float(mu),
                                _p(bu), _p(bi), _p(ucnt), _p(icnt),
                                len(bu), len(bi), float(reg))


# ------------------------------------------------------------ factor ALS
def als_half_sweep(ent, oth, r, mu, ob, oq, n_ent, reg):
    """Factor-model ALS, one side, FP64 (the restatement mf_als_sweep is
    checked against; BASELINE config 5 has no reference counterpart).

    For each entity e: x_e = [w_e; b_e] solves
        (sum_n y_n y_n^T + reg I) x_e = sum_n t_n y_n,
        y_n = [oq[oth_n]; 1],  t_n = r_n - mu - ob[oth_n],
    the latent-factor extension of baseline_model.py:328-337 (with k = 0 it
    is (reg + n_e) b_e = sum_n t_n exactly).  Returns (biases, rows)."""
    ent = np.asarray(ent, np.int64)
    oth = np.asarray(oth, np.int64)
    r = np.asarray(r, np.float64)
    oq = np.asarray(oq, np.float64)
    ob = np.asarray(ob, np.float64)
    k = oq.shape[1]
    order = np.argsort(ent, kind="stable")
    ptr = np.zeros(n_ent + 1, np.int64)
    np.cumsum(np.bincount(ent, minlength=n_ent), out=ptr[1:])
    bias = np.zeros(n_ent)
    feat = np.zeros((n_ent, k))
    eye = reg * np.eye(k + 1)
    for e in range(n_ent):
        idx = order[ptr[e]:ptr[e + 1]]
        Y = np.empty((len(idx), k + 1))
        Y[:, :k] = oq[oth[idx]]
        Y[:, k] = 1.0
        t = (r[idx] - mu) - ob[oth[idx]]
        x = np.linalg.solve(Y.T @ Y + eye, Y.T @ t)
        feat[e] = x[:k]
        bias[e] = x[k]
    return bias, feat


def als_epoch(u, i, r, mu, bu, bi, P, Q, reg):
    """One factor-ALS epoch as baseline_model.py:326-348 orders the bias
    model's: users from the current item side, then items from the new user
    side.  Returns (bu, bi, P, Q) (new arrays)."""
    bu, P = als_half_sweep(u, i, r, mu, bi, Q, len(bu), reg)
    bi, Q = als_half_sweep(i, u, r, mu, bu, P, len(bi), reg)
    return bu, bi, P, Q


def linear_rmse(u, i, r, mu, bu, bi, P, Q) -> float:
    """Training RMSE of the linear predictor ((mu + b_i) + b_u) + p.q
    (kernels.py:42-44, kernel_matrix_factorization.py:271-315), NumPy."""
    pred = ((mu + bi[i]) + bu[u]) + np.einsum("nk,nk->n", P[u], Q[i])
    return float(np.sqrt(np.mean((np.asarray(r, np.float64) - pred) ** 2)))


# ------------------------------------------------------------ host side
def preprocess_fit(X: pd.DataFrame, y) -> tuple:
    """recommender_base.py:120-164 for type='fit'.

    Returns (triples (n,3) float64 in post-shuffle order, user_ids, item_ids)
    where user_ids/item_ids are the first-appearance unique arrays (the keys of
    user_id_map / item_id_map in id order).
    """
    X = X.loc[:, ["user_id", "item_id"]]
    X["rating"] = y
    if X.duplicated(subset=["user_id", "item_id"]).sum() != 0:
        raise ValueError("Duplicate user-item ratings in matrix")
    X = X.sample(frac=1, replace=False)                  # RNG draw #1
    user_ids = X["user_id"].unique()
    item_ids = X["item_id"].unique()
    umap = {v: n for n, v in enumerate(user_ids)}
    imap = {v: n for n, v in enumerate(item_ids)}
    X.loc[:, "user_id"] = X["user_id"].map(umap)
    X.loc[:, "item_id"] = X["item_id"].map(imap)
    return X, user_ids, item_ids


def oracle_kernel_fit(X: pd.DataFrame, y, n_factors=100, n_epochs=100,
                      kernel="linear", gamma="auto", reg=1.0, lr=0.01,
                      init_mean=0.0, init_sd=0.1, min_rating=0.0,
                      max_rating=5.0) -> dict:
    """KernelMF.fit (kernel_matrix_factorization.py:81-128 + _sgd :320-445)
    restated on the CPU oracle.  Caller seeds np.random beforehand."""
    g = 1 / n_factors if gamma == "auto" else gamma
    Xp, user_ids, item_ids = preprocess_fit(X, y)
    mu = Xp["rating"].mean()                               # :90
    nu, ni = len(user_ids), len(item_ids)
    bu = np.zeros(nu); bi = np.zeros(ni)                   # :93-94
    P = np.random.normal(init_mean, init_sd, (nu, n_factors))   # RNG #2
    Q = np.random.normal(init_mean, init_sd, (ni, n_factors))   # RNG #3
    arr = Xp.to_numpy(dtype=np.float64)
    u = arr[:, 0].astype(np.int32); i = arr[:, 1].astype(np.int32)
    r = arr[:, 2].copy()
    order = np.arange(len(u), dtype=np.int64)
    train_rmse = []
    for _ in range(n_epochs):
        np.random.shuffle(order)                            # :371, RNG #4/epoch
        sgd_pass(u, i, r, mu, bu, bi, P, Q, kernel=kernel, gamma=g, lr=lr,
                 reg=reg, min_rating=min_rating, max_rating=max_rating,
                 order=order)
        train_rmse.append(rmse(u, i, r, mu, bu, bi, P, Q, kernel=kernel,
                               gamma=g, min_rating=min_rating,
                               max_rating=max_rating))
    return dict(user_ids=user_ids, item_ids=item_ids, global_mean=mu,
                user_biases=bu, item_biases=bi, user_features=P,
                item_features=Q, train_rmse=np.array(train_rmse),
                u=u, i=i, r=r, gamma=g)

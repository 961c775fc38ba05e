"""KernelMF on MI355X: the reference estimator, trained by libmf_hip.so.

Surface and semantics of ``KernelMF`` (kernel_matrix_factorization.py:19-237):
same constructor arguments and defaults, same attributes (NumPy float64 after
fit), same RNG draw order, same ``fit / predict / update_users`` behaviour.
Three keyword arguments are new and default to the reference's behaviour:

``dtype``     "float64" (reference precision) or "float32" (half the HBM
              traffic; the throughput setting).
``schedule``  "exact" (default): the reference's visit order every epoch,
              reproduced bit-for-bit up to dot-product summation order;
              "colored": a conflict-free edge-colouring schedule, a different
              valid sequential order per epoch;
              "strata": the stratified sweep (users x items cut into B x B
              blocks, item slabs resident in LDS; mf_strata.hpp), also a
              valid sequential order per epoch -- the throughput setting.
``device``    HIP device ("cuda", "cuda:1", ...); None = current device.
"""

from __future__ import annotations

from typing import Union

import numpy as np
import pandas as pd

from .engine import SGDEngine, canonical_dtype, fit_epochs
from .recommender_base import RecommenderBase


class KernelMF(RecommenderBase):
    """Kernel matrix factorisation, r_ui ~ K(p_u, q_i) with SGD
    (kernel_matrix_factorization.py:19-79).

    Arguments (reference defaults): n_factors=100, n_epochs=100,
    kernel='linear' | 'sigmoid' | 'rbf', gamma='auto' (1/n_factors, rbf
    only), reg=1, lr=0.01, init_mean=0, init_sd=0.1, min_rating=0,
    max_rating=5, verbose=1; plus dtype, schedule, device (module docstring).
    """

    def __init__(self, n_factors: int = 100, n_epochs: int = 100,
                 kernel: str = "linear", gamma: Union[str, float] = "auto",
                 reg: float = 1, lr: float = 0.01, init_mean: float = 0,
                 init_sd: float = 0.1, min_rating: int = 0, max_rating: int = 5,
                 verbose: int = 1, dtype: str = "float64",
                 schedule: str = "exact", device=None):
        if kernel not in ("linear", "sigmoid", "rbf"):
            raise ValueError("Kernel must be one of linear, sigmoid, or rbf")
        if schedule not in ("exact", "colored", "strata"):
            raise ValueError("schedule must be 'exact', 'colored' or 'strata'")
        canonical_dtype(dtype)
        super().__init__(min_rating=min_rating, max_rating=max_rating, verbose=verbose)
        self.n_factors = n_factors
        self.n_epochs = n_epochs
        self.kernel = kernel
        # resolved at construction, as the reference does (:74)
        self.gamma = 1 / n_factors if gamma == "auto" else gamma
        self.reg = reg
        self.lr = lr
        self.init_mean = init_mean
        self.init_sd = init_sd
        self.dtype = dtype
        self.schedule = schedule
        self.device = device

    # ----------------------------------------------------- device state
    def _make_engine(self, X: pd.DataFrame) -> SGDEngine:
        n = len(X)
        u = X["user_id"].to_numpy(np.int32) if n else np.zeros(0, np.int32)
        i = X["item_id"].to_numpy(np.int32) if n else np.zeros(0, np.int32)
        r = X["rating"].to_numpy(np.float64) if n else np.zeros(0)
        return SGDEngine(u, i, r, len(self.user_features), len(self.item_features),
                         self.n_factors, self.kernel, self.dtype, self.device,
                         gamma=self.gamma, min_rating=self.min_rating,
                         max_rating=self.max_rating, global_mean=self.global_mean)

    def _sync_params(self, eng: SGDEngine) -> None:
        P, Q, bu, bi = eng.params_numpy()
        self.user_features, self.item_features = P, Q
        self.user_biases, self.item_biases = bu, bi
        self._param_ids = self._ids()

    def _ids(self):
        return tuple(id(a) for a in (self.user_features, self.item_features,
                                     self.user_biases, self.item_biases))

    def _predictor(self) -> SGDEngine:
        """Engine holding the current parameters (re-uploaded when the
        attribute arrays were replaced, e.g. after unpickling)."""
        eng = getattr(self, "_pred_engine", None)
        if eng is None or getattr(self, "_param_ids", None) != self._ids():
            eng = SGDEngine(np.zeros(0, np.int32), np.zeros(0, np.int32), np.zeros(0),
                            len(self.user_features), len(self.item_features),
                            self.n_factors, self.kernel, self.dtype, self.device,
                            gamma=self.gamma, min_rating=self.min_rating,
                            max_rating=self.max_rating, global_mean=self.global_mean)
            eng.load_params(self.user_features, self.item_features,
                            self.user_biases, self.item_biases)
            self._pred_engine = eng
            self._param_ids = self._ids()
        return eng

    def __getstate__(self):
        # pickles carry plain NumPy state only (loadable without a GPU)
        state = self.__dict__.copy()
        state.pop("_pred_engine", None)
        state.pop("_param_ids", None)
        return state

    # ------------------------------------------------------------ API
    def fit(self, X: pd.DataFrame, y: pd.Series):
        """kernel_matrix_factorization.py:81-128 (RNG: sample, normal(P),
        normal(Q), then one draw per epoch)."""
        X = self._preprocess_data(X=X, y=y, type="fit")
        self.global_mean = X["rating"].mean()
        self.user_biases = np.zeros(self.n_users)
        self.item_biases = np.zeros(self.n_items)
        self.user_features = np.random.normal(self.init_mean, self.init_sd,
                                              (self.n_users, self.n_factors))
        self.item_features = np.random.normal(self.init_mean, self.init_sd,
                                              (self.n_items, self.n_factors))
        eng = self._make_engine(X)
        eng.load_params(self.user_features, self.item_features,
                        self.user_biases, self.item_biases)
        self.train_rmse = fit_epochs(eng, self.n_epochs, self.schedule, self.lr,
                                     self.reg, verbose=self.verbose)
        self._sync_params(eng)
        self._pred_engine = eng
        return self

    def predict(self, X: pd.DataFrame, bound_ratings: bool = True) -> list:
        """kernel_matrix_factorization.py:130-163."""
        if X.shape[0] == 0:
            return []
        X = self._preprocess_data(X=X, type="predict")
        u = X["user_id"].to_numpy(np.int32)
        i = X["item_id"].to_numpy(np.int32)
        pred = self._predictor().predict(u, i, bound_ratings)
        self.predictions_possible = ((u != -1) & (i != -1)).tolist()
        return pred.tolist()

    def update_users(self, X: pd.DataFrame, y: pd.Series, lr: float = 0.01,
                     n_epochs: int = 20, verbose: int = 0):
        """kernel_matrix_factorization.py:165-237: re-initialise known users,
        append new users, SGD with item parameters frozen."""
        X, known_users, new_users = self._preprocess_data(X=X, y=y, type="update")
        n_new_users = len(new_users)
        for user in known_users:
            user_index = self.user_id_map[user]
            self.user_biases[user_index] = 0
            self.user_features[user_index, :] = np.random.normal(
                self.init_mean, self.init_sd, (1, self.n_factors))
        self.user_biases = np.append(self.user_biases, np.zeros(n_new_users))
        new_user_features = np.random.normal(self.init_mean, self.init_sd,
                                             (n_new_users, self.n_factors))
        self.user_features = np.concatenate((self.user_features, new_user_features),
                                            axis=0)
        eng = self._make_engine(X)
        eng.load_params(self.user_features, self.item_features,
                        self.user_biases, self.item_biases)
        self.train_rmse = fit_epochs(eng, n_epochs, self.schedule, lr, self.reg,
                                     update_user=True, update_item=False,
                                     verbose=verbose)
        self._sync_params(eng)
        self._pred_engine = eng

    def recommend_batch(self, users, amount: int = 10, exclude_known=None,
                        bound_ratings: bool = True) -> pd.DataFrame:
        """Top ``amount`` items for many users in one GPU pass (mf_topk).

        ``exclude_known``: optional DataFrame[user_id, item_id] of pairs to
        skip.  Ties rank the lower internal item id first (recommend() keeps
        pandas' order instead).  Returns DataFrame[user_id, item_id,
        rating_pred] ordered by user then rank."""
        users = list(users)
        uid = self._remap(pd.Series(users, dtype=object), self.user_id_map)
        exclude = None
        if exclude_known is not None and len(exclude_known):
            exclude = np.zeros((len(users), self.n_items), np.uint8)
            pos = {u: n for n, u in enumerate(users)}
            ex_u = exclude_known["user_id"].map(pos)
            ex_i = self._remap(exclude_known["item_id"], self.item_id_map)
            ok = ex_u.notna().to_numpy() & (ex_i >= 0)
            exclude[ex_u[ok].astype(np.int64).to_numpy(), ex_i[ok]] = 1
        amount = min(amount, self.n_items)
        items, scores = self._predictor().topk(uid, amount, exclude)
        inv = np.asarray(list(self.item_id_map.keys()), dtype=object)
        rows_u, rows_i, rows_s = [], [], []
        for q, user in enumerate(users):
            valid = items[q] >= 0
            rows_u += [user] * int(valid.sum())
            rows_i += list(inv[items[q][valid]])
            rows_s += list(scores[q][valid])
        out = pd.DataFrame({"user_id": rows_u, "item_id": rows_i, "rating_pred": rows_s})
        if bound_ratings:
            out["rating_pred"] = out["rating_pred"].clip(lower=self.min_rating,
                                                         upper=self.max_rating)
        return out

"""BaselineModel on MI355X: r_ui ~ mu + b_u + b_i (baseline_model.py:10-180).

The bias-only member of the family, exported because examples/example.py
imports it.  SGD runs the same conflict-free batch schedules as KernelMF
(mf_bias_sgd_epoch); ALS sums every id's ratings in the reference's row order
(mf_bias_als_epoch), so both match the reference loop bit for bit (SGD up to
nothing: there is no dot product in the bias model).
"""

from __future__ import annotations

import numpy as np
import pandas as pd

from .engine import BiasALS, SGDEngine, canonical_dtype, fit_epochs
from .recommender_base import RecommenderBase


class BaselineModel(RecommenderBase):
    """Arguments (reference defaults): method='sgd' | 'als', n_epochs=100,
    reg=1, lr=0.01, min_rating=0, max_rating=5, verbose=1; plus dtype,
    schedule and device as in KernelMF."""

    def __init__(self, method: str = "sgd", n_epochs: int = 100, reg: float = 1,
                 lr: float = 0.01, min_rating: int = 0, max_rating: int = 5,
                 verbose=1, dtype: str = "float64", schedule: str = "exact",
                 device=None):
        if method not in ("sgd", "als"):
            raise ValueError('Method param must be either "sgd" or "als"')
        if schedule not in ("exact", "colored"):
            raise ValueError("schedule must be 'exact' or 'colored'")
        canonical_dtype(dtype)
        super().__init__(min_rating=min_rating, max_rating=max_rating, verbose=verbose)
        self.method = method
        self.n_epochs = n_epochs
        self.reg = reg
        self.lr = lr
        self.dtype = dtype
        self.schedule = schedule
        self.device = device

    def _engine(self, X: pd.DataFrame) -> SGDEngine:
        n = len(X)
        u = X["user_id"].to_numpy(np.int32) if n else np.zeros(0, np.int32)
        i = X["item_id"].to_numpy(np.int32) if n else np.zeros(0, np.int32)
        r = X["rating"].to_numpy(np.float64) if n else np.zeros(0)
        eng = SGDEngine(u, i, r, len(self.user_biases), len(self.item_biases), 0, "bias",
                        self.dtype, self.device, min_rating=self.min_rating,
                        max_rating=self.max_rating, global_mean=self.global_mean)
        eng.load_params(bu=self.user_biases, bi=self.item_biases)
        return eng

    def _sync(self, eng: SGDEngine) -> None:
        _, _, self.user_biases, self.item_biases = eng.params_numpy()

    def __getstate__(self):
        return self.__dict__.copy()

    def fit(self, X: pd.DataFrame, y: pd.Series):
        """baseline_model.py:63-102."""
        X = self._preprocess_data(X=X, y=y, type="fit")
        self.global_mean = X["rating"].mean()
        self.user_biases = np.zeros(self.n_users)
        self.item_biases = np.zeros(self.n_items)
        eng = self._engine(X)
        if self.method == "sgd":
            self.train_rmse = fit_epochs(eng, self.n_epochs, self.schedule, self.lr,
                                         self.reg, verbose=self.verbose)
        else:
            als = BiasALS(eng)
            self.train_rmse = []
            for epoch in range(self.n_epochs):          # baseline_model.py:326-360
                als.epoch(self.reg)
                eng.sse_async(epoch)
                if self.verbose == 1:
                    rmse = eng.rmse_values(epoch + 1)[epoch]
                    self.train_rmse.append(rmse)
                    print("Epoch ", epoch + 1, "/", self.n_epochs, " -  train_rmse:", rmse)
            if self.verbose != 1:
                self.train_rmse = eng.rmse_values(self.n_epochs)
        self._sync(eng)
        return self

    def predict(self, X: pd.DataFrame, bound_ratings: bool = True) -> list:
        """baseline_model.py:104-134."""
        if X.shape[0] == 0:
            return []
        X = self._preprocess_data(X=X, type="predict")
        u = X["user_id"].to_numpy(np.int32)
        i = X["item_id"].to_numpy(np.int32)
        eng = SGDEngine(np.zeros(0, np.int32), np.zeros(0, np.int32), np.zeros(0),
                        len(self.user_biases), len(self.item_biases), 0, "bias",
                        self.dtype, self.device, min_rating=self.min_rating,
                        max_rating=self.max_rating, global_mean=self.global_mean)
        eng.load_params(bu=self.user_biases, bi=self.item_biases)
        pred = eng.predict(u, i, bound_ratings)
        self.predictions_possible = ((u != -1) & (i != -1)).tolist()
        return pred.tolist()

    def update_users(self, X: pd.DataFrame, y: pd.Series, lr: float = 0.01,
                     n_epochs: int = 20, verbose: int = 0):
        """baseline_model.py:136-180: item biases frozen."""
        X, known_users, new_users = self._preprocess_data(X=X, y=y, type="update")
        for user in known_users:
            self.user_biases[self.user_id_map[user]] = 0
        self.user_biases = np.append(self.user_biases, np.zeros(len(new_users)))
        eng = self._engine(X)
        self.train_rmse = fit_epochs(eng, n_epochs, self.schedule, lr, self.reg,
                                     update_user=True, update_item=False,
                                     verbose=verbose)
        self._sync(eng)

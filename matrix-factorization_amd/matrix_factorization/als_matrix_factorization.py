"""ALSMF: the linear-kernel factor model trained by alternating least squares.

BASELINE.json config 5 (rank-128 ALS normal-equations path, MFMA Gramian).
The reference has no factor ALS; its bias-only ALS (BaselineModel
method='als', baseline_model.py:283-362) alternates closed-form user and item
updates, and this estimator extends exactly that to the latent factors of
KernelMF's linear kernel (kernels.py:21-44):

    per user u, items fixed:  (sum_i y_i y_i^T + reg I) [p_u; b_u] = sum_i t_ui y_i
                              y_i = [q_i; 1],  t_ui = r_ui - mu - b_i
    then per item, users fixed (same form),

which for n_factors = 0 is the reference's bias update
(reg + n_u) b_u = sum_i (r_ui - mu - b_i) (:328-337).  One epoch = users then
items then the training RMSE, as `_als` orders it.  Everything around fit --
constructor arguments, RNG draw order of the initial factors, predict,
recommend, pickling -- is KernelMF's (linear kernel, float32 parameters).
"""

from __future__ import annotations

import numpy as np
import pandas as pd

from .engine import FactorALS
from .kernel_matrix_factorization import KernelMF


class ALSMF(KernelMF):
    """Factor model r_ui ~ mu + b_u + b_i + p_u . q_i fitted by ALS on the GPU
    (mf_als_sweep: f32-input MFMA Gramian + LDS elimination per entity).

    Arguments: n_factors (1..128), n_epochs, reg (> 0), init_mean, init_sd,
    min_rating, max_rating, verbose, device -- as KernelMF.
    """

    def __init__(self, n_factors: int = 100, n_epochs: int = 10, reg: float = 1,
                 init_mean: float = 0, init_sd: float = 0.1, min_rating: int = 0,
                 max_rating: int = 5, verbose: int = 1, device=None):
        super().__init__(n_factors=n_factors, n_epochs=n_epochs, kernel="linear",
                         reg=reg, init_mean=init_mean, init_sd=init_sd,
                         min_rating=min_rating, max_rating=max_rating, verbose=verbose,
                         dtype="float32", schedule="exact", device=device)

    def _run(self, eng, n_epochs: int, users_only: bool, verbose: int) -> list:
        als = FactorALS(eng)
        rmse = []
        for epoch in range(n_epochs):
            als.sweep_users(self.reg)
            if not users_only:
                als.sweep_items(self.reg)
            eng.sse_async(epoch)
            if verbose == 1:
                rmse.append(eng.rmse_values(epoch + 1)[epoch])
                print("Epoch ", epoch + 1, "/", n_epochs, " -  train_rmse:", rmse[-1])
        if verbose != 1:
            rmse = eng.rmse_values(n_epochs)
        return rmse

    def fit(self, X: pd.DataFrame, y: pd.Series):
        """As KernelMF.fit (same preprocessing and RNG order: sample,
        normal(P), normal(Q)), then n_epochs ALS epochs."""
        X = self._preprocess_data(X=X, y=y, type="fit")
        self.global_mean = X["rating"].mean()
        self.user_biases = np.zeros(self.n_users)
        self.item_biases = np.zeros(self.n_items)
        self.user_features = np.random.normal(self.init_mean, self.init_sd,
                                              (self.n_users, self.n_factors))
        self.item_features = np.random.normal(self.init_mean, self.init_sd,
                                              (self.n_items, self.n_factors))
        eng = self._make_engine(X, len(self.user_features), len(self.item_features))
        eng.load_params(self.user_features, self.item_features,
                        self.user_biases, self.item_biases)
        self.train_rmse = self._run(eng, self.n_epochs, False, self.verbose)
        self._sync_params(eng)
        self._pred_engine = eng
        return self

    def update_users(self, X: pd.DataFrame, y: pd.Series, lr: float = 0.01,
                     n_epochs: int = 1, verbose: int = 0):
        """KernelMF.update_users with the item side frozen: known users are
        re-initialised, new users appended (same RNG order), then the user
        half-sweep (the exact least-squares update; ``lr`` is unused)."""
        X, known_users, new_users = self._preprocess_data(X=X, y=y, type="update")
        for user in known_users:
            user_index = self.user_id_map[user]
            self.user_biases[user_index] = 0
            self.user_features[user_index, :] = np.random.normal(
                self.init_mean, self.init_sd, (1, self.n_factors))
        self.user_biases = np.append(self.user_biases, np.zeros(len(new_users)))
        new_user_features = np.random.normal(self.init_mean, self.init_sd,
                                             (len(new_users), self.n_factors))
        self.user_features = np.concatenate((self.user_features, new_user_features), axis=0)
        eng = self._make_engine(X, len(self.user_features), len(self.item_features))
        eng.load_params(self.user_features, self.item_features,
                        self.user_biases, self.item_biases)
        self.train_rmse = self._run(eng, n_epochs, True, verbose)
        self._sync_params(eng)
        self._pred_engine = eng

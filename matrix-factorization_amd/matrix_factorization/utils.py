"""train_update_test_split (utils.py:8-72 of the reference).

Host-side data preparation for update_users experiments; exported because
examples/example.py imports it.  Draws from NumPy's global RandomState in the
reference's order (choice -> sample -> sklearn's train_test_split), so a seeded
run splits identically.
"""

from __future__ import annotations

from typing import Tuple

import numpy as np
import pandas as pd
from sklearn.model_selection import train_test_split


def train_update_test_split(
    X: pd.DataFrame, frac_new_users: float
) -> Tuple[pd.DataFrame, pd.Series, pd.DataFrame, pd.Series, pd.DataFrame, pd.Series]:
    """Split ratings into (initial training, update training, update test).

    A fraction ``frac_new_users`` of the users is held out of the initial
    training set; each held-out user's ratings are split 50/50 (stratified by
    user) into an update set and a test set.  Returns
    X_train_initial, y_train_initial, X_train_update, y_train_update,
    X_test_update, y_test_update.
    """
    users = X["user_id"].unique()
    held_out = np.random.choice(users, size=round(frac_new_users * len(users)),
                                replace=False)
    is_new = X["user_id"].isin(held_out)
    initial = X[~is_new].sample(frac=1, replace=False)
    data_update = X[is_new]
    upd, test = train_test_split(data_update, stratify=data_update["user_id"],
                                 test_size=0.5)
    cols = ["user_id", "item_id"]
    return (initial[cols], initial["rating"], upd[cols], upd["rating"],
            test[cols], test["rating"])

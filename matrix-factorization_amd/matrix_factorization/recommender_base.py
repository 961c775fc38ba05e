"""Estimator base class: the reference's public surface, GPU underneath.

Mirrors ``RecommenderBase`` (recommender_base.py:14-271): an sklearn
estimator with id remapping, ``recommend`` and the known-user/item helpers.
Every random draw happens in the reference's order through NumPy's global
legacy RandomState (``X.sample(frac=1)`` here, ``np.random.normal`` /
``np.random.shuffle`` in the subclasses), so ``np.random.seed(s)`` followed by
the same calls gives the reference's results.
"""

from __future__ import annotations

from abc import ABCMeta, abstractmethod
from concurrent.futures import Future, ThreadPoolExecutor
from typing import Any, Tuple, Union

import numpy as np
import pandas as pd
from sklearn.base import BaseEstimator, RegressorMixin

from . import _prep

# integer id columns of at least this many rows take the native
# preprocessing path (mf_prep.cpp); results are identical either way
FAST_PREP_MIN_ROWS = 1 << 16

# one worker for id maps built beside fit()'s device work
_MAP_POOL = ThreadPoolExecutor(1, thread_name_prefix="mf-idmap")


def _id_map(uniq: np.ndarray) -> dict:
    """{id: position} in first-appearance order (recommender_base.py:135-138:
    ``{uid: n for n, uid in enumerate(unique)}``, NumPy scalar keys)."""
    return dict(zip(uniq, range(len(uniq))))


def _index_of(keys) -> pd.Index:
    return pd.Index(list(keys))


def _aligned_rating(X: pd.DataFrame, y):
    """The values ``X["rating"] = y`` puts in the column (recommender_base.py:
    123), read without copying the frame: a Series on the same index as is,
    else reindexed to X's index as the assignment aligns it; None (take the
    pandas path) for anything that is not a Series."""
    if not isinstance(y, pd.Series):
        return None
    if y.index.equals(X.index):
        return y.to_numpy()
    if not X.index.is_unique or not y.index.is_unique:
        return None
    return y.reindex(X.index).to_numpy()


class RecommenderBase(BaseEstimator, RegressorMixin, metaclass=ABCMeta):
    """Abstract base of every model (recommender_base.py:14-51).

    Attributes after fit: n_users, n_items, global_mean, user_id_map,
    item_id_map (dict: external id -> internal id, first-appearance order of
    the shuffled training data).
    """

    @abstractmethod
    def __init__(self, min_rating: float = 0, max_rating: float = 5, verbose: int = 0):
        self.min_rating = min_rating
        self.max_rating = max_rating
        self.verbose = verbose

    # ------------------------------------------------ known ids (:53-95)
    @property
    def known_users(self):
        return set(self.user_id_map.keys())

    @property
    def known_items(self):
        return set(self.item_id_map.keys())

    def contains_user(self, user_id: Any) -> bool:
        return user_id in self.user_id_map

    def contains_item(self, item_id: Any) -> bool:
        return item_id in self.item_id_map

    # ---------------------------------------------------- id remapping
    @staticmethod
    def _remap(values: pd.Series, id_map: dict) -> np.ndarray:
        """External ids -> internal int64 ids, -1 where unknown.

        The maps are built so that the internal id of a key equals its
        insertion position, which lets pandas' hash index do the lookup."""
        idx = _index_of(id_map.keys())
        if len(id_map) and next(reversed(id_map.values())) != len(id_map) - 1:
            # not positional (never produced by this package); use the dict
            return values.map(id_map).fillna(-1).to_numpy().astype(np.int64)
        return idx.get_indexer(values.to_numpy()).astype(np.int64)

    def _preprocess_data(
        self, X: pd.DataFrame, y: pd.Series = None, type: str = "fit"
    ) -> Union[pd.DataFrame, Tuple[pd.DataFrame, list, list]]:
        """recommender_base.py:97-173.

        fit:     duplicate check, ``X.sample(frac=1)`` (one RNG draw), new id
                 maps in first-appearance order of the shuffled rows;
        update:  same check and shuffle, drop ratings of unknown items, append
                 new users to user_id_map (ids max + 1, ...);
        predict: unknown ids become -1.
        Returns a frame with int64 user_id / item_id (and rating).

        Integer ids of at least FAST_PREP_MIN_ROWS rows take the native path
        (mf_prep.cpp), same results: the duplicate check runs on worker
        threads while this thread draws the permutation (the RNG state is
        put back if the check then raises, so a failed fit draws nothing, as
        in the reference), and fit reads the id columns and ``y`` in place
        instead of copying the frame first.
        """
        native = None
        if type in ("fit", "update"):
            ids = self._int64_ids(X)
            if ids is not None:
                perm, dense = self._checked_permutation(ids, dense=type == "fit",
                                                        draw=self._draw_permutation)
                rating = _aligned_rating(X, y) if type == "fit" else None
                if rating is not None:
                    return self._fit_maps_native(X.index, ids, rating, perm, dense)
                native = perm

        X = X.loc[:, ["user_id", "item_id"]]
        if type != "predict":
            X["rating"] = y

        if type in ("fit", "update"):
            if native is not None:
                if type == "fit":
                    return self._fit_maps_native(X.index, ids, X["rating"].to_numpy(), native,
                                                 dense)
                X = X.iloc[native]
            else:
                if X.duplicated(subset=["user_id", "item_id"]).sum() != 0:
                    raise ValueError("Duplicate user-item ratings in matrix")
                X = X.sample(frac=1, replace=False)

        if type == "fit":
            ucodes, uniq_u = pd.factorize(X["user_id"], sort=False)
            icodes, uniq_i = pd.factorize(X["item_id"], sort=False)
            self.user_id_map = {uid: n for n, uid in enumerate(uniq_u)}
            self.item_id_map = {iid: n for n, iid in enumerate(uniq_i)}
            self.n_users = len(uniq_u)
            self.n_items = len(uniq_i)
            out = pd.DataFrame({"user_id": ucodes.astype(np.int64),
                                "item_id": icodes.astype(np.int64)}, index=X.index)
            out["rating"] = X["rating"]
            return out

        known_users, new_users = [], []
        if type == "update":
            X = X[X["item_id"].isin(list(self.item_id_map.keys()))].copy()
            new_id = max(self.user_id_map.values()) + 1
            for user in X["user_id"].unique():
                if user in self.user_id_map:
                    known_users.append(user)
                    continue
                new_users.append(user)
                self.user_id_map[user] = new_id
                new_id += 1

        out = pd.DataFrame({"user_id": self._remap(X["user_id"], self.user_id_map),
                            "item_id": self._remap(X["item_id"], self.item_id_map)},
                           index=X.index)
        if type != "predict":
            out["rating"] = X["rating"]
        if type == "update":
            return out, known_users, new_users
        return out

    def _join_maps(self) -> None:
        """Wait for a user id map built on a worker thread (see
        _fit_maps_native) and install it."""
        fut = self.__dict__.pop("_maps_pending", None)
        if fut is not None:
            self.user_id_map = fut.result()

    def _int64_ids(self, X: pd.DataFrame):
        """(user ids, item ids) as int64 arrays when both columns are integer
        and the frame is large enough for the native path, else None."""
        if len(X) < FAST_PREP_MIN_ROWS:
            return None
        cu, ci = X["user_id"], X["item_id"]
        u = _prep.as_int64_ids(cu.to_numpy())
        i = _prep.as_int64_ids(ci.to_numpy())
        self._id_dtypes = (cu.dtype, ci.dtype)
        return None if u is None or i is None else (u, i)

    def _draw_permutation(self, n: int) -> np.ndarray:
        """``np.random.permutation(n)``: X.sample(frac=1)'s draw (int64)."""
        return _prep.legacy_permutation(n)

    @staticmethod
    def _checked_permutation(ids, dense: bool = False, draw=None):
        """(perm, dense ids or None): the duplicate-pair check
        (recommender_base.py:125-128) -- and with ``dense`` the columns'
        ``_prep.dense_ids`` -- on worker threads beside ``X.sample(frac=1)``'s
        draw (:131) on this one; if the check fails, the RNG state is
        restored before the ValueError."""
        state = np.random.get_state()
        with ThreadPoolExecutor(3 if dense else 1) as ex:
            dup = ex.submit(_prep.pairs_duplicated, *ids)
            dn = [ex.submit(_prep.dense_ids, v) for v in ids] if dense else None
            n = len(ids[0])
            perm = draw(n) if draw is not None else _prep.legacy_permutation(n)   # = X.sample's
            if dup.result():
                np.random.set_state(state)
                raise ValueError("Duplicate user-item ratings in matrix")
            dn = [f.result() for f in dn] if dense else None
        return perm, dn

    def _fit_maps_native(self, index: pd.Index, ids, rating: np.ndarray,
                         perm: np.ndarray, dense=None) -> pd.DataFrame:
        """The fit branch for integer ids: the rows in ``perm`` order (the
        order X.sample(frac=1) gives), id maps in first-appearance order of
        that order (pd.factorize / unique of the shuffled column), all in
        mf_prep.cpp: from the columns' dense ids (``dense``, drawn beside the
        permutation, or here), users, items and the ratings on three threads;
        this one builds each id map as soon as its column is done."""
        if dense is None:
            dense = [_prep.dense_ids(v) for v in ids]
        with ThreadPoolExecutor(3) as ex:
            # items first: their map is small and is built while the users finish
            fut = [ex.submit(_prep.factorize_shuffled, d, perm) for d in dense[::-1]][::-1]
            num = rating.dtype.kind in "fiu"
            rfut = ex.submit(_prep.gather, rating, perm) if num else None
            maps, codes, sizes = [None, None], [None, None], [0, 0]
            defer = getattr(self, "_defer_maps", False)
            for k in (1, 0):
                c, uniq = fut[k].result()
                dt = self._id_dtypes[k]
                uniq = uniq.view(dt) if dt.itemsize == 8 else uniq.astype(dt)
                sizes[k] = len(uniq)
                if defer and k == 0:
                    # the user map (10^6 entries at C3, ~0.2 s of dict
                    # inserts) is built on a worker thread while fit() goes
                    # on; fit() joins it before it returns (_join_maps)
                    maps[k] = _MAP_POOL.submit(_id_map, uniq)
                else:
                    maps[k] = _id_map(uniq)
                codes[k] = c
            rating = rfut.result() if num else rating[perm]
        if isinstance(maps[0], Future):
            self._maps_pending = maps[0]
            self.user_id_map = None
        else:
            self.user_id_map = maps[0]
        self.item_id_map = maps[1]
        self.n_users, self.n_items = sizes
        idx = index
        if isinstance(idx, pd.RangeIndex):
            idx = pd.Index(idx.start + idx.step * perm if (idx.start, idx.step) != (0, 1)
                           else perm)
        else:
            idx = idx.take(perm)
        return pd.DataFrame({"user_id": codes[0], "item_id": codes[1], "rating": rating},
                            index=idx, copy=False)

    @abstractmethod
    def fit(self, X: pd.DataFrame, y: pd.Series):
        return self

    @abstractmethod
    def predict(self, X: pd.DataFrame, bound_ratings: bool = True) -> list:
        return []

    def recommend(self, user: Any, amount: int = 10, items_known: list = None,
                  include_user: bool = True, bound_ratings: bool = True) -> pd.DataFrame:
        """Top ``amount`` unseen items for ``user``, best first
        (recommender_base.py:214-271): every candidate is scored with
        ``predict(bound_ratings=False)`` on the GPU and ranked by pandas'
        ``sort_values`` exactly as the reference ranks them."""
        items = list(self.item_id_map.keys())
        if items_known is not None:
            known = set(items_known)
            items = [item for item in items if item not in known]
        recs = pd.DataFrame({"user_id": user, "item_id": items})
        recs["rating_pred"] = self.predict(X=recs, bound_ratings=False)
        recs.sort_values(by="rating_pred", ascending=False, inplace=True)
        recs = recs.head(amount).copy()
        if bound_ratings:
            recs["rating_pred"] = recs["rating_pred"].clip(lower=self.min_rating,
                                                           upper=self.max_rating)
        if not include_user:
            recs.drop(["user_id"], axis="columns", inplace=True)
        return recs

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
              Known deviation: a different order trains to a slightly
              different model.  At C3 (20 epochs) the default strata plan
              ends +0.32e-5 train RMSE over the mean of the reference's
              random orders (24 draws against 28 reference runs, round 5;
              +0.60e-5 pooled with round 4's 48 draws, about 2.7 standard
              errors), where the reference's own run-to-run SD is ~1e-5;
              "exact" has no such gap.
``device``    HIP device ("cuda", "cuda:1", ...); None = current device.
``distributed`` False (default) or True: process-group mode.  When
              torch.distributed is initialised with world_size > 1, every
              rank calls ``fit`` with the same data and the same NumPy RNG
              state; users are sharded across the ranks (one GPU each,
              distributed.fit_sharded) and every rank ends with the full
              model.  How the ranks share the item rows is ``exchange``
              below: by default ("rotate") each rank holds one item range
              at a time and passes it round the ring (RCCL send / recv)
              between N sub-epochs, then one all-gather; "delta" is the
              once-per-epoch all-reduce of the item-row deltas.  Needs
              schedule "strata" or "colored".
``strata_classes``  schedule "strata" only: user-range classes of the plan,
              "auto" (default: 4 for the linear kernel where an item meets
              >= 2 ratings per user range and block, else 1 -- the order
              then trains like the reference's random order, DESIGN.md
              section 3) or 1..4 (1: the fastest plan).
``strata_regroup``  schedule "strata" only: relabelled plans drawn epoch by
              epoch (which users share a range, which items a slab),
              "auto" (default: 2 for the linear kernel's multi-class plans,
              else 1) or 1..4.  Each relabelled plan
              costs device memory: its relabelled user / item ids (8 B per
              rating), its padded copy of the ratings in plan order (4 + 4 +
              itemsize bytes per position) and a second set of P, Q, b_u,
              b_i -- at C3 ~2.4 GB (float32) / 3.1 GB (float64) per plan.
              strata_regroup=1 avoids it (the plan's order then sits
              further from the reference's, section 3.1).
``exchange``  process-group mode only: "rotate" (default; exact -- items are
              cut into one range per rank and the ranges are passed round the
              ring between sub-epochs, so every rating is applied with the
              current user and item rows: a sequential order like the
              single-GPU schedules; which items share a range is redrawn
              each epoch from 8 fixed item relabellings,
              distributed.RotationSet) or "delta" (item-row deltas all-reduced
              once per epoch and applied damped: faster per epoch, item
              updates one epoch late).  DESIGN.md section 6 has both measured.
"""

from __future__ import annotations

import contextlib
from concurrent.futures import ThreadPoolExecutor
from typing import Union

import numpy as np
import pandas as pd

from . import _lib, _prep
from .distributed import EXCHANGES, fit_sharded, world_info
from .engine import (EXACT_GPU_SHUFFLE_MIN, SGDEngine, canonical_dtype, fit_epochs,
                     legacy_permutation_device, resolve_device)
from .recommender_base import RecommenderBase

# fit() inputs from this many rows are narrowed natively (_make_engine)
NATIVE_NARROW_MIN_ROWS = 1 << 20


def _fingerprint(a) -> tuple:
    a = np.ascontiguousarray(a)
    return (a.shape, a.dtype.str, int(_lib.load().mf_fingerprint(a.ctypes.data, a.nbytes)))


def _warn_if_no_device() -> None:
    """Unpickling on a host without a usable GPU stack: the model loads (its
    NumPy attributes are complete) but cannot score.  Say so at load time:
    a serving wrapper that turns predict()'s exception into a default score
    (the reference's project_template/app/api.py:49-52 returns zeros) would
    otherwise hide it."""
    import warnings

    reason = None
    try:
        import torch

        if not torch.cuda.is_available():
            reason = "no HIP device is visible"
    except Exception as e:  # pragma: no cover - torch is a dependency
        reason = f"torch is unavailable ({e})"
    if reason is None:
        try:
            _lib.load()
        except _lib.MFLibraryError as e:
            reason = str(e)
    if reason is not None:
        warnings.warn(f"KernelMF loaded, but {reason}: predict() and recommend() will raise "
                      "MFLibraryError on this host (they run on an AMD Instinct GPU "
                      "through libmf_hip.so); the parameters are plain NumPy attributes",
                      RuntimeWarning, stacklevel=3)


class KernelMF(RecommenderBase):
    """Kernel matrix factorisation, r_ui ~ K(p_u, q_i) with SGD
    (kernel_matrix_factorization.py:19-79).

    Arguments (reference defaults): n_factors=100, n_epochs=100,
    kernel='linear' | 'sigmoid' | 'rbf', gamma='auto' (1/n_factors, rbf
    only), reg=1, lr=0.01, init_mean=0, init_sd=0.1, min_rating=0,
    max_rating=5, verbose=1; plus dtype, schedule, device, distributed,
    exchange (module docstring).
    """

    def __init__(self, n_factors: int = 100, n_epochs: int = 100,
                 kernel: str = "linear", gamma: Union[str, float] = "auto",
                 reg: float = 1, lr: float = 0.01, init_mean: float = 0,
                 init_sd: float = 0.1, min_rating: int = 0, max_rating: int = 5,
                 verbose: int = 1, dtype: str = "float64",
                 schedule: str = "exact", device=None, distributed: bool = False,
                 exchange: str = "rotate", strata_classes="auto", strata_regroup="auto"):
        if kernel not in ("linear", "sigmoid", "rbf"):
            raise ValueError("Kernel must be one of linear, sigmoid, or rbf")
        if schedule not in ("exact", "colored", "strata"):
            raise ValueError("schedule must be 'exact', 'colored' or 'strata'")
        if exchange not in EXCHANGES:
            raise ValueError(f"exchange must be one of {EXCHANGES}")
        if strata_classes != "auto" and strata_classes not in (1, 2, 3, 4):
            raise ValueError("strata_classes must be 'auto' or 1..4")
        if strata_regroup != "auto" and strata_regroup not in (1, 2, 3, 4):
            raise ValueError("strata_regroup must be 'auto' or 1..4")
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
        self.distributed = distributed
        self.exchange = exchange
        self.strata_classes = strata_classes
        self.strata_regroup = strata_regroup

    # ----------------------------------------------------- device state
    def _make_engine(self, X: pd.DataFrame, n_users: int, n_items: int,
                     schedule: str = None, device=None, worker: bool = False) -> SGDEngine:
        """Ratings uploaded, evaluation order built and, for ``schedule``
        "strata" / "colored", the schedule planned (what fit_epochs would
        otherwise do first).

        ``device``: the concrete device, resolved by the CALLER (the current
        device is thread-local: a worker thread would see device 0 whatever
        the caller's ``torch.cuda.set_device``).  ``worker``: built on a
        worker thread -- its copies ran on that thread's current stream of
        ``device``, which is synchronised before the engine is handed back,
        so the caller's stream (e.g. inside ``with torch.cuda.stream(s)``)
        never races them."""
        import torch

        dev = resolve_device(self.device) if device is None else device
        n = len(X)
        cu, ci = X["user_id"], X["item_id"]
        checked = False
        if n >= NATIVE_NARROW_MIN_ROWS and cu.dtype == np.int64 and ci.dtype == np.int64:
            # 10^8-row columns narrowed (and range-checked) on the host
            # threads rather than by NumPy's one-thread casts
            try:
                u = _prep.ids_to_i32(cu.to_numpy(), n_users)
                i = _prep.ids_to_i32(ci.to_numpy(), n_items)
            except _lib.MFLibraryError:
                raise ValueError("rating ids outside [0, n_users) x [0, n_items)") from None
            checked = True
        else:
            u = cu.to_numpy(np.int32) if n else np.zeros(0, np.int32)
            i = ci.to_numpy(np.int32) if n else np.zeros(0, np.int32)
        r = X["rating"].to_numpy(np.float64) if n else np.zeros(0)
        if n >= NATIVE_NARROW_MIN_ROWS and canonical_dtype(self.dtype) == "float32":
            r = _prep.f64_to_f32(r)
        on_gpu = isinstance(dev, torch.device) and dev.type == "cuda"
        with (torch.cuda.device(dev) if on_gpu else contextlib.nullcontext()):
            eng = SGDEngine(u, i, r, n_users, n_items,
                            self.n_factors, self.kernel, self.dtype, dev,
                            gamma=self.gamma, min_rating=self.min_rating,
                            max_rating=self.max_rating, global_mean=self.global_mean,
                            **({"check_ids": False} if checked else {}))
            eng.strata_classes = getattr(self, "strata_classes", "auto")
            eng.strata_regroup = getattr(self, "strata_regroup", "auto")
            if schedule == "strata" and n:
                eng.prepare_strata()
            elif schedule == "colored" and n:
                eng.prepare_colored()
            if worker and on_gpu:
                torch.cuda.current_stream(dev).synchronize()
        return eng

    def _draw_permutation(self, n: int) -> np.ndarray:
        """X.sample(frac=1)'s draw: at 10^8 rows with the shuffle's swaps on
        the GPU (legacy_permutation_device; MF_PREP_GPU_PERM=0: the host),
        the same permutation and RandomState."""
        import os

        import torch

        if (n >= EXACT_GPU_SHUFFLE_MIN and n < (1 << 31)
                and os.environ.get("MF_PREP_GPU_PERM") != "0" and torch.cuda.is_available()):
            return legacy_permutation_device(n, resolve_device(self.device))
        return super()._draw_permutation(n)

    def _sync_params(self, eng: SGDEngine) -> None:
        P, Q, bu, bi = eng.params_numpy()
        self.user_features, self.item_features = P, Q
        self.user_biases, self.item_biases = bu, bi
        self._pred_key = self._param_key()

    # predict / recommend re-check the parameter arrays' bytes on every call
    # (in-place edits are seen, as the reference sees them); False: only a
    # replaced array triggers a re-upload (serving a model nobody edits)
    track_inplace_edits = True

    def _param_key(self):
        """What the device copies were made from: the attribute arrays (by
        identity) and a fingerprint of their bytes, so replaced arrays and
        in-place edits (``model.item_features[3] = ...``, update_users'
        row resets) are both seen -- the reference predicts from the live
        arrays (kernel_matrix_factorization.py:148-160).  The fingerprint
        reads every parameter byte on the host (mf_fingerprint, ~10 GB/s on
        16 threads: ~28 ms per call for a C3 model of 282 MB);
        ``track_inplace_edits = False`` skips it."""
        arrs = (self.user_features, self.item_features, self.user_biases, self.item_biases)
        if not self.track_inplace_edits:
            return arrs, None
        return arrs, tuple(_fingerprint(a) for a in arrs)

    def _predictor(self) -> SGDEngine:
        """Engine holding the current parameters, re-uploaded whenever the
        attribute arrays were replaced or edited since the last upload."""
        eng = getattr(self, "_pred_engine", None)
        key = self._param_key()
        old = getattr(self, "_pred_key", None)
        same = (old is not None and all(a is b for a, b in zip(old[0], key[0]))
                and old[1] == key[1])
        if eng is None or not same:
            eng = SGDEngine(np.zeros(0, np.int32), np.zeros(0, np.int32), np.zeros(0),
                            len(self.user_features), len(self.item_features),
                            self.n_factors, self.kernel, self.dtype, self.device,
                            gamma=self.gamma, min_rating=self.min_rating,
                            max_rating=self.max_rating, global_mean=self.global_mean)
            eng.load_params(self.user_features, self.item_features,
                            self.user_biases, self.item_biases)
            self._pred_engine = eng
            self._pred_key = key
        return eng

    def __getstate__(self):
        # pickles carry plain NumPy state only: they load on a host without a
        # GPU or libmf_hip.so (attributes, get_params, recommend's id maps);
        # predict / recommend need a HIP device (see __setstate__)
        state = self.__dict__.copy()
        state.pop("_pred_engine", None)
        state.pop("_pred_key", None)
        state.pop("_param_ids", None)
        state.pop("_maps_pending", None)
        state.pop("_defer_maps", None)
        return state

    def __setstate__(self, state):
        # build-only arguments added after a pickle was written take their
        # defaults (the reference's pickles have none of them)
        for key, default in (("dtype", "float64"), ("schedule", "exact"), ("device", None),
                             ("distributed", False), ("exchange", "rotate"),
                             ("strata_classes", "auto"), ("strata_regroup", "auto")):
            state.setdefault(key, default)
        self.__dict__.update(state)
        _warn_if_no_device()

    # ------------------------------------------------------------ API
    def fit(self, X: pd.DataFrame, y: pd.Series):
        """kernel_matrix_factorization.py:81-128 (RNG: sample, normal(P),
        normal(Q), then one draw per epoch)."""
        # the user id map may be built on a worker thread beside the rest of
        # fit() (RecommenderBase._fit_maps_native); joined before fit returns
        self._defer_maps = True
        try:
            X = self._preprocess_data(X=X, y=y, type="fit")
        finally:
            self._defer_maps = False
        try:
            return self._fit_prepared(X)
        finally:
            self._join_maps()

    def _fit_prepared(self, X: pd.DataFrame):
        """fit() after _preprocess_data: initial draws, device epochs."""
        self.global_mean = X["rating"].mean()
        self.user_biases = np.zeros(self.n_users)
        self.item_biases = np.zeros(self.n_items)
        sharded = self.distributed and world_info()[0] > 1
        fut = None
        with ThreadPoolExecutor(1) as ex:
            if not sharded:
                # the device side (upload, evaluation order, schedule plan)
                # is built on a worker thread while this one draws the
                # initial factors: the worker draws nothing, so the RNG
                # stream is the reference's (sample, normal P, normal Q)
                fut = ex.submit(self._make_engine, X, self.n_users, self.n_items,
                                self.schedule, resolve_device(self.device), True)
            self.user_features = np.random.normal(self.init_mean, self.init_sd,
                                                  (self.n_users, self.n_factors))
            self.item_features = np.random.normal(self.init_mean, self.init_sd,
                                                  (self.n_items, self.n_factors))
            eng = fut.result() if fut is not None else None
        if sharded:
            n = len(X)
            P, Q, bu, bi, rmse, _ = fit_sharded(
                X["user_id"].to_numpy(np.int32), X["item_id"].to_numpy(np.int32),
                X["rating"].to_numpy(np.float64), self.n_users, self.n_items,
                self.user_features, self.item_features, self.user_biases, self.item_biases,
                self.n_epochs, self.kernel, self.n_factors, self.dtype, self.device, self.gamma,
                self.min_rating, self.max_rating, self.global_mean, self.lr, self.reg,
                self.schedule, verbose=self.verbose, exchange=self.exchange) if n else (
                self.user_features, self.item_features, self.user_biases, self.item_biases,
                [float("nan")] * self.n_epochs, None)
            self.user_features, self.item_features = P, Q
            self.user_biases, self.item_biases = bu, bi
            self.train_rmse = rmse
            self._pred_engine = None
            return self
        eng.load_params(self.user_features, self.item_features,
                        self.user_biases, self.item_biases)
        self.train_rmse = fit_epochs(eng, self.n_epochs, self.schedule, self.lr,
                                     self.reg, verbose=self.verbose)
        self._sync_params(eng)
        self._pred_engine = eng
        return self

    def predict(self, X: pd.DataFrame, bound_ratings: bool = True) -> list:
        """kernel_matrix_factorization.py:130-163.  Scores on the GPU from
        device copies of the parameters, refreshed when the attribute arrays
        were replaced or edited in place since the last call (a host pass
        over the parameters per call, see _param_key; set
        ``track_inplace_edits = False`` on a model that is not edited to skip
        it)."""
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
        # n_users is not updated by update_users (the reference's quirk,
        # :213-235): the engine takes the row counts of the arrays
        eng = self._make_engine(X, len(self.user_features), len(self.item_features))
        eng.load_params(self.user_features, self.item_features,
                        self.user_biases, self.item_biases)
        self.train_rmse = fit_epochs(eng, n_epochs, self.schedule, lr, self.reg,
                                     update_user=True, update_item=False,
                                     verbose=verbose)
        self._sync_params(eng)
        self._pred_engine = eng

    def recommend_batch(self, users, amount: int = 10, exclude_known=None,
                        bound_ratings: bool = True) -> pd.DataFrame:
        """Top ``amount`` items for many users on the GPU (mf_topk) -- the
        batched form of ``recommend`` (recommender_base.py:214-271).

        ``exclude_known``: optional DataFrame[user_id, item_id] of pairs to
        skip (recommend's ``items_known`` per user), passed to the device as
        a CSR list.  Scores are recommend()'s (the unbounded prediction);
        equal scores rank the lower internal item id first -- the order a
        stable sort gives; the reference's ``sort_values`` default quicksort
        leaves tie order unspecified.  Users go in chunks (engine
        ``topk_ws_budget``).  Returns DataFrame[user_id, item_id,
        rating_pred] ordered by user then rank."""
        users = list(users)
        uid = self._remap(pd.Series(users, dtype=object), self.user_id_map)
        ex_ptr = ex_items = None
        if exclude_known is not None and len(exclude_known):
            pos = pd.Series(np.arange(len(users)), index=pd.Index(users, dtype=object))
            pos = pos[~pos.index.duplicated(keep="first")]
            q = exclude_known["user_id"].map(pos)
            it = self._remap(exclude_known["item_id"], self.item_id_map)
            ok = q.notna().to_numpy() & (it >= 0)
            qv = q[ok].to_numpy().astype(np.int64)
            iv = it[ok].astype(np.int32)
            # duplicate users in `users` share the first position's list
            first = pos.reindex(pd.Index(users, dtype=object)).to_numpy().astype(np.int64)
            order = np.argsort(qv, kind="stable")
            qv, iv = qv[order], iv[order]
            cnt = np.bincount(qv, minlength=len(users)).astype(np.int64)
            start = np.concatenate([[0], np.cumsum(cnt)])
            per = [iv[start[f]:start[f + 1]] for f in first]
            ex_ptr = np.concatenate([[0], np.cumsum([len(x) for x in per])]).astype(np.int64)
            ex_items = (np.concatenate(per) if len(per) else np.zeros(0)).astype(np.int32)
        amount = min(amount, self.n_items)
        items, scores = self._predictor().topk(uid, amount, ex_ptr, ex_items)
        inv = np.asarray(list(self.item_id_map.keys()), dtype=object)
        valid = items >= 0
        out = pd.DataFrame({
            "user_id": np.repeat(np.asarray(users, dtype=object), valid.sum(axis=1)),
            "item_id": inv[items[valid]],
            "rating_pred": scores[valid],
        })
        if bound_ratings:
            out["rating_pred"] = out["rating_pred"].clip(lower=self.min_rating,
                                                         upper=self.max_rating)
        return out

"""CPU tests of the host side: C-ABI exports, schedulers, estimator logic.

No GPU: the estimator flows (RNG order, id maps, update_users bookkeeping,
batch schedules) run here against a test double of the device engine whose
sweeps are the CPU oracle.  The double exists only in this file; the product
path has no CPU fallback (see test_product_has_no_cpu_path).
"""

import ctypes
import os
import re

import numpy as np
import pandas as pd
import pytest

import oracle
from conftest import ROOT, golden_hp, load_golden

HEADER = os.path.join(ROOT, "include", "mf_hip.h")


# ---------------------------------------------------------------- C ABI
def _declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[A-Za-z_][\w\s\*]*?\b(mf_\w+)\s*\(", text, flags=re.M)
    return sorted(set(names))


def test_library_exports_every_declared_symbol():
    from matrix_factorization import _lib

    lib = _lib.load()
    declared = _declared_functions()
    assert len(declared) >= 15
    for name in declared:
        assert hasattr(lib, name), f"{name} not exported by libmf_hip.so"
    # the Python binding covers the header one to one
    assert sorted(_lib.SIGNATURES) == declared
    assert lib.mf_abi_version() == 1
    assert lib.mf_max_factors() == 1024


def test_library_errors_are_reported():
    from matrix_factorization import _lib

    lib = _lib.load()
    offs = np.array([0, 5], np.int64)
    # n_factors out of range -> MF_ERR_INVALID before any device work
    rc = lib.mf_sgd_epoch(None, None, None, 0, None, offs.ctypes.data_as(ctypes.c_void_p),
                          1, None, 0, 0.0, None, None, None, None, 0, 0, 4096, 0, 0, 0.0,
                          0.01, 0.02, 0.0, 5.0, 1, 1, 0, None, 0, None, None)
    assert rc == 1 and "batch_offsets" in _lib.last_error() or "n_factors" in _lib.last_error()
    with pytest.raises(_lib.MFLibraryError):
        _lib.call("mf_predict", None, None, -1, 0.0, None, None, None, None, 8, 0, 0, 0.0,
                  0.0, 5.0, 1, None, None)


# ------------------------------------------------------------ schedulers
def _random_ratings(seed, nu, ni, nnz):
    rs = np.random.RandomState(seed)
    keys = rs.choice(nu * ni, nnz, replace=False)
    return (keys // ni).astype(np.int32), (keys % ni).astype(np.int32), \
        rs.randint(1, 6, nnz).astype(np.float64)


def test_levels_reproduce_the_sequential_sweep_bit_for_bit():
    from matrix_factorization.engine import sched_levels

    nu, ni, nnz, k = 60, 45, 1500, 8
    u, i, r = _random_ratings(0, nu, ni, nnz)
    rs = np.random.RandomState(1)
    order = rs.permutation(nnz).astype(np.int64)
    P = rs.normal(0, 0.1, (nu, k)); Q = rs.normal(0, 0.1, (ni, k))
    bu = np.zeros(nu); bi = np.zeros(ni)
    args = dict(kernel="sigmoid", lr=0.05, reg=0.02, min_rating=1, max_rating=5)
    ref = [a.copy() for a in (bu, bi, P, Q)]
    oracle.sgd_pass(u, i, r, 3.0, *ref, order=order, **args)
    sched, offs = sched_levels(u, i, order, nu, ni)
    assert np.array_equal(np.sort(sched), np.arange(nnz))
    got = [a.copy() for a in (bu, bi, P, Q)]
    for b in range(len(offs) - 1):
        lvl = sched[offs[b]:offs[b + 1]]
        assert len(np.unique(u[lvl])) == len(lvl) and len(np.unique(i[lvl])) == len(lvl)
        # inside a level any order gives the same result: use a reversed one
        oracle.sgd_pass(u, i, r, 3.0, *got, order=lvl[::-1].astype(np.int64), **args)
    for a, b in zip(got, ref):
        assert np.array_equal(a, b)


def test_levels_user_only_for_frozen_items():
    from matrix_factorization.engine import sched_levels

    u, i, r = _random_ratings(2, 30, 20, 300)
    order = np.random.RandomState(0).permutation(300)
    s_full, o_full = sched_levels(u, i, order, 30, 20, True, True)
    s_user, o_user = sched_levels(u, i, order, 30, 20, True, False)
    assert len(o_user) - 1 == np.bincount(u).max()
    assert len(o_user) <= len(o_full)


def test_color_schedule_is_a_conflict_free_partition():
    from matrix_factorization.engine import sched_color

    nu, ni = 400, 150
    u, i, r = _random_ratings(3, nu, ni, 20000)
    sched, offs = sched_color(u, i, nu, ni)
    assert np.array_equal(np.sort(sched), np.arange(len(u)))
    assert len(offs) - 1 <= np.bincount(u).max() + np.bincount(i).max() - 1
    for b in range(len(offs) - 1):
        c = sched[offs[b]:offs[b + 1]]
        assert len(np.unique(u[c])) == len(c)
        assert len(np.unique(i[c])) == len(c)
        assert np.all(np.diff(i[c]) > 0)          # item-sorted inside a colour


def test_schedulers_reject_bad_ids():
    from matrix_factorization import _lib
    from matrix_factorization.engine import sched_color, sched_levels

    u = np.array([0, 5], np.int32)
    i = np.array([0, 1], np.int32)
    with pytest.raises(_lib.MFLibraryError):
        sched_levels(u, i, None, 3, 3)
    with pytest.raises(_lib.MFLibraryError):
        sched_color(u, i, 3, 3)


def test_schedulers_handle_empty_input():
    from matrix_factorization.engine import sched_color, sched_levels

    e = np.zeros(0, np.int32)
    s, o = sched_levels(e, e, None, 0, 0)
    assert len(s) == 0 and list(o) == [0]
    s, o = sched_color(e, e, 0, 0)
    assert len(s) == 0 and list(o) == [0]


# ------------------------------------------------- estimator host logic
class OracleEngine:
    """Test double of engine.SGDEngine: same interface, oracle sweeps."""

    def __init__(self, u, i, r, n_users, n_items, n_factors, kernel, dtype="float64",
                 device=None, gamma=0.0, min_rating=0.0, max_rating=5.0, global_mean=0.0):
        self.u_host = np.ascontiguousarray(u, np.int32)
        self.i_host = np.ascontiguousarray(i, np.int32)
        self.r_host = np.ascontiguousarray(r, np.float64)
        self.n = len(u)
        self.n_users, self.n_items, self.k = n_users, n_items, n_factors
        self.kernel, self.gamma = kernel, gamma
        self.min_rating, self.max_rating = min_rating, max_rating
        self.global_mean = global_mean
        self.colored = None
        self.sse = {}
        self.P = self.Q = self.bu = self.bi = None

    def load_params(self, P=None, Q=None, bu=None, bi=None):
        if P is not None:
            self.P = np.array(P, np.float64).reshape(self.n_users, self.k)
        if Q is not None:
            self.Q = np.array(Q, np.float64).reshape(self.n_items, self.k)
        if bu is not None:
            self.bu = np.array(bu, np.float64)
        if bi is not None:
            self.bi = np.array(bi, np.float64)

    def params_numpy(self):
        return tuple(None if a is None else a.copy() for a in (self.P, self.Q, self.bu, self.bi))

    def _kw(self):
        return dict(kernel=self.kernel, gamma=self.gamma, min_rating=self.min_rating,
                    max_rating=self.max_rating)

    def epoch_exact(self, order, lr, reg, update_user=True, update_item=True):
        from matrix_factorization.engine import sched_levels, sched_levels_chunked

        if order.dtype == np.int32:      # the product's path: chunked levels (3 chunks)
            sched, offs = sched_levels_chunked(self.u_host, self.i_host, order, self.n_users,
                                               self.n_items, update_user, update_item,
                                               n_chunks=3)
        else:
            sched, offs = sched_levels(self.u_host, self.i_host, order, self.n_users,
                                       self.n_items, update_user, update_item)
        for b in range(len(offs) - 1):
            lvl = sched[offs[b]:offs[b + 1]].astype(np.int64)
            if self.kernel == "bias":
                oracle.bias_sgd_pass(self.u_host, self.i_host, self.r_host, self.global_mean,
                                     self.bu, self.bi, lr, reg, order=lvl,
                                     update_user=update_user, update_item=update_item)
            else:
                oracle.sgd_pass(self.u_host, self.i_host, self.r_host, self.global_mean,
                                self.bu, self.bi, self.P, self.Q, lr=lr, reg=reg, order=lvl,
                                update_user=update_user, update_item=update_item,
                                **self._kw())

    def sse_async(self, slot):
        if self.kernel == "bias":
            self.sse[slot] = oracle.bias_sse(self.u_host, self.i_host, self.r_host,
                                             self.global_mean, self.bu, self.bi)
        else:
            self.sse[slot] = oracle.sse(self.u_host, self.i_host, self.r_host,
                                        self.global_mean, self.bu, self.bi, self.P, self.Q,
                                        **self._kw())

    def rmse_values(self, n):
        if self.n == 0:
            return [float("nan")] * n
        return [float(np.sqrt(self.sse[s] / self.n)) for s in range(n)]

    def predict(self, u, i, bound):
        if self.kernel == "bias":
            out = []
            for a, b in zip(u, i):
                p = self.global_mean
                if a != -1:
                    p += self.bu[a]
                if b != -1:
                    p += self.bi[b]
                if bound:
                    p = min(max(p, self.min_rating), self.max_rating) if (
                        p > self.max_rating or p < self.min_rating) else p
                out.append(p)
            return np.array(out)
        return oracle.predict(u, i, self.global_mean, self.bu, self.bi, self.P, self.Q,
                              bound=bound, **self._kw())


@pytest.fixture
def cpu_engine(monkeypatch):
    import matrix_factorization.baseline_model as bm
    import matrix_factorization.kernel_matrix_factorization as kmf

    monkeypatch.setattr(kmf, "SGDEngine", OracleEngine)
    monkeypatch.setattr(kmf, "resolve_device", lambda device=None: device)
    monkeypatch.setattr(bm, "SGDEngine", OracleEngine)
    return OracleEngine


@pytest.mark.parametrize("name", ["tiny_linear", "tiny_sigmoid", "tiny_rbf", "tiny_defaults",
                                  "mid_k100", "c1_linear"])
def test_kernelmf_host_flow_matches_reference(cpu_engine, name, capsys):
    # c1_linear (80K ratings >= FAST_PREP_MIN_ROWS) takes the native
    # preprocessing path, its user id map built beside the epochs
    from matrix_factorization import KernelMF

    d = load_golden(name)
    hp = golden_hp(d)
    X = pd.DataFrame({"user_id": d["user_id"], "item_id": d["item_id"]})
    np.random.seed(int(d["seed"]))
    m = KernelMF(**hp).fit(X, pd.Series(d["rating"]))
    out = capsys.readouterr().out
    if hp.get("verbose", 1) == 1:
        assert out.count("Epoch ") == hp["n_epochs"]
    assert list(m.user_id_map) == d["user_ids"].tolist()
    assert list(m.item_id_map) == d["item_ids"].tolist()
    for key in ("user_features", "item_features", "user_biases", "item_biases"):
        assert np.max(np.abs(getattr(m, key) - d[key])) < 1e-12, key
    assert np.max(np.abs(np.asarray(m.train_rmse) - d["train_rmse"])) < 1e-13
    T = pd.DataFrame({"user_id": d["test_user"], "item_id": d["test_item"]})
    assert np.max(np.abs(np.asarray(m.predict(T)) - d["pred_bound"])) < 1e-12
    assert m.predictions_possible == d["pred_possible"].tolist()
    df = X.assign(rating=d["rating"])
    for j, user in enumerate(d["rec_users"]):
        known = df.loc[df.user_id == user, "item_id"].to_numpy()
        known = known[: len(known) // 2] if j % 2 == 0 else None
        rec = m.recommend(user=user, amount=10, items_known=known)
        assert rec["item_id"].tolist() == d["rec_items"][j].tolist()


def test_update_users_host_flow_matches_reference(cpu_engine):
    from matrix_factorization import KernelMF, train_update_test_split

    d = load_golden("update_users")
    hp = golden_hp(d)
    df = pd.DataFrame({"user_id": d["user_id"], "item_id": d["item_id"],
                       "rating": d["rating"]})
    np.random.seed(int(d["seed"]))
    Xi, yi, Xu, yu, Xt, yt = train_update_test_split(df, frac_new_users=0.25)
    assert Xi.index.tolist() == d["split_train_index"].tolist()
    assert Xu.index.tolist() == d["split_update_index"].tolist()
    assert Xt.index.tolist() == d["split_test_index"].tolist()
    m = KernelMF(**hp).fit(Xi, yi)
    extra = Xi.loc[d["extra_index"]]
    Q_before = m.item_features.copy()
    m.update_users(pd.concat([Xu, extra]), pd.concat([yu, yi.loc[extra.index]]),
                   lr=0.03, n_epochs=5, verbose=0)
    assert list(m.user_id_map.values()) == d["user_id_vals"].tolist()
    assert m.n_users == d["n_users"]
    assert np.max(np.abs(m.user_features - d["user_features"])) < 1e-12
    assert np.array_equal(m.item_features, Q_before)          # frozen bit for bit
    assert np.max(np.abs(m.item_features - d["fit_item_features"])) < 1e-12
    assert np.max(np.abs(np.asarray(m.predict(Xt)) - d["pred_test"])) < 1e-12


@pytest.mark.parametrize("method", ["sgd"])
def test_baseline_host_flow_matches_reference(cpu_engine, method):
    from matrix_factorization import BaselineModel

    d = load_golden(f"baseline_{method}")
    hp = golden_hp(d)
    X = pd.DataFrame({"user_id": d["user_id"], "item_id": d["item_id"]})
    np.random.seed(int(d["seed"]))
    m = BaselineModel(**hp).fit(X, pd.Series(d["rating"]))
    assert np.array_equal(m.user_biases, d["user_biases"])
    assert np.array_equal(m.item_biases, d["item_biases"])
    np.random.seed(int(d["seed"]) + 1)
    m.update_users(pd.DataFrame({"user_id": d["upd_user"], "item_id": d["upd_item"]}),
                   pd.Series(d["upd_rating"]), lr=0.05, n_epochs=3)
    assert np.array_equal(m.user_biases, d["upd_user_biases"])


def test_duplicate_ratings_rejected():
    from matrix_factorization import KernelMF

    X = pd.DataFrame({"user_id": [1, 1], "item_id": [2, 2]})
    with pytest.raises(ValueError, match="Duplicate"):
        KernelMF(verbose=0).fit(X, pd.Series([3.0, 4.0]))


def test_constructor_validation_and_sklearn_clone():
    from sklearn.base import clone

    from matrix_factorization import BaselineModel, KernelMF

    with pytest.raises(ValueError, match="Kernel must be"):
        KernelMF(kernel="poly")
    with pytest.raises(ValueError):
        BaselineModel(method="gd")
    m = KernelMF(n_factors=8, gamma="auto", kernel="rbf", dtype="float32", schedule="colored")
    assert m.gamma == 1 / 8
    c = clone(m)
    assert c.get_params() == m.get_params()
    assert c.dtype == "float32" and c.schedule == "colored"
    assert m.strata_classes == "auto" and clone(KernelMF(strata_classes=2)).strata_classes == 2
    with pytest.raises(ValueError, match="strata_classes"):
        KernelMF(strata_classes=5)
    assert m.strata_regroup == "auto" and clone(KernelMF(strata_regroup=1)).strata_regroup == 1
    with pytest.raises(ValueError, match="strata_regroup"):
        KernelMF(strata_regroup=0)


def test_auto_classes_rule():
    """SGDEngine.auto_classes: 4 user-range classes for the linear kernel
    where an item meets >= 2 ratings per user range of the one-class plan
    (C3: 100M / (100K items x B 256) = 3.9), else 1 (sigmoid / rbf, sparse
    blocks, the bias model)."""
    from types import SimpleNamespace

    from matrix_factorization.engine import SGDEngine

    def eng(kernel, n, n_items):
        return SimpleNamespace(kernel=kernel, n=n, n_items=n_items,
                               AUTO_CLASSES=SGDEngine.AUTO_CLASSES,
                               AUTO_CLASSES_MIN_DEGREE=SGDEngine.AUTO_CLASSES_MIN_DEGREE)

    assert SGDEngine.auto_classes(eng("linear", 100_000_000, 100_000), 256) == 4
    assert SGDEngine.auto_classes(eng("sigmoid", 5_000_000, 10_000), 69) == 1
    assert SGDEngine.auto_classes(eng("linear", 1_000_000, 100_000), 256) == 1
    assert SGDEngine.auto_classes(eng("bias", 100_000_000, 100_000), 256) == 1


def test_product_has_no_cpu_path(monkeypatch):
    """Without a GPU the product path raises instead of computing on the CPU."""
    import torch

    from matrix_factorization import KernelMF, _lib

    if torch.cuda.is_available():
        pytest.skip("GPU visible")
    X = pd.DataFrame({"user_id": [1, 2], "item_id": [2, 3]})
    with pytest.raises(_lib.MFLibraryError, match="no HIP device"):
        KernelMF(verbose=0, n_epochs=1).fit(X, pd.Series([3.0, 4.0]))


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    from matrix_factorization import _lib

    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "nope.so"))
    with pytest.raises(_lib.MFLibraryError, match="not found"):
        _lib.load()


def test_slice_order_groups_items_then_users():
    from matrix_factorization.engine import sched_slices

    nu, ni = 200, 64
    u, i, r = _random_ratings(5, nu, ni, 5000)
    sched, offs = sched_slices(u, i, nu, ni, 8)
    assert np.array_equal(np.sort(sched), np.arange(len(u)))
    assert offs[0] == 0 and offs[-1] == len(u) and len(offs) == 9
    for x in range(8):
        seg = sched[offs[x]:offs[x + 1]]
        assert np.all(i[seg] * 8 // ni == x)          # one item slice
        assert np.all(np.diff(u[seg]) >= 0)           # user-sorted inside it


# ------------------------------------------------------------ strata plan
def test_tile_order_chunks_users_and_slices_items():
    """mf_sched_tiles (the FP64 RMSE pass's evaluation order): (1, S) is
    mf_sched_slices(S) exactly; tile c * S + s holds the ratings of user
    chunk c (contiguous id ranges of about equal rating counts) and item
    slice s, users ascending (stable) inside a tile."""
    from matrix_factorization.engine import sched_slices, sched_tiles

    rs = np.random.RandomState(5)
    nu, ni, n = 3000, 700, 60000
    u = rs.randint(0, nu, n).astype(np.int32)
    i = rs.randint(0, ni, n).astype(np.int32)
    a, oa = sched_slices(u, i, nu, ni, 8)
    b, ob = sched_tiles(u, i, nu, ni, 1, 8)
    assert np.array_equal(a, b) and np.array_equal(oa, ob)
    C, S = 4, 16
    t, ot = sched_tiles(u, i, nu, ni, C, S)
    assert np.array_equal(np.sort(t), np.arange(n)) and ot[0] == 0 and ot[-1] == n
    chunk_hi = []
    for c in range(C):
        for s_ in range(S):
            rows = t[ot[c * S + s_]:ot[c * S + s_ + 1]]
            assert np.all(i[rows] * S // ni == s_)
            assert np.all(np.diff(u[rows]) >= 0)
            eq = np.diff(u[rows]) == 0                     # stable inside a user
            assert np.all(np.diff(rows)[eq] > 0)
        rows = t[ot[c * S]:ot[(c + 1) * S]]
        chunk_hi.append((u[rows].min(), u[rows].max(), len(rows)))
    for c in range(C - 1):
        assert chunk_hi[c][1] < chunk_hi[c + 1][0]         # contiguous user ranges
    sizes = np.array([x[2] for x in chunk_hi])
    assert sizes.max() - sizes.min() < 0.02 * n
    from matrix_factorization import _lib
    with pytest.raises(_lib.MFLibraryError):
        sched_tiles(u, i, nu, ni, 16, 16)                  # > 128 tiles


@pytest.mark.parametrize("B,NS,C", [(1, 32, 1), (3, 16, 1), (8, 128, 1), (1, 32, 2),
                                    (3, 16, 2), (8, 64, 3), (5, 32, 4)])
def test_strata_plan_is_valid(B, NS, C):
    """mf_strata_plan_build_classes: every rating placed once; block (s, w),
    s < C*B, holds user range (s + C*w) mod C*B x item range w (C = 1: the
    plain plan, (w+s) mod B); a step holds each slot and each item at most
    once; every user of a block stays on one slot; the block has exactly
    D = max(slot load, item degree) steps (Koenig colouring)."""
    from matrix_factorization import engine as E

    rs = np.random.RandomState(0)
    nu, ni, n = 1500, 300, 30000
    keys = rs.choice(nu * ni, n, replace=False)
    u = (keys // ni).astype(np.int32)
    i = (keys % ni).astype(np.int32)
    ub = E.balanced_bounds(u, nu, C * B)
    ib = E.balanced_bounds(i, ni, B)
    sched, bstep = E.sched_strata(u, i, nu, ni, B, ub, ib, NS, C)
    assert len(bstep) == C * B * B + 1
    assert len(sched) == bstep[-1] * NS
    valid = sched[sched >= 0]
    assert np.array_equal(np.sort(valid), np.arange(n))
    for s in range(C * B):
        for w in range(B):
            blk = s * B + w
            nst = bstep[blk + 1] - bstep[blk]
            grid = sched[bstep[blk] * NS:bstep[blk + 1] * NS].reshape(nst, NS)
            ubk = (s + C * w) % (C * B)
            assert ubk % C == s % C                 # stratum s: class s mod C only
            js = grid[grid >= 0]
            assert np.all((u[js] >= ub[ubk]) & (u[js] < ub[ubk + 1]))
            assert np.all((i[js] >= ib[w]) & (i[js] < ib[w + 1]))
            owner = {}
            load = np.zeros(NS, np.int64)
            for t in range(nst):
                row = grid[t]
                on = row >= 0
                items = i[row[on]]
                assert len(set(items)) == len(items)          # item once per step
                for slot in np.nonzero(on)[0]:
                    user = int(u[row[slot]])
                    assert owner.setdefault(user, slot) == slot   # one slot per user
                    load[slot] += 1
            if len(js):
                D = max(load.max(), np.bincount(i[js]).max())
                assert nst == D
            else:
                assert nst == 0


def test_strata_plans_are_pinned():
    """The planner's output (sched + block step offsets) on skewed inputs is
    the one it had before the one-pass rewrite of round 5 (tools/plan_hash.py:
    the same sha256 from the two-pass build, here and on the GPU box's host;
    C3 at full scale is pinned there too).  Any change to the planner that
    moves a rating shows up here."""
    import hashlib

    from matrix_factorization import engine as E

    want = ["4e332a691e1ae04ad6782bf0ae7301f64c2cb4f38f703cf6dce9819863f05c25",
            "a150593315c716afb5c326d8874e69025f626ba8b2767d77a4d674dce57b4609",
            "6eecfc3dd146cb5c5d8065c4684ed33ee1794b5d87bee70acbef2ff4bd6a0269",
            "607bf684bd7297f2a93fe1367c79178d662f2881b0fe59f48e734a31fd337fd3"]
    rng = np.random.default_rng(7)
    got = []
    for (nu, ni, n, B, C, ns) in [(500, 300, 20000, 8, 1, 64), (500, 300, 20000, 8, 3, 32),
                                  (40000, 9000, 600000, 32, 4, 128),
                                  (40000, 9000, 600000, 48, 2, 256)]:
        u = rng.integers(0, nu, n).astype(np.int32)
        i = np.minimum((rng.pareto(1.2, n) * 50).astype(np.int64), ni - 1).astype(np.int32)
        sched, bstep = E.sched_strata(u, i, nu, ni, B, E.balanced_bounds(u, nu, C * B),
                                      E.balanced_bounds(i, ni, B), ns, C)
        h = hashlib.sha256(sched.tobytes())
        h.update(bstep.tobytes())
        got.append(h.hexdigest())
    assert got == want


@pytest.mark.parametrize("n,shapes", [(20000, [(128, 16), (64, 8)]), (20000, [(64, 16), (32, 8)]),
                                      (200000, [(128, 16), (64, 8)]),
                                      (200000, [(64, 16), (32, 8)]), (3000, [(64, 16)]),
                                      (-400000, [(64, 16), (32, 8)]),
                                      (-400000, [(128, 16), (64, 8)])])
def test_strata_plan_pick_is_the_rule_over_full_plans(n, shapes):
    """mf_strata_plan_build_pick (step counts without colouring, only the pick
    coloured) returns the shape and the plan that building every shape in
    full and keeping the least steps * waves returns (the 16-wave one
    outright at >= 70 % fill) -- SGDEngine._build_plan's rule before."""
    from matrix_factorization import engine as E

    # n < 0: |n| ratings in 4 x 4 dense blocks of uniform items (plans of
    # >= 70 % fill, so the 16-wave shape is taken outright); else skewed
    # items in 16 x 8 sparse blocks
    rng = np.random.default_rng(abs(n) + len(shapes) + shapes[0][0])
    dense, n = n < 0, abs(n)
    nu, ni, B, C = (3000, 2000, 4, 1) if dense else (3000, 2000, 8, 2)
    u = rng.integers(0, nu, n).astype(np.int32)
    i = (rng.integers(0, ni, n) if dense else
         np.minimum((rng.pareto(1.5, n) * 200).astype(np.int64), ni - 1)).astype(np.int32)
    ub, ib = E.balanced_bounds(u, nu, C * B), E.balanced_bounds(i, ni, B)
    for fill_stop in (0.7, 0.0):
        best = None
        for j, (ns, wv) in enumerate(shapes):
            sched, bstep = E.sched_strata(u, i, nu, ni, B, ub, ib, ns, C)
            cost = int(bstep[-1]) * wv
            if best is None or cost < best[0]:
                best = (cost, j, sched, bstep)
            if j == 0 and fill_stop and n / max(len(sched), 1) >= fill_stop:
                break
        sched, bstep, j = E.sched_strata_pick(u, i, nu, ni, B, ub, ib, shapes, C, fill_stop)
        if dense and fill_stop:
            assert j == 0 and n / len(sched) >= fill_stop
        assert j == best[1]
        assert np.array_equal(sched, best[2]) and np.array_equal(bstep, best[3])


def test_strata_serial_order_and_rejections():
    from matrix_factorization import _lib
    from matrix_factorization import engine as E

    u = np.array([0, 0, 1, 2, 2, 3], np.int32)
    i = np.array([0, 1, 1, 0, 2, 2], np.int32)
    ub = np.array([0, 2, 4], np.int32)
    ib = np.array([0, 1, 3], np.int32)
    sched, bstep = E.sched_strata(u, i, 4, 3, 2, ub, ib, 4)
    plan = E.StrataPlan(2, 4, ub, ib, bstep, sched)
    order = plan.serial_order([1, 0], 12345)
    assert np.array_equal(np.sort(order), np.arange(6))
    # stratum 1 first: its ratings come before stratum 0's
    sizes = plan.stratum_sizes()
    assert sizes.sum() == 6
    s1 = sched[bstep[2] * 4:bstep[4] * 4]
    assert set(order[: sizes[1]]) == set(s1[s1 >= 0])
    with pytest.raises(_lib.MFLibraryError):
        E.sched_strata(u, i, 4, 3, 2, np.array([0, 3, 2], np.int32), ib, 4)
    with pytest.raises(_lib.MFLibraryError):
        E.sched_strata(u, i, 4, 3, 2, ub, ib, 0)
    assert E.strata_mix(0, 0) == 0 and E.strata_mix(1, 2) != E.strata_mix(2, 1)
    # slots per step follow the kernel's row layout
    assert E.strata_slots(64, _lib.MF_F32) == 128
    assert E.strata_slots(16, _lib.MF_F32) == 256
    assert E.strata_slots(64, _lib.MF_F64) == 64          # one slot per group (FP64 rows)
    assert _lib.load().mf_strata_slots(-1, 0) == -1


@pytest.mark.parametrize("C", [1, 2, 3, 4])
def test_stratum_order_cycles_classes(C):
    """stratum_order with C user-range classes: a permutation of the C*B
    strata that deals the classes round-robin (what the persistent kernel's
    C-positions-back wait needs: a user range is used again exactly C
    positions later); C = 1 draws exactly rs.permutation(B), as before."""
    from types import SimpleNamespace

    from matrix_factorization.engine import stratum_order

    B = 7
    seq = stratum_order(np.random.RandomState(3), SimpleNamespace(B=B, classes=C))
    assert seq.dtype == np.int32 and np.array_equal(np.sort(seq), np.arange(C * B))
    cls = seq % C
    assert len(set(cls[:C])) == C
    assert np.all(cls == cls[np.arange(C * B) % C])
    if C == 1:
        assert np.array_equal(seq, np.random.RandomState(3).permutation(B))
    # the serial order of a classes plan: every rating once, stratum by stratum
    from matrix_factorization import engine as E

    rs = np.random.RandomState(1)
    nu, ni, n = 400, 90, 4000
    keys = rs.choice(nu * ni, n, replace=False)
    u = (keys // ni).astype(np.int32)
    i = (keys % ni).astype(np.int32)
    ub, ib = E.balanced_bounds(u, nu, C * B), E.balanced_bounds(i, ni, B)
    sched, bstep = E.sched_strata(u, i, nu, ni, B, ub, ib, 16, C)
    plan = E.StrataPlan(B, 16, ub, ib, bstep, sched, C)
    assert plan.n_strata == C * B and len(plan.stratum_sizes()) == C * B
    order = plan.serial_order(seq, 99)
    assert np.array_equal(np.sort(order), np.arange(n))


def test_phased_strata_host_composition():
    """PhasedStrata (item phases, host side): the epoch's serial order is the
    phases' serial orders mapped back to global rating indices, phase 0
    first; it lists every rating once; stratum sizes add up per stratum."""
    from matrix_factorization.engine import (PhasedStrata, StrataPlan, balanced_bounds,
                                             sched_strata)

    rs = np.random.RandomState(5)
    nu, ni, n, B, NS = 300, 240, 6000, 4, 64
    keys = rs.choice(nu * ni, n, replace=False)
    u = (keys // ni).astype(np.int32)
    i = (keys % ni).astype(np.int32)
    ilo = balanced_bounds(i, ni, 2).astype(np.int64)
    plans, idx = [], []
    for p in range(2):
        ix = np.flatnonzero((i >= ilo[p]) & (i < ilo[p + 1]))
        ui, ii = u[ix], i[ix] - int(ilo[p])
        nip = int(ilo[p + 1] - ilo[p])
        ub, ib = balanced_bounds(ui, nu, B), balanced_bounds(ii, nip, B)
        sched, bstep = sched_strata(ui, ii, nu, nip, B, ub, ib, NS)
        plans.append(StrataPlan(B, NS, ub, ib, bstep, sched))
        idx.append(ix)
    ph = PhasedStrata(plans, idx, ilo)
    seq = np.array([2, 0, 3, 1], np.int32)
    order = ph.serial_order(seq, 77)
    assert np.array_equal(np.sort(order), np.arange(n))
    n0 = len(idx[0])
    assert np.all(i[order[:n0]] < ilo[1]) and np.all(i[order[n0:]] >= ilo[1])
    assert np.array_equal(order[:n0], idx[0][plans[0].serial_order(seq, 77)])
    assert np.array_equal(ph.stratum_sizes(), plans[0].stratum_sizes() + plans[1].stratum_sizes())
    assert ph.n_positions == plans[0].n_positions + plans[1].n_positions
    assert ph.B == B and ph.NS == NS


def test_deep_pipe_default_by_plan_shape(monkeypatch):
    """MF_FLAG_DEEP_PIPE by plan shape: on for 8-wave plans and for 16-wave
    plans filled below 70 %, off for well-filled 16-wave plans and for the
    narrow kernels; MF_STRATA_DEEP / strata_deep_pipe override."""
    from types import SimpleNamespace

    from matrix_factorization.engine import SGDEngine, strata_slots

    monkeypatch.delenv("MF_STRATA_DEEP", raising=False)
    k, dcode = 64, 0
    ns16, ns8 = strata_slots(k, dcode, 16), strata_slots(k, dcode, 8)
    eng = SimpleNamespace(n=1000, k=k, dcode=dcode, strata_deep_pipe=None)
    plan = lambda ns, npos, narrow=False: SimpleNamespace(NS=ns, n_positions=npos,  # noqa: E731
                                                           narrow=narrow)
    deep = lambda pl: SGDEngine._deep_pipe(eng, pl)  # noqa: E731
    assert deep(plan(ns16, 1100)) is False          # 91 % filled
    assert deep(plan(ns16, 1500)) is True           # 67 % filled
    assert deep(plan(ns8, 1050)) is True            # 8 waves
    assert deep(plan(ns8, 1050, narrow=True)) is False
    eng.strata_deep_pipe = False
    assert deep(plan(ns8, 1050)) is False
    monkeypatch.setenv("MF_STRATA_DEEP", "1")
    assert deep(plan(ns16, 1100)) is True


def test_stream_form_gated_on_block_steps(monkeypatch):
    """MF_FLAG_STREAM only for plans whose every block fits the stream
    kernel's 16-bit step field: one oversized block of one item
    phase sends the whole plan to the per-block form."""
    from types import SimpleNamespace

    from matrix_factorization import _lib
    from matrix_factorization.engine import STREAM_MAX_STEPS, SGDEngine, max_block_steps

    for v in ("MF_STRATA_STREAM", "MF_STRATA_DEEP", "MF_STRATA_COOP", "MF_STRATA_L2",
              "MF_STRATA_EARLY", "MF_PROFILER_PLAIN"):
        monkeypatch.delenv(v, raising=False)
    monkeypatch.setenv("LD_PRELOAD", "")
    eng = SimpleNamespace(strata_persistent=True, strata_deep_pipe=True, strata_stream=None,
                          STREAM_DEFAULT=True)
    eng._deep_pipe = lambda pl: SGDEngine._deep_pipe(eng, pl)
    eng._stream = lambda: SGDEngine._stream(eng)

    def plan(steps_per_block, phases=1):
        subs = [SimpleNamespace(bstep=np.concatenate([[0], np.cumsum(s)]).astype(np.int64))
                for s in steps_per_block]
        pl = SimpleNamespace(classes=4, narrow=False, l2_handoff=False)
        if phases > 1:
            pl.phases = subs
        else:
            pl.bstep = subs[0].bstep
        return pl

    ok = plan([[3, 9, STREAM_MAX_STEPS]])
    big = plan([[3, 9, 12], [4, STREAM_MAX_STEPS + 1]], phases=2)
    assert max_block_steps(ok) == STREAM_MAX_STEPS
    assert max_block_steps(big) == STREAM_MAX_STEPS + 1
    flags = lambda pl: SGDEngine._strata_flags(eng, pl, True)  # noqa: E731
    assert flags(ok) & _lib.MF_FLAG_STREAM
    assert not flags(big) & _lib.MF_FLAG_STREAM
    assert flags(big) & _lib.MF_FLAG_DEEP_PIPE             # the per-block form, still deep


def test_profiler_detection_is_the_preload_only(monkeypatch):
    """Persistent sweeps launch plainly only under rocprofv3's preloaded tool
    library, not because some ROCPROF* variable is set."""
    from matrix_factorization.engine import _under_rocprofiler, launch_form_label

    monkeypatch.delenv("MF_PROFILER_PLAIN", raising=False)
    monkeypatch.delenv("MF_STRATA_COOP", raising=False)
    monkeypatch.setenv("LD_PRELOAD", "")
    monkeypatch.setenv("ROCPROFILER_SOMETHING", "1")
    assert not _under_rocprofiler() and launch_form_label() == "cooperative"
    monkeypatch.setenv("LD_PRELOAD", "/opt/rocm/lib/rocprofiler-sdk/librocprofiler-sdk-tool.so")
    assert _under_rocprofiler() and launch_form_label() == "plain (profiler)"
    monkeypatch.setenv("MF_PROFILER_PLAIN", "0")
    assert not _under_rocprofiler()


def test_strata_planner_refuses_int32_grid_overflow():
    """A block whose D x NS grid reaches 2^31 positions is refused with an
    error instead of wrapping the int32 grid index: one item
    rated by 600K users is a block of D = 600K steps; at 4096 slots that is
    2.46e9 positions."""
    from matrix_factorization import _lib
    from matrix_factorization.engine import sched_strata

    m = 600_000
    u = np.arange(m, dtype=np.int32)
    i = np.zeros(m, dtype=np.int32)
    ub = np.array([0, m], np.int32)
    ib = np.array([0, 1], np.int32)
    with pytest.raises(_lib.MFLibraryError, match="2\\^31"):
        sched_strata(u, i, m, 1, 1, ub, ib, 4096)
    sched, bstep = sched_strata(u[:1000], i[:1000], 1000, 1, 1, np.array([0, 1000], np.int32),
                                ib, 4096)                 # 1000 x 4096: fine
    assert int(bstep[-1]) == 1000


def test_bench_traffic_lookup_is_keyed_on_world_and_emulation():
    """bench.py's roofline.traffic comes from PMC counters of exactly the
    configuration measured: an --emulate-rank N line must not borrow the
    N = 1 run's counters."""
    import sys

    sys.path.insert(0, ROOT)
    import bench

    kern = "k_sgd_strata_stream"                              # the default C3 kernel
    got = bench.traffic_from_profiles("c3", 1, "strata_persistent", "float32", kern)
    assert got is not None and got > 1e9                      # the committed N = 1 counters
    assert bench.traffic_from_profiles("c3", 1, "strata_persistent", "float32", kern,
                                       emulate=8) is None
    assert bench.traffic_from_profiles("c3", 8, "strata_persistent", "float32", kern) is None
    assert bench.traffic_from_profiles("c3", 1, "strata_persistent", "float32",
                                       "k_sgd_strata_epoch") is None     # another kernel


@pytest.mark.parametrize("chunks", [1, 2, 5, 16])
def test_chunked_levels_are_an_exact_schedule(chunks):
    """mf_sched_levels_chunked: a permutation of the ratings whose levels are
    conflict-free and respect every user's and item's visit order (so the
    level-by-level sweep is the sequential sweep, bit for bit); one chunk is
    exactly mf_sched_levels' greedy schedule."""
    from matrix_factorization.engine import sched_levels, sched_levels_chunked

    rs = np.random.RandomState(chunks)
    nu, ni, n = 300, 120, 9000
    keys = rs.choice(nu * ni, n, replace=False)
    u, i = (keys // ni).astype(np.int32), (keys % ni).astype(np.int32)
    u[:200] = 7                                   # a heavy user and item
    i[200:400] = 3
    keep = np.unique(u.astype(np.int64) * ni + i, return_index=True)[1]
    u, i = u[np.sort(keep)], i[np.sort(keep)]
    n = len(u)
    order = rs.permutation(n).astype(np.int32)
    for uu, ui in ((True, True), (True, False)):
        s, o = sched_levels_chunked(u, i, order, nu, ni, uu, ui, n_chunks=chunks)
        assert np.array_equal(np.sort(s), np.arange(n))
        assert o[0] == 0 and o[-1] == n and np.all(np.diff(o) > 0)
        if chunks == 1:
            g, go = sched_levels(u, i, order.astype(np.int64), nu, ni, uu, ui)
            assert np.array_equal(s, g) and np.array_equal(o, go)
        pos = np.empty(n, np.int64)
        pos[order] = np.arange(n)
        lev = np.empty(n, np.int64)
        for L in range(len(o) - 1):
            lev[s[o[L]:o[L + 1]]] = L
            assert np.all(np.diff(pos[s[o[L]:o[L + 1]]]) > 0)   # visit order inside a level
        for ids in ((u, i) if ui else (u,)):
            srt = np.lexsort((pos, ids))
            same = ids[srt][1:] == ids[srt][:-1]
            assert np.all(lev[srt][1:][same] > lev[srt][:-1][same])
    with pytest.raises(Exception, match="out of range"):
        bad = order.copy()
        bad[5] = n + 3
        sched_levels_chunked(u, i, bad, nu, ni, n_chunks=chunks)


def test_exact_pipeline_draws_the_reference_shuffles(cpu_engine, monkeypatch):
    """fit_epochs' exact schedule draws epoch e+1's np.random.shuffle on a
    worker thread during epoch e: same model, same train_rmse and the same
    global RandomState afterwards as the unpipelined loop."""
    import matrix_factorization.engine as E
    from matrix_factorization import KernelMF

    d = load_golden("tiny_linear")
    hp = golden_hp(d)
    hp["verbose"] = 0
    X = pd.DataFrame({"user_id": d["user_id"], "item_id": d["item_id"]})
    out = []
    for pipe_min in (1 << 40, 0):
        monkeypatch.setattr(E, "EXACT_PIPELINE_MIN", pipe_min)
        np.random.seed(int(d["seed"]))
        m = KernelMF(**hp).fit(X, pd.Series(d["rating"]))
        out.append((m.user_features.copy(), list(m.train_rmse), np.random.randint(0, 2**31 - 1)))
    assert np.array_equal(out[0][0], out[1][0])
    assert out[0][1] == out[1][1]
    assert out[0][2] == out[1][2]                  # the RNG stream afterwards
    assert np.max(np.abs(out[1][0] - d["user_features"])) < 1e-12

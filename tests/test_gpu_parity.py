"""GPU parity: libmf_hip.so vs the reference's golden vectors and the oracle.

Tolerances (FP64, schedule='exact'): the GPU reproduces the reference's visit
order and per-rating arithmetic exactly; the only difference is the summation
order of the k-long dot products (fixed butterfly vs BLAS ddot), i.e. ULP-level
perturbations that SGD carries forward.  Stated bars:
  parameters / predictions: max |diff| <= 1e-10 * max(1, |value|)
  train_rmse:               |diff| <= 1e-12
  recommend() top-10 ids:   identical
FP32 runs are compared on RMSE only (|diff| <= 1e-5, the north-star bar).
"""

import numpy as np
import pandas as pd
import pytest

from conftest import golden_hp, load_golden

pytestmark = pytest.mark.gpu

KERNEL_CASES = ["tiny_linear", "tiny_sigmoid", "tiny_rbf", "tiny_defaults",
                "mid_k100", "mid_sigmoid_k32", "c1_linear"]


def _close(a, b, tol=1e-10):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    assert a.shape == b.shape
    if a.size == 0:
        return
    scale = max(1.0, float(np.max(np.abs(b))))
    err = float(np.max(np.abs(a - b)))
    assert err <= tol * scale, f"max |diff| {err:.3e} > {tol:.0e} * {scale:.3g}"


@pytest.fixture(scope="module")
def mf():
    import matrix_factorization

    matrix_factorization._lib.load()
    return matrix_factorization


def _frame(d):
    return (pd.DataFrame({"user_id": d["user_id"], "item_id": d["item_id"]}),
            pd.Series(d["rating"]))


@pytest.mark.parametrize("name", KERNEL_CASES)
def test_kernelmf_matches_reference(mf, name, capsys):
    d = load_golden(name)
    hp = golden_hp(d)
    X, y = _frame(d)
    np.random.seed(int(d["seed"]))
    m = mf.KernelMF(**hp).fit(X, y)
    out = capsys.readouterr().out
    if hp.get("verbose", 1) == 1 and name == "tiny_linear":
        # same print format as the reference (kernel_matrix_factorization.py:443)
        ref_lines = str(d["stdout"]).strip().splitlines()
        got_lines = out.strip().splitlines()
        assert len(ref_lines) == len(got_lines)
        for a, b in zip(got_lines, ref_lines):
            assert a.split(":")[0] == b.split(":")[0]
            assert abs(float(a.split(":")[1]) - float(b.split(":")[1])) < 1e-12
    assert list(m.user_id_map.keys()) == list(d["user_ids"])
    assert list(m.item_id_map.keys()) == list(d["item_ids"])
    assert m.global_mean == d["global_mean"]
    _close(m.user_features, d["user_features"])
    _close(m.item_features, d["item_features"])
    _close(m.user_biases, d["user_biases"])
    _close(m.item_biases, d["item_biases"])
    _close(m.train_rmse, d["train_rmse"], 1e-12)
    T = pd.DataFrame({"user_id": d["test_user"], "item_id": d["test_item"]})
    _close(m.predict(T, bound_ratings=True), d["pred_bound"])
    assert m.predictions_possible == d["pred_possible"].tolist()
    _close(m.predict(T, bound_ratings=False), d["pred_unbound"])
    df = X.assign(rating=y)
    excl = []
    for j, user in enumerate(d["rec_users"]):
        known = df.loc[df.user_id == user, "item_id"].to_numpy()
        known = known[: len(known) // 2] if j % 2 == 0 else None
        rec = m.recommend(user=user, amount=10, items_known=known)
        assert rec["item_id"].tolist() == d["rec_items"][j].tolist()
        _close(rec["rating_pred"].to_numpy(), d["rec_pred"][j])
        if known is not None:
            excl.append(pd.DataFrame({"user_id": user, "item_id": known}))
    # the batched GPU top-k (mf_topk, row f1) against the same golden lists:
    # all rec_users in one call, items_known passed as the exclusion CSR
    users = list(d["rec_users"])
    got = m.recommend_batch(users, amount=10, exclude_known=pd.concat(excl))
    for j, user in enumerate(users):
        g = got[got.user_id == user]
        assert g["item_id"].tolist() == d["rec_items"][j].tolist()
        _close(g["rating_pred"].to_numpy(), d["rec_pred"][j])


def test_update_users_matches_reference(mf):
    d = load_golden("update_users")
    hp = golden_hp(d)
    df = pd.DataFrame({"user_id": d["user_id"], "item_id": d["item_id"],
                       "rating": d["rating"]})
    np.random.seed(int(d["seed"]))
    Xi, yi, Xu, yu, Xt, yt = mf.train_update_test_split(df, frac_new_users=0.25)
    assert Xi.index.tolist() == d["split_train_index"].tolist()
    assert Xu.index.tolist() == d["split_update_index"].tolist()
    assert Xt.index.tolist() == d["split_test_index"].tolist()
    m = mf.KernelMF(**hp).fit(Xi, yi)
    _close(m.user_features, d["fit_user_features"])
    _close(m.item_features, d["fit_item_features"])
    extra = Xi.loc[d["extra_index"]]
    Q_before = m.item_features.copy()
    m.update_users(pd.concat([Xu, extra]), pd.concat([yu, yi.loc[extra.index]]),
                   lr=0.03, n_epochs=5, verbose=0)
    assert list(m.user_id_map.keys()) == d["user_ids"].tolist()
    assert list(m.user_id_map.values()) == d["user_id_vals"].tolist()
    assert m.n_users == d["n_users"]          # reference quirk: not updated
    _close(m.user_features, d["user_features"])
    assert np.array_equal(m.item_features, Q_before)          # frozen bit for bit
    assert np.max(np.abs(m.item_features - d["fit_item_features"])) < 1e-12
    _close(m.user_biases, d["user_biases"])
    _close(m.train_rmse, d["train_rmse"], 1e-12)
    _close(m.predict(Xt), d["pred_test"])


@pytest.mark.parametrize("method", ["sgd", "als"])
def test_baseline_matches_reference(mf, method):
    d = load_golden(f"baseline_{method}")
    hp = golden_hp(d)
    X = pd.DataFrame({"user_id": d["user_id"], "item_id": d["item_id"]})
    np.random.seed(int(d["seed"]))
    m = mf.BaselineModel(**hp).fit(X, pd.Series(d["rating"]))
    # no dot product in the bias model: bit-identical to the reference loop
    assert np.array_equal(m.user_biases, d["user_biases"])
    assert np.array_equal(m.item_biases, d["item_biases"])
    _close(m.train_rmse, d["train_rmse"], 1e-13)
    T = pd.DataFrame({"user_id": d["test_user"], "item_id": d["test_item"]})
    assert np.array_equal(np.asarray(m.predict(T)), d["pred"])
    assert m.predictions_possible == d["pred_possible"].tolist()
    if method == "sgd":
        np.random.seed(int(d["seed"]) + 1)
        m.update_users(pd.DataFrame({"user_id": d["upd_user"], "item_id": d["upd_item"]}),
                       pd.Series(d["upd_rating"]), lr=0.05, n_epochs=3)
        assert np.array_equal(m.user_biases, d["upd_user_biases"])
        _close(m.train_rmse, d["upd_train_rmse"], 1e-13)


# ------------------------------------------------------------ oracle checks
def _synthetic(seed, n_users, n_items, nnz):
    rs = np.random.RandomState(seed)
    keys = np.unique(rs.randint(0, n_users * n_items, int(nnz * 1.2)).astype(np.int64))
    keys = rs.permutation(keys)[:nnz]
    u = (keys // n_items).astype(np.int32)
    i = (keys % n_items).astype(np.int32)
    r = rs.randint(1, 6, len(keys)).astype(np.float64)
    return u, i, r


@pytest.mark.parametrize("kernel,k", [("linear", 64), ("sigmoid", 32), ("rbf", 16),
                                      ("linear", 100), ("sigmoid", 7)])
def test_colored_epoch_equals_serialized_oracle(mf, kernel, k):
    """The colour schedule is a valid sequential order: the GPU epoch equals
    the oracle's sequential sweep over (colours in launch order)."""
    import oracle
    from matrix_factorization.engine import SGDEngine

    nu, ni, nnz = 3000, 800, 120000
    u, i, r = _synthetic(3, nu, ni, nnz)
    rs = np.random.RandomState(4)
    P = rs.normal(0, 0.1, (nu, k)); Q = rs.normal(0, 0.1, (ni, k))
    bu = np.zeros(nu); bi = np.zeros(ni)
    mu = float(r.mean())
    hyp = dict(gamma=1.0 / k, min_rating=1.0, max_rating=5.0)
    eng = SGDEngine(u, i, r, nu, ni, k, kernel, "float64", "cuda:0",
                    global_mean=mu, **hyp)
    eng.load_params(P, Q, bu, bi)
    nb = eng.prepare_colored()
    seq = rs.permutation(nb).astype(np.int32)
    eng.epoch_colored(seq, lr=0.01, reg=0.02)
    eng.sse_async(0)
    Pg, Qg, bug, big = eng.params_numpy()
    # serialised order on the host
    order = np.concatenate([np.arange(eng.colored[b], eng.colored[b + 1]) for b in seq])
    P2, Q2, bu2, bi2 = P.copy(), Q.copy(), bu.copy(), bi.copy()
    oracle.sgd_pass(eng.u_host, eng.i_host, eng.r_host, mu, bu2, bi2, P2, Q2,
                    kernel=kernel, lr=0.01, reg=0.02, order=order, **hyp)
    _close(Pg, P2, 1e-11)
    _close(Qg, Q2, 1e-11)
    _close(bug, bu2, 1e-11)
    _close(big, bi2, 1e-11)
    rm = eng.rmse_values(1)[0]
    ro = oracle.rmse(eng.u_host, eng.i_host, eng.r_host, mu, bu2, bi2, P2, Q2,
                     kernel=kernel, **hyp)
    assert abs(rm - ro) < 1e-12


def test_float32_rmse_within_1e5_of_oracle(mf):
    """FP32 state, exact order, 3 epochs: RMSE within the north-star 1e-5."""
    import oracle

    u, i, r = _synthetic(5, 2000, 500, 60000)
    df = pd.DataFrame({"user_id": u, "item_id": i})
    hp = dict(n_factors=64, n_epochs=3, lr=0.01, reg=0.02, min_rating=1, max_rating=5)
    np.random.seed(3)
    m = mf.KernelMF(verbose=0, dtype="float32", **hp).fit(df, pd.Series(r))
    np.random.seed(3)
    o = oracle.oracle_kernel_fit(df, pd.Series(r), **hp)
    assert np.max(np.abs(np.asarray(m.train_rmse) - o["train_rmse"])) < 1e-5


def test_predict_edge_cases(mf):
    d = load_golden("tiny_linear")
    hp = golden_hp(d)
    hp["verbose"] = 0
    X, y = _frame(d)
    np.random.seed(int(d["seed"]))
    m = mf.KernelMF(**hp).fit(X, y)
    assert m.predict(X.iloc[:0]) == []
    # unknown user and item: global mean + zero vectors (clipped)
    T = pd.DataFrame({"user_id": [-5, d["user_id"][0]], "item_id": [d["item_id"][0], -7]})
    p = m.predict(T, bound_ratings=False)
    u0 = m.user_id_map[d["user_id"][0]]
    i0 = m.item_id_map[d["item_id"][0]]
    assert p[0] == (m.global_mean + m.item_biases[i0]) + 0.0
    assert p[1] == (m.global_mean + 0.0) + m.user_biases[u0]
    assert m.predictions_possible == [False, False]


def test_topk_ties_and_chunking(mf):
    """Equal scores: recommend_batch ranks the lower internal item id first,
    the order a stable descending sort of recommend()'s candidate list gives
    (the reference's quicksort leaves tie order unspecified,
    recommender_base.py:259).  Several chunks of users give the same result
    as one launch; duplicate query users are answered twice."""
    d = load_golden("c1_linear")
    hp = golden_hp(d)
    hp.update(n_epochs=2, verbose=0)
    X, y = _frame(d)
    np.random.seed(int(d["seed"]))
    m = mf.KernelMF(**hp).fit(X, y)
    Q, bi = m.item_features.copy(), m.item_biases.copy()
    # five items share the parameters of item 0: exact ties
    for t in (7, 3, 900, 1500, 42):
        Q[t] = Q[0]
        bi[t] = bi[0]
    m.item_features, m.item_biases = Q, bi
    inv = list(m.item_id_map.keys())
    users = list(d["rec_users"]) + [d["rec_users"][0]]
    one = m.recommend_batch(users, amount=40, bound_ratings=False)
    eng = m._predictor()
    lib = mf._lib.load()
    eng.topk_ws_budget = lib.mf_topk_workspace_bytes(2, m.n_items, 40)   # two users per launch
    try:
        many = m.recommend_batch(users, amount=40, bound_ratings=False)
    finally:
        eng.topk_ws_budget = type(eng).topk_ws_budget
    pd.testing.assert_frame_equal(one, many)
    for user in users:
        cand = pd.DataFrame({"user_id": user, "item_id": inv})
        cand["rating_pred"] = m.predict(cand, bound_ratings=False)
        ref = cand.sort_values("rating_pred", ascending=False, kind="stable").head(40)
        g = one[one.user_id == user]
        assert len(g) == 40 * users.count(user)
        assert g["item_id"].tolist()[:40] == ref["item_id"].tolist()
        assert np.array_equal(g["rating_pred"].to_numpy()[:40], ref["rating_pred"].to_numpy())


@pytest.mark.parametrize("amount", [1, 10, 64])
def test_topk_fused_equals_two_stage(mf, amount, monkeypatch):
    """k_topk_fused + k_topk_merge (scores never materialised) return exactly
    what the two-stage path (all keys in HBM, radix select) returns: same
    ids, same scores, exclusions applied, for a batch large enough to split
    the item range across workgroups."""
    d = load_golden("c1_linear")
    hp = golden_hp(d)
    hp.update(n_epochs=2, verbose=0)
    X, y = _frame(d)
    np.random.seed(int(d["seed"]))
    m = mf.KernelMF(**hp).fit(X, y)
    users = list(m.user_id_map)[:300]
    known = X.assign(r=y)
    known = known[known.user_id.isin(users[::3])]
    fused = m.recommend_batch(users, amount=amount, exclude_known=known, bound_ratings=False)
    monkeypatch.setenv("MF_TOPK_TWO_STAGE", "1")
    two = m.recommend_batch(users, amount=amount, exclude_known=known, bound_ratings=False)
    pd.testing.assert_frame_equal(fused, two)
    assert len(fused) == amount * len(users)
    pairs = set(zip(known.user_id, known.item_id))
    assert not any((u, i) in pairs for u, i in zip(fused.user_id, fused.item_id))


def test_predict_sees_in_place_edits(mf):
    """The device copy follows the NumPy attributes, in-place edits included
    (the reference predicts from the live arrays, :148-160)."""
    d = load_golden("tiny_linear")
    hp = golden_hp(d)
    hp["verbose"] = 0
    X, y = _frame(d)
    np.random.seed(int(d["seed"]))
    m = mf.KernelMF(**hp).fit(X, y)
    T = X.iloc[:30]
    before = m.predict(T, bound_ratings=False)
    m.item_features[:] *= 2.0                       # same array object, new content
    m.user_biases[0] += 0.5
    after = m.predict(T, bound_ratings=False)
    assert before != after
    u = T["user_id"].map(m.user_id_map).to_numpy()
    i = T["item_id"].map(m.item_id_map).to_numpy()
    expect = ((m.global_mean + m.item_biases[i]) + m.user_biases[u]) + np.einsum(
        "nk,nk->n", m.user_features[u], m.item_features[i])
    _close(after, expect, 1e-12)


def test_fit_empty_and_pickle(mf):
    import pickle

    d = load_golden("tiny_linear")
    X, y = _frame(d)
    np.random.seed(0)
    m = mf.KernelMF(n_factors=4, n_epochs=2, verbose=0).fit(X, y)
    m2 = pickle.loads(pickle.dumps(m))
    assert isinstance(m2.user_features, np.ndarray)
    T = X.iloc[:20]
    assert m2.predict(T) == m.predict(T)


def _topk_engine(k, nu, ni, seed, dup_items=0, zero_users=0):
    from matrix_factorization.engine import SGDEngine

    rs = np.random.RandomState(seed)
    P = rs.normal(0, 0.3, (nu, k)).astype(np.float32)
    Q = rs.normal(0, 0.3, (ni, k)).astype(np.float32)
    bu = rs.normal(0, 0.1, nu).astype(np.float32)
    bi = rs.normal(0, 0.1, ni).astype(np.float32)
    if dup_items:                     # blocks of identical items: exact score ties
        Q[:dup_items] = Q[0]
        bi[:dup_items] = bi[0]
    if zero_users:                    # all-zero rows: every score is mu + b_i + b_u
        P[:zero_users] = 0.0
    eng = SGDEngine(np.zeros(0, np.int32), np.zeros(0, np.int32), np.zeros(0), nu, ni, k,
                    "linear", "float32", "cuda:0", min_rating=1.0, max_rating=5.0,
                    global_mean=3.5)
    eng.load_params(P, Q, bu, bi)
    return eng


def _topk_both(eng, users, amount, ex_ptr=None, ex_items=None):
    q = eng.topk_prepare(users, amount, ex_ptr, ex_items)
    assert q["mm"], "the MFMA filter should take this case"
    eng.topk_launch(q)
    fell_back = eng.topk_finish(q)
    mi, ms = q["items"].cpu().numpy(), q["scores"].cpu().numpy()
    eng.topk_launch(q, exact=True)
    return mi, ms, q["items"].cpu().numpy(), q["scores"].cpu().numpy(), fell_back


@pytest.mark.parametrize("bf16", ["1", "0"])
@pytest.mark.parametrize("k,amount", [(8, 10), (20, 1), (32, 64), (64, 10), (64, 64)])
def test_topk_mfma_filter_equals_exact(k, amount, bf16, monkeypatch):
    """mf_topk_mm (MFMA scores only select candidates; survivors rescored
    with predict's arithmetic) returns exactly mf_topk's ids and scores:
    ragged item / user counts, unknown users (-1), CSR exclusions -- with
    k_topk_mw's operands as bf16 hi + lo parts (the default) and as f32."""
    monkeypatch.setenv("MF_TOPK_BF16", bf16)
    nu, ni = 900, 5003
    eng = _topk_engine(k, nu, ni, 40 + k)
    rs = np.random.RandomState(k)
    users = rs.choice(nu, 333, replace=False).astype(np.int32)
    users[::50] = -1
    cnt = rs.randint(0, 40, len(users))
    ex_ptr = np.concatenate([[0], np.cumsum(cnt)]).astype(np.int64)
    ex_items = rs.randint(0, ni, ex_ptr[-1]).astype(np.int32)
    mi, ms, ei, es, _ = _topk_both(eng, users, amount, ex_ptr, ex_items)
    assert np.array_equal(mi, ei)
    assert np.array_equal(ms, es)
    for q in range(len(users)):
        assert not set(mi[q]) & set(ex_items[ex_ptr[q]:ex_ptr[q + 1]])


def test_topk_mfma_filter_ties_and_overflow():
    """Masses of exactly equal scores (duplicated items, all-zero users):
    ties keep the lower item id as in mf_topk; where a band outgrows its
    list the overflow word sends topk() to the exact path, same result."""
    k, nu, ni = 32, 200, 3000
    eng = _topk_engine(k, nu, ni, 7, dup_items=700, zero_users=40)
    users = np.arange(nu, dtype=np.int32)
    mi, ms, ei, es, _ = _topk_both(eng, users, 64)
    assert np.array_equal(mi, ei)
    assert np.array_equal(ms, es)
    ids, sc = eng.topk(users, 64)
    assert np.array_equal(ids, ei)


@pytest.mark.parametrize("merge_wave", ["1", "0"])
@pytest.mark.parametrize("ties", [False, True])
def test_topk_merge_forms_agree(ties, merge_wave, monkeypatch):
    """The merge of the splits' bands -- one wave per user for users whose
    bands hold <= 64 entries (round 6), one workgroup per user for the rest,
    or for every user with MF_TOPK_MERGE_WAVE=0 -- gives exactly mf_topk's
    ids and scores: random scores (small bands, the wave form) and 160
    exactly tied top items spread over all 8 splits (bands of 160 entries,
    the workgroup form)."""
    monkeypatch.setenv("MF_TOPK_MERGE_WAVE", merge_wave)
    k, nu, ni = 64, 2000, 20000
    eng = _topk_engine(k, nu, ni, 91)
    if ties:
        P, Q, bu, bi = (np.array(x, np.float32) for x in eng.params_numpy())
        # 20 in each of the 8 item splits (2528 ids each: the split length
        # rounded up to whole 32-item tiles), within the 32 a list keeps
        tied = np.array([t * 2528 + 100 + j for t in range(8) for j in range(20)])
        Q[tied] = Q[tied[0]]
        bi[tied] = 10.0                   # above every other score of every user
        eng.load_params(P, Q, bu, bi)
    users = np.arange(nu, dtype=np.int32)
    mi, ms, ei, es, fell_back = _topk_both(eng, users, 10)
    assert not fell_back
    assert np.array_equal(mi, ei)
    assert np.array_equal(ms, es)
    if ties:
        assert np.array_equal(np.sort(mi, axis=1), np.tile(np.sort(tied)[:10], (nu, 1)))


@pytest.mark.parametrize("bf16", ["1", "0"])
@pytest.mark.parametrize("ni", [20000, 65600])
def test_topk_probe_floor_with_excluded_top_items(ni, bf16, monkeypatch):
    """k_topk_mw's probe walk (the best item of each group of ids scored
    first; the amount-th best s' of a user's non-excluded probe items, less
    2M, floors every admission bound) under exclusions aimed at it: users
    whose exact top-40 items are all excluded (so are most probe items that
    rank high for them), a user left with 5 candidates (fewer than amount:
    no floor, -1 padding) and one with every item excluded.  Same ids and
    scores as mf_topk, no excluded item returned.  65600 items: 512 groups of
    129 ids would leave the last group empty (the probe count is trimmed to
    509; an empty group once read a row past the end of Q)."""
    monkeypatch.setenv("MF_TOPK_BF16", bf16)
    k, nu, amount = 64, 400, 10
    eng = _topk_engine(k, nu, ni, 23)
    rs = np.random.RandomState(5)
    users = rs.choice(nu, 260, replace=False).astype(np.int32)
    top, _ = eng.topk(users, 40)
    lists = []
    for q in range(len(users)):
        if q == 7:
            ex = np.setdiff1d(np.arange(ni), rs.choice(ni, 5, replace=False))
        elif q == 8:
            ex = np.arange(ni)
        elif q % 2:
            ex = np.union1d(top[q], rs.choice(ni, 30, replace=False))
        else:
            ex = rs.choice(ni, rs.randint(0, 50), replace=False)
        lists.append(np.sort(ex).astype(np.int32))
    ex_ptr = np.concatenate([[0], np.cumsum([len(x) for x in lists])]).astype(np.int64)
    ex_items = np.concatenate(lists).astype(np.int32)
    mi, ms, ei, es, _ = _topk_both(eng, users, amount, ex_ptr, ex_items)
    assert np.array_equal(mi, ei)
    assert np.array_equal(np.nan_to_num(ms, nan=-7.0), np.nan_to_num(es, nan=-7.0))
    assert (mi[7] >= 0).sum() == 5 and (mi[8] < 0).all()
    for q in range(len(users)):
        assert not set(mi[q][mi[q] >= 0]) & set(lists[q])


@pytest.mark.parametrize("mfma", [True, False])
def test_topk_unsorted_exclusions(mfma):
    """The ABI wants each user's exclusion list sorted ascending (the kernels
    binary-search it, include/mf_hip.h); engine.topk_prepare sorts whatever
    the caller passes, so shuffled lists give the sorted lists' result on the
    MFMA filter and the exact fused path alike, and no excluded item comes
    back."""
    k, nu, ni, amount = 32, 300, 4000, 10
    eng = _topk_engine(k, nu, ni, 11)
    eng.topk_mfma = mfma
    rs = np.random.RandomState(2)
    users = rs.choice(nu, 120, replace=False).astype(np.int32)
    cnt = rs.randint(0, 300, len(users))
    ex_ptr = np.concatenate([[0], np.cumsum(cnt)]).astype(np.int64)
    srt = np.concatenate([np.sort(rs.choice(ni, c, replace=False)) for c in cnt]).astype(np.int32)
    shuf = srt.copy()
    for q in range(len(users)):
        rs.shuffle(shuf[ex_ptr[q]:ex_ptr[q + 1]])
    a_i, a_s = eng.topk(users, amount, ex_ptr, srt)
    b_i, b_s = eng.topk(users, amount, ex_ptr, shuf)
    assert np.array_equal(a_i, b_i) and np.array_equal(a_s, b_s)
    for q in range(len(users)):
        assert not set(b_i[q]) & set(srt[ex_ptr[q]:ex_ptr[q + 1]])


def test_exact_chunked_levels_equal_greedy_levels_10m(mf):
    """The exact schedule at scale (fit_epochs' 32-bit visit order ->
    mf_sched_levels_chunked on host threads, pinned asynchronous upload)
    against the greedy single-thread levels (int64 order -> mf_sched_levels):
    same visit orders, so the same sequential sweep -- parameters and SSE
    bit for bit equal after every epoch (10M ratings, 16 chunks)."""
    import torch

    from matrix_factorization.engine import SGDEngine

    rs = np.random.RandomState(11)
    nu, ni, n, k = 200_000, 20_000, 10_000_000, 32
    keys = np.unique(rs.randint(0, nu * ni, size=n + n // 50, dtype=np.int64))[:n]
    keys = keys[rs.permutation(len(keys))]
    u, i = (keys // ni).astype(np.int32), (keys % ni).astype(np.int32)
    r = rs.randint(1, 6, len(keys)).astype(np.float64)
    n = len(u)
    P0 = rs.normal(0, 0.1, (nu, k))
    Q0 = rs.normal(0, 0.1, (ni, k))
    engs = []
    for _ in range(2):
        e = SGDEngine(u, i, r, nu, ni, k, "linear", "float32", "cuda:0",
                      global_mean=float(r.mean()), min_rating=1, max_rating=5)
        e.load_params(P0, Q0, np.zeros(nu), np.zeros(ni))
        engs.append(e)
    for ep in range(2):
        order = rs.permutation(n)
        engs[0].epoch_exact(order.astype(np.int64), 0.01, 0.02)
        engs[1].epoch_exact(order.astype(np.int32), 0.01, 0.02)
        for e in engs:
            e.sse_async(ep)
        torch.cuda.synchronize()
        a, b = engs[0].params_numpy(), engs[1].params_numpy()
        for x, y in zip(a, b):
            assert np.array_equal(x, y)
    assert engs[0].rmse_values(2) == engs[1].rmse_values(2)

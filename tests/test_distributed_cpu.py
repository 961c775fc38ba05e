"""User-sharded data parallelism, rehearsed on CPU with gloo (world_size 2).

The per-epoch exchange of matrix_factorization.distributed (colored:
snapshot -> local epoch -> delta; strata: delta-out epoch; then
all_reduce(SUM) -> replica += sum / world) runs in two real processes over
gloo.  The device sweeps are replaced by the CPU oracle and the
replica arithmetic by torch on CPU tensors (test doubles, this file only); the
sharding, schedules, collective and bookkeeping are the product code.  The
result must equal a single-process simulation of the same algorithm.
"""

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle

NU, NI, NNZ, K = 300, 80, 6000, 8
LR, REG, EPOCHS, SEED = 0.02, 0.05, 3, 99
STRATA_B = 3                                     # strata per epoch on each rank


def _scale(world):
    from matrix_factorization.distributed import default_delta_scale

    return default_delta_scale(world)


def _data():
    rs = np.random.RandomState(0)
    keys = rs.choice(NU * NI, NNZ, replace=False)
    u = (keys // NI).astype(np.int32)
    i = (keys % NI).astype(np.int32)
    r = rs.randint(1, 6, NNZ).astype(np.float64)
    P0 = rs.normal(0, 0.1, (NU, K))
    Q0 = rs.normal(0, 0.1, (NI, K))
    return u, i, r, P0, Q0


class CpuEngine:
    """Test double of SGDEngine for the colored and strata schedules (oracle
    sweeps in the schedule's serial order; the plans are the product's)."""

    strata_persistent = False      # no persistent sweep: nothing can give up waiting

    def __init__(self, u, i, r, n_users, n_items, k, mu):
        self.u_host, self.i_host, self.r_host = u, i, r
        self.n, self.n_users, self.n_items, self.k = len(u), n_users, n_items, k
        self.global_mean = mu
        self.colored = None
        self.strata = None
        self.dcode = 1                           # MF_F64
        self.sse_buf = torch.zeros(16, dtype=torch.float64)
        self.tdt, self.dev = torch.float64, torch.device("cpu")
        self.P = self.Q = self.bu = self.bi = None

    def load_params(self, P=None, Q=None, bu=None, bi=None):
        t = lambda a: torch.as_tensor(np.array(a, np.float64))  # noqa: E731
        if P is not None:
            self.P = t(P).reshape(self.n_users, self.k)
        if Q is not None:
            self.Q = t(Q).reshape(self.n_items, self.k)
        if bu is not None:
            self.bu = t(bu)
        if bi is not None:
            self.bi = t(bi)

    def prepare_colored(self):
        from matrix_factorization.engine import sched_color

        sched, offs = sched_color(self.u_host, self.i_host, self.n_users, self.n_items)
        self.u_host, self.i_host, self.r_host = (self.u_host[sched], self.i_host[sched],
                                                 self.r_host[sched])
        self.colored = offs
        return len(offs) - 1

    def prepare_strata(self, n_blocks=None, item_bounds=None, classes=None, regroup=None):
        from matrix_factorization.engine import (PhasedStrata, StrataPlan, balanced_bounds,
                                                 sched_strata, strata_slots)

        B = STRATA_B if n_blocks is None else n_blocks
        C = classes or 1
        if item_bounds is not None:          # the product's PhasedStrata over given ranges
            ilo = np.asarray(item_bounds, np.int64)
            ns = strata_slots(self.k, self.dcode)
            plans, idx = [], []
            for p in range(len(ilo) - 1):
                ix = np.flatnonzero((self.i_host >= ilo[p]) & (self.i_host < ilo[p + 1]))
                uu, ii = self.u_host[ix], self.i_host[ix] - int(ilo[p])
                m = int(ilo[p + 1] - ilo[p])
                ub = balanced_bounds(uu, self.n_users, C * B)
                ib = balanced_bounds(ii, m, B)
                sched, bstep = sched_strata(uu, ii, self.n_users, m, B, ub, ib, ns, C)
                plans.append(StrataPlan(B, ns, ub, ib, bstep, sched, C))
                idx.append(ix)
            self.strata = PhasedStrata(plans, idx, ilo)
            return self.strata
        ub = balanced_bounds(self.u_host, self.n_users, C * B)
        ib = balanced_bounds(self.i_host, self.n_items, B)
        ns = strata_slots(self.k, self.dcode)
        sched, bstep = sched_strata(self.u_host, self.i_host, self.n_users, self.n_items, B,
                                    ub, ib, ns, C)
        self.strata = StrataPlan(B, ns, ub, ib, bstep, sched, C)
        return self.strata

    def epoch_strata(self, seq, seed, lr, reg, update_user=True, update_item=True,
                     timing=False, delta=None, persistent=None):
        order = self.strata.serial_order(seq, seed)
        Q0, bi0 = self.Q.clone(), self.bi.clone()
        oracle.sgd_pass(self.u_host, self.i_host, self.r_host, self.global_mean,
                        self.bu.numpy(), self.bi.numpy(), self.P.numpy(), self.Q.numpy(),
                        lr=lr, reg=reg, order=order)
        if delta is not None:          # delta-out form: replica untouched
            delta[0].copy_(self.Q - Q0)
            delta[1].copy_(self.bi - bi0)
            self.Q.copy_(Q0)
            self.bi.copy_(bi0)

    def epoch_phase(self, c, seq, seed, lr, reg, update_user=True, update_item=True,
                    timing=False, persistent=None):
        order = self.strata.phase_order(c, seq, seed)
        oracle.sgd_pass(self.u_host, self.i_host, self.r_host, self.global_mean,
                        self.bu.numpy(), self.bi.numpy(), self.P.numpy(), self.Q.numpy(),
                        lr=lr, reg=reg, order=order)

    def check_strata(self):
        pass

    def strata_failed(self):
        return False

    def sse_values(self, n):
        return self.sse_buf[:n].numpy().copy()

    def _ensure_sse_slots(self, n):
        if self.sse_buf.numel() < n:
            self.sse_buf = torch.cat([self.sse_buf, torch.zeros(n - self.sse_buf.numel(),
                                                                dtype=torch.float64)])

    def epoch_colored(self, seq, lr, reg, update_user=True, update_item=True, timing=False):
        order = np.concatenate([np.arange(self.colored[b], self.colored[b + 1])
                                for b in seq]).astype(np.int64)
        Q = self.Q.numpy()
        bi = self.bi.numpy()
        oracle.sgd_pass(self.u_host, self.i_host, self.r_host, self.global_mean,
                        self.bu.numpy(), bi, self.P.numpy(), Q, lr=lr, reg=reg, order=order)

    def sse_join(self):
        pass

    def sse_async(self, slot):
        self.sse_buf[slot] = oracle.sse(self.u_host, self.i_host, self.r_host,
                                        self.global_mean, self.bu.numpy(), self.bi.numpy(),
                                        self.P.numpy(), self.Q.numpy())


def _exchange_cls():
    from matrix_factorization.distributed import ReplicaExchange

    class CpuExchange(ReplicaExchange):
        def _delta(self, mode):                       # mf_replica_delta on CPU
            from matrix_factorization import _lib
            if mode == _lib.MF_DELTA_TAKE:
                self.flat.sub_(self.delta)
            else:
                self.flat.add_(self.delta)

        def _apply(self):                             # mf_replica_apply on CPU
            self.flat.add_(self.scale * self.delta)

    return CpuExchange


def _run_rank(rank, world, port, out_dir, schedule="colored"):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from matrix_factorization.distributed import (global_rmse, local_shard, shard_users,
                                                  sharded_epochs)

    u, i, r, P0, Q0 = _data()
    mu = float(r.mean())
    bounds = shard_users(u, NU, world)
    lu, li, lr_ = local_shard(u, i, r, bounds, rank)
    lo, hi = int(bounds[rank]), int(bounds[rank + 1])
    eng = CpuEngine(lu, li, lr_, hi - lo, NI, K, mu)
    eng.load_params(P=P0[lo:hi], bu=np.zeros(hi - lo))
    ex = _exchange_cls()(eng)
    ex.bind(Q0, np.zeros(NI))
    sharded_epochs(eng, ex, EPOCHS, LR, REG, SEED, schedule=schedule, n_blocks=STRATA_B)
    rm = global_rmse(eng, EPOCHS, NNZ)
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), Q=eng.Q.numpy(), bi=eng.bi.numpy(),
             P=eng.P.numpy(), bu=eng.bu.numpy(), lo=lo, hi=hi, rmse=np.array(rm))
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _simulate(world, schedule="colored"):
    """Single-process restatement of the same algorithm."""
    from matrix_factorization.distributed import local_shard, shard_users

    u, i, r, P0, Q0 = _data()
    mu = float(r.mean())
    bounds = shard_users(u, NU, world)
    engs = []
    for rank in range(world):
        lu, li, lr_ = local_shard(u, i, r, bounds, rank)
        lo, hi = int(bounds[rank]), int(bounds[rank + 1])
        e = CpuEngine(lu, li, lr_, hi - lo, NI, K, mu)
        e.load_params(P=P0[lo:hi], bu=np.zeros(hi - lo), Q=Q0, bi=np.zeros(NI))
        if schedule == "strata":
            e.prepare_strata(STRATA_B)
        else:
            e.prepare_colored()
        engs.append(e)
    Q = Q0.copy()
    bi = np.zeros(NI)
    sse = np.zeros(EPOCHS)
    for ep in range(EPOCHS):
        dQ = np.zeros_like(Q)
        dbi = np.zeros_like(bi)
        for e in engs:
            e.Q = torch.as_tensor(Q.copy())
            e.bi = torch.as_tensor(bi.copy())
            rs_ep = np.random.RandomState((SEED * 1000003 + ep) & 0x7FFFFFFF)
            if schedule == "strata":
                seq = rs_ep.permutation(e.strata.B)
                e.epoch_strata(seq, int(rs_ep.randint(0, 2**31 - 1)), LR, REG)
            else:
                seq = rs_ep.permutation(len(e.colored) - 1)
                e.epoch_colored(seq, LR, REG)
            dQ += e.Q.numpy() - Q
            dbi += e.bi.numpy() - bi
        Q = Q + _scale(world) * dQ                    # damped sum (default_delta_scale)
        bi = bi + _scale(world) * dbi
        for e in engs:
            e.Q = torch.as_tensor(Q.copy())
            e.bi = torch.as_tensor(bi.copy())
            e.sse_async(ep)
            sse[ep] += float(e.sse_buf[ep])
    return Q, bi, np.sqrt(sse / NNZ), engs, bounds


def test_shard_users_balances_ratings():
    from matrix_factorization.distributed import local_shard, shard_users

    u, i, r, _, _ = _data()
    for world in (1, 2, 3, 8):
        b = shard_users(u, NU, world)
        assert b[0] == 0 and b[-1] == NU and np.all(np.diff(b) >= 0)
        sizes = [len(local_shard(u, i, r, b, k)[0]) for k in range(world)]
        assert sum(sizes) == NNZ
        assert max(sizes) - min(sizes) <= np.bincount(u).max() + NNZ // (world * 10) + 1


@pytest.mark.timeout(300)
@pytest.mark.parametrize("schedule", ["colored", "strata"])
def test_two_rank_gloo_exchange_matches_simulation(tmp_path, schedule):
    world = 2
    mp.start_processes(_run_rank, args=(world, _free_port(), str(tmp_path), schedule),
                       nprocs=world, join=True, start_method="spawn")
    res = [dict(np.load(tmp_path / f"rank{k}.npz")) for k in range(world)]
    # every rank ends with the same item replica
    assert np.array_equal(res[0]["Q"], res[1]["Q"])
    assert np.array_equal(res[0]["bi"], res[1]["bi"])
    Q, bi, rmse, engs, bounds = _simulate(world, schedule)
    assert np.max(np.abs(res[0]["Q"] - Q)) < 1e-12
    assert np.max(np.abs(res[0]["bi"] - bi)) < 1e-12
    for k in range(world):
        assert np.max(np.abs(res[k]["P"] - engs[k].P.numpy())) < 1e-12
    assert np.max(np.abs(res[0]["rmse"] - rmse)) < 1e-12
    assert rmse[-1] < rmse[0]


# ------------------------------------------------ the estimator surface
def _cpu_engine_factory(u, i, r, n_users, n_items, k, kernel, dtype, device, gamma=0.0,
                        min_rating=0.0, max_rating=5.0, global_mean=0.0):
    return CpuEngine(u, i, r.astype(np.float64), n_users, n_items, k, global_mean)


FIT_HP = dict(n_factors=K, n_epochs=EPOCHS, lr=LR, reg=REG, min_rating=1, max_rating=5,
              verbose=0, schedule="strata")


def _frame():
    import pandas as pd

    u, i, r, _, _ = _data()
    # external ids differ from internal ones (first appearance after the shuffle)
    return pd.DataFrame({"user_id": u * 7 + 3, "item_id": i * 5 + 1}), pd.Series(r)


def _fit_rank(rank, world, port, out_dir, exchange="delta"):
    """KernelMF(distributed=True).fit on every rank: the product's sharding,
    per-epoch draws, delta all-reduce and final gathers; the device sweeps
    are the CPU test double."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import matrix_factorization as mf
    import matrix_factorization.distributed as D

    D.SGDEngine = _cpu_engine_factory
    D.ReplicaExchange = _exchange_cls()
    X, y = _frame()
    np.random.seed(SEED)
    m = mf.KernelMF(distributed=True, exchange=exchange, **FIT_HP).fit(X, y)
    np.savez(os.path.join(out_dir, f"fit{rank}.npz"), P=m.user_features, Q=m.item_features,
             bu=m.user_biases, bi=m.item_biases, rmse=np.asarray(m.train_rmse),
             uids=np.asarray(list(m.user_id_map)), iids=np.asarray(list(m.item_id_map)))
    dist.destroy_process_group()


def _simulate_fit(world, blocks=None):
    """Single-process restatement of KernelMF(distributed=True).fit: the
    reference's draws (sample, normal(P), normal(Q)), then per epoch one
    np.random.randint shared by all ranks, rank r's strata drawn from
    RandomState([draw, r]); replica = start + sum of the rank deltas."""
    import matrix_factorization as mf
    from matrix_factorization.distributed import local_shard, shard_users
    from matrix_factorization.engine import stratum_order

    X, y = _frame()
    np.random.seed(SEED)
    m = mf.KernelMF(**FIT_HP)
    Xp = m._preprocess_data(X=X, y=y, type="fit")
    mu = Xp["rating"].mean()
    P = np.random.normal(0, 0.1, (m.n_users, K))
    Q = np.random.normal(0, 0.1, (m.n_items, K))
    u = Xp["user_id"].to_numpy(np.int32)
    i = Xp["item_id"].to_numpy(np.int32)
    r = Xp["rating"].to_numpy(np.float64)
    bounds = shard_users(u, m.n_users, world)
    engs = []
    for rank in range(world):
        lu, li, lr_ = local_shard(u, i, r, bounds, rank)
        lo, hi = int(bounds[rank]), int(bounds[rank + 1])
        e = CpuEngine(lu, li, lr_, hi - lo, m.n_items, K, mu)
        e.load_params(P=P[lo:hi], bu=np.zeros(hi - lo), Q=Q, bi=np.zeros(m.n_items))
        if blocks == "auto":            # the GPU engine's own choice of B and classes
            from matrix_factorization.engine import auto_strata_classes, choose_strata_blocks
            B = choose_strata_blocks(lu, li, hi - lo, m.n_items, K, 1)[0]
            C = auto_strata_classes("linear", len(lu), m.n_items, B)
            if C > 1:
                B = choose_strata_blocks(lu, li, hi - lo, m.n_items, K, 1, classes=C)[0]
            e.prepare_strata(B, classes=C)
        else:
            e.prepare_strata(blocks)
        engs.append(e)
    bi = np.zeros(m.n_items)
    sse = np.zeros(EPOCHS)
    for ep in range(EPOCHS):
        draw = int(np.random.randint(0, 2**31 - 1))
        dQ, dbi = np.zeros_like(Q), np.zeros_like(bi)
        for rank, e in enumerate(engs):
            e.Q = torch.as_tensor(Q.copy())
            e.bi = torch.as_tensor(bi.copy())
            rs = np.random.RandomState([draw, rank])
            seq = stratum_order(rs, e.strata)
            e.epoch_strata(seq, int(rs.randint(0, 2**31 - 1)), LR, REG)
            dQ += e.Q.numpy() - Q
            dbi += e.bi.numpy() - bi
        Q, bi = Q + _scale(world) * dQ, bi + _scale(world) * dbi
        for e in engs:
            e.Q = torch.as_tensor(Q.copy())
            e.bi = torch.as_tensor(bi.copy())
            e.sse_async(ep)
            sse[ep] += float(e.sse_buf[ep])
    P = np.concatenate([e.P.numpy() for e in engs])
    bu = np.concatenate([e.bu.numpy() for e in engs])
    return P, Q, bu, bi, np.sqrt(sse / len(u))


@pytest.mark.timeout(300)
def test_kernelmf_distributed_fit_two_ranks(tmp_path):
    """The estimator's process-group mode (row 8(e) through fit()): both
    ranks end with the same full model, equal to the restated algorithm."""
    world = 2
    mp.start_processes(_fit_rank, args=(world, _free_port(), str(tmp_path), "delta"),
                       nprocs=world, join=True, start_method="spawn")
    res = [dict(np.load(tmp_path / f"fit{k}.npz")) for k in range(world)]
    for key in ("P", "Q", "bu", "bi", "rmse", "uids", "iids"):
        assert np.array_equal(res[0][key], res[1][key]), key
    P, Q, bu, bi, rmse = _simulate_fit(world)
    for key, ref in (("P", P), ("Q", Q), ("bu", bu), ("bi", bi), ("rmse", rmse)):
        assert np.max(np.abs(res[0][key] - ref)) < 1e-12, key
    assert rmse[-1] < rmse[0]


# ------------------------------------------------ exchange="rotate" (exact)
def _mapped():
    """The fit frame after the reference's preprocessing and initial draws
    (sample, normal(P), normal(Q)): internal ids, ratings, P0, Q0."""
    import matrix_factorization as mf

    X, y = _frame()
    np.random.seed(SEED)
    m = mf.KernelMF(**FIT_HP)
    Xp = m._preprocess_data(X=X, y=y, type="fit")
    P = np.random.normal(0, 0.1, (m.n_users, K))
    Q = np.random.normal(0, 0.1, (m.n_items, K))
    return (Xp["user_id"].to_numpy(np.int32), Xp["item_id"].to_numpy(np.int32),
            Xp["rating"].to_numpy(np.float64), m.n_users, m.n_items, P, Q,
            float(Xp["rating"].mean()))


def _replay(world):
    """RotationReplay (the product's one-process form of the N-rank rotation)
    on the CPU test double, with the fit's draws: (P, Q, bu, bi, rmse, draws,
    replay)."""
    from matrix_factorization.distributed import RotationReplay

    u, i, r, nu, ni, P0, Q0, mu = _mapped()
    rp = RotationReplay(u, i, r, nu, ni, world, K, "linear", "float64", None,
                        global_mean=mu, engine_cls=_cpu_engine_factory)
    rp.load(P0, Q0, np.zeros(nu), np.zeros(ni))
    draws, sse = [], []
    for ep in range(EPOCHS):
        draws.append(int(np.random.randint(0, 2**31 - 1)))   # the fit's one draw per epoch
        rp.epoch(draws[-1], LR, REG, epoch=ep)
        sse.append(rp.sse(ep))
    P, Q, bu, bi = rp.params()
    return P, Q, bu, bi, np.sqrt(np.asarray(sse) / len(u)), draws, rp


def test_item_ranges_cover_and_balance():
    from matrix_factorization.distributed import item_ranges

    u, i, r, _, _ = _data()
    for world in (1, 2, 3, 8):
        b = item_ranges(i, NI, world)
        assert b[0] == 0 and b[-1] == NI and np.all(np.diff(b) > 0)
    # a degenerate skew (every rating on item 0) still leaves no range empty
    b = item_ranges(np.zeros(100, np.int32), 10, 4)
    assert b[0] == 0 and b[-1] == 10 and np.all(np.diff(b) > 0)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 3])
def test_rotation_epoch_is_a_sequential_sweep(world):
    """Every rotation epoch equals the oracle's plain sequential sweep over
    RotationReplay.serial_order (each rating once, with the current user AND
    item rows): the exchange is exact, not an approximation."""
    u, i, r, nu, ni, P0, Q0, mu = _mapped()
    P, Q, bu, bi, rmse, draws, rp = _replay(world)
    Po, Qo, buo, bio = P0.copy(), Q0.copy(), np.zeros(nu), np.zeros(ni)
    sse = []
    for ep, d in enumerate(draws):
        order = rp.serial_order(d, ep)
        assert np.array_equal(np.sort(order), np.arange(len(u)))     # each rating once
        oracle.sgd_pass(u, i, r, mu, buo, bio, Po, Qo, lr=LR, reg=REG, order=order)
        sse.append(oracle.sse(u, i, r, mu, buo, bio, Po, Qo))
    for got, ref in ((P, Po), (Q, Qo), (bu, buo), (bi, bio)):
        assert np.max(np.abs(got - ref)) < 1e-12
    assert np.max(np.abs(rmse - np.sqrt(np.asarray(sse) / len(u)))) < 1e-12
    assert rmse[-1] < rmse[0]


@pytest.mark.timeout(300)
def test_kernelmf_distributed_rotate_two_ranks(tmp_path):
    """KernelMF(distributed=True, exchange="rotate").fit on two gloo ranks:
    the product's item ranges, ring hand-offs (batched send / recv) and
    final all-gather; both ranks end with the same model, equal to the
    one-process replay of the same draws."""
    world = 2
    mp.start_processes(_fit_rank, args=(world, _free_port(), str(tmp_path), "rotate"),
                       nprocs=world, join=True, start_method="spawn")
    res = [dict(np.load(tmp_path / f"fit{k}.npz")) for k in range(world)]
    for key in ("P", "Q", "bu", "bi", "rmse", "uids", "iids"):
        assert np.array_equal(res[0][key], res[1][key]), key
    P, Q, bu, bi, rmse, _, _ = _replay(world)
    for key, ref in (("P", P), ("Q", Q), ("bu", bu), ("bi", bi), ("rmse", rmse)):
        assert np.max(np.abs(res[0][key] - ref)) < 1e-12, key


def test_relabelled_item_ranges_helpers():
    """The rotation's item relabellings (distributed.RotationSet): fixed
    permutations drawn from their own RandomStates (the global one is not
    touched), a pick per epoch draw, balanced ranges over the new ids, and
    exact row moves between labellings."""
    from matrix_factorization.distributed import (_moves, item_relabellings, relabel_pick,
                                                  relabel_ranges, relabel_rows)

    u, i, r, _, _ = _data()
    st = np.random.get_state()
    perms = item_relabellings(NI, 8)
    assert np.array_equal(np.random.get_state()[1], st[1])        # global RNG untouched
    assert perms[0] is None and len(perms) == 8
    for p in perms[1:]:
        assert np.array_equal(np.sort(p), np.arange(NI))
    assert not np.array_equal(perms[1], perms[2])
    picks = [relabel_pick(d, 8) for d in range(2000)]
    assert set(picks) == set(range(8)) and relabel_pick(123, 1) == 0
    assert picks == [relabel_pick(d, 8) for d in range(2000)]      # a function of the draw
    for p in perms:
        b = relabel_ranges(i, NI, 4, p)
        ids = i if p is None else p[i]
        cnt = np.array([np.sum((ids >= b[c]) & (ids < b[c + 1])) for c in range(4)])
        assert b[0] == 0 and b[-1] == NI and cnt.max() - cnt.min() <= 2 * np.bincount(i).max()
    mv = _moves(perms, torch.device("cpu"))
    Q = torch.as_tensor(np.random.RandomState(3).normal(size=(NI, K)))
    A, Bq, C = torch.empty_like(Q), torch.empty_like(Q), torch.empty_like(Q)
    relabel_rows(Q, A, mv, 0, 3)                  # canonical -> labelling 3
    assert torch.equal(A[torch.as_tensor(perms[3])], Q)
    relabel_rows(A, Bq, mv, 3, 5)                 # 3 -> 5
    assert torch.equal(Bq[torch.as_tensor(perms[5])], Q)
    relabel_rows(Bq, C, mv, 5, 0)                 # 5 -> canonical
    assert torch.equal(C, Q)


@pytest.mark.timeout(300)
def test_rotation_relabel_one_is_the_plain_rotation():
    """relabel=1 is the rotation without relabellings (the round-5 product
    path), and the default (8 relabellings) trains a different sequential
    order from the same draws -- the relabellings are in use."""
    from matrix_factorization.distributed import RotationReplay, relabel_pick

    u, i, r, nu, ni, P0, Q0, mu = _mapped()
    draws = [int(d) for d in np.random.RandomState(4).randint(0, 2**31 - 1, EPOCHS)]
    assert any(relabel_pick(d, 8) != 0 for d in draws)
    out = {}
    for K_ in (1, 8):
        rp = RotationReplay(u, i, r, nu, ni, 2, K, "linear", "float64", None,
                            global_mean=mu, engine_cls=_cpu_engine_factory, relabel=K_)
        rp.load(P0, Q0, np.zeros(nu), np.zeros(ni))
        orders = []
        for ep, d in enumerate(draws):
            orders.append(rp.serial_order(d, ep))
            rp.epoch(d, LR, REG, epoch=ep)
        out[K_] = (orders, rp.params())
    # K = 1: the plain rotation's order, item ranges over canonical ids
    from matrix_factorization.distributed import item_ranges
    ilo = item_ranges(i, ni, 2)
    first = out[1][0][0]                     # epoch 0 starts with rank 0's first range
    c0 = (i[first[:10]] >= ilo[0]) & (i[first[:10]] < ilo[1])
    assert c0.all() or (~c0).all()
    # relabelled epochs are another order (and another model)
    assert any(not np.array_equal(a, b) for a, b in zip(out[1][0], out[8][0]))
    assert np.max(np.abs(out[1][1][1] - out[8][1][1])) > 0

"""Sharded training on the GPU box: two ranks share cuda:0 (gloo carries the
collective; RCCL needs one GPU per rank, which the 8-GPU driver run uses).
The device path is the product one: libmf_hip.so sweeps, mf_replica_delta,
all_reduce of the flat [Q | b_i] replica."""

import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _rank(rank, world, port, out, schedule="colored"):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch

    dist.init_process_group("gloo", rank=rank, world_size=world)
    from matrix_factorization.distributed import (ReplicaExchange, global_rmse, local_shard,
                                                  shard_users, sharded_epochs)
    from matrix_factorization.engine import SGDEngine
    from test_distributed_cpu import EPOCHS, K, LR, NI, NNZ, NU, REG, SEED, STRATA_B, _data

    u, i, r, P0, Q0 = _data()
    mu = float(r.mean())
    b = shard_users(u, NU, world)
    lu, li, lr_ = local_shard(u, i, r, b, rank)
    lo, hi = int(b[rank]), int(b[rank + 1])
    eng = SGDEngine(lu, li, lr_, hi - lo, NI, K, "linear", "float64", "cuda:0",
                    global_mean=mu)
    eng.load_params(P=P0[lo:hi], bu=np.zeros(hi - lo))
    ex = ReplicaExchange(eng)
    ex.bind(Q0, np.zeros(NI))
    sharded_epochs(eng, ex, EPOCHS, LR, REG, SEED, schedule=schedule, n_blocks=STRATA_B)
    rm = global_rmse(eng, EPOCHS, NNZ)
    P, Q, bu, bi = eng.params_numpy()
    np.savez(os.path.join(out, f"g{rank}.npz"), P=P, Q=Q, bi=bi, rmse=np.array(rm))
    dist.destroy_process_group()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("schedule", ["colored", "strata"])
def test_two_ranks_on_one_gpu_match_cpu_simulation(tmp_path, schedule):
    """strata: both ranks' persistent kernels (3 workgroups each) share the
    card; the result is the serial-order simulation's."""
    from test_distributed_cpu import _free_port, _simulate

    world = 2
    mp.start_processes(_rank, args=(world, _free_port(), str(tmp_path), schedule),
                       nprocs=world, join=True, start_method="spawn")
    res = [dict(np.load(tmp_path / f"g{k}.npz")) for k in range(world)]
    assert np.array_equal(res[0]["Q"], res[1]["Q"])
    Q, bi, rmse, engs, bounds = _simulate(world, schedule)
    assert np.max(np.abs(res[0]["Q"] - Q)) < 1e-10
    assert np.max(np.abs(res[0]["bi"] - bi)) < 1e-10
    for k in range(world):
        assert np.max(np.abs(res[k]["P"] - engs[k].P.numpy())) < 1e-10
    assert np.max(np.abs(res[0]["rmse"] - rmse)) < 1e-10


def _fit_rank(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import matrix_factorization as mf
    from test_distributed_cpu import FIT_HP, SEED, _frame

    X, y = _frame()
    np.random.seed(SEED)
    m = mf.KernelMF(distributed=True, exchange="delta", device="cuda:0", **FIT_HP).fit(X, y)
    np.savez(os.path.join(out, f"fit{rank}.npz"), P=m.user_features, Q=m.item_features,
             bu=m.user_biases, bi=m.item_biases, rmse=np.asarray(m.train_rmse),
             pred=np.asarray(m.predict(X.iloc[:50])))
    dist.destroy_process_group()


@pytest.mark.timeout(600)
def test_kernelmf_distributed_fit_on_one_gpu(tmp_path):
    """KernelMF(distributed=True, exchange="delta").fit with two gloo ranks sharing cuda:0: the
    product path end to end (delta-out persistent sweeps, all-reduce,
    mf_replica_delta, gathers); equal to the restated algorithm."""
    from test_distributed_cpu import _free_port, _simulate_fit

    world = 2
    mp.start_processes(_fit_rank, args=(world, _free_port(), str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    res = [dict(np.load(tmp_path / f"fit{k}.npz")) for k in range(world)]
    for key in ("P", "Q", "bu", "bi", "rmse", "pred"):
        assert np.array_equal(res[0][key], res[1][key]), key
    P, Q, bu, bi, rmse = _simulate_fit(world, blocks="auto")
    for key, ref in (("P", P), ("Q", Q), ("bu", bu), ("bi", bi), ("rmse", rmse)):
        assert np.max(np.abs(res[0][key] - ref)) < 1e-10, key


# ------------------------------------------------ exchange="rotate" (exact)
def _fit_rank_rotate(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import matrix_factorization as mf
    from test_distributed_cpu import FIT_HP, SEED, _frame

    X, y = _frame()
    np.random.seed(SEED)
    m = mf.KernelMF(distributed=True, exchange="rotate", device="cuda:0", **FIT_HP).fit(X, y)
    np.savez(os.path.join(out, f"rot{rank}.npz"), P=m.user_features, Q=m.item_features,
             bu=m.user_biases, bi=m.item_biases, rmse=np.asarray(m.train_rmse))
    dist.destroy_process_group()


def _gpu_replay(world, persistent=None):
    """RotationReplay on cuda:0 (the product engines) with the fit's draws."""
    from matrix_factorization.distributed import RotationReplay
    from test_distributed_cpu import EPOCHS, K, LR, REG, _mapped

    u, i, r, nu, ni, P0, Q0, mu = _mapped()
    rp = RotationReplay(u, i, r, nu, ni, world, K, "linear", "float64", "cuda:0",
                        min_rating=1, max_rating=5, global_mean=mu)
    rp.load(P0, Q0, np.zeros(nu), np.zeros(ni))
    sse, draws = [], []
    for ep in range(EPOCHS):
        draws.append(int(np.random.randint(0, 2**31 - 1)))
        rp.epoch(draws[-1], LR, REG, persistent=persistent, epoch=ep)
        sse.append(rp.sse(ep))
    return rp.params() + (np.sqrt(np.asarray(sse) / len(u)), rp, draws)


@pytest.mark.timeout(600)
def test_kernelmf_distributed_rotate_on_one_gpu(tmp_path):
    """KernelMF(distributed=True, exchange="rotate") with two gloo ranks
    sharing cuda:0: item ranges handed round the ring (staged through host
    memory under gloo), final all-gather; both ranks equal, bit-equal to the
    one-GPU RotationReplay of the same draws, and equal to the oracle's
    sequential sweep of that replay's stated serial order to FP64
    rounding."""
    import oracle
    from test_distributed_cpu import EPOCHS, LR, REG, _free_port, _mapped

    world = 2
    mp.start_processes(_fit_rank_rotate, args=(world, _free_port(), str(tmp_path)),
                       nprocs=world, join=True, start_method="spawn")
    res = [dict(np.load(tmp_path / f"rot{k}.npz")) for k in range(world)]
    for key in ("P", "Q", "bu", "bi", "rmse"):
        assert np.array_equal(res[0][key], res[1][key]), key
    P, Q, bu, bi, rmse, rp, draws = _gpu_replay(world)
    for key, ref in (("P", P), ("Q", Q), ("bu", bu), ("bi", bi)):
        assert np.array_equal(res[0][key], ref), key
    assert np.max(np.abs(res[0]["rmse"] - rmse)) < 1e-13
    u, i, r, nu, ni, Po, Qo, mu = _mapped()
    buo, bio, sse = np.zeros(nu), np.zeros(ni), []
    for ep, d in enumerate(draws):
        order = rp.serial_order(d, ep)
        assert np.array_equal(np.sort(order), np.arange(len(u)))
        oracle.sgd_pass(u, i, r, mu, buo, bio, Po, Qo, lr=LR, reg=REG, order=order)
        sse.append(oracle.sse(u, i, r, mu, buo, bio, Po, Qo))
    rmo = np.sqrt(np.asarray(sse) / len(u))
    assert EPOCHS == len(draws)
    for key, ref in (("P", Po), ("Q", Qo), ("bu", buo), ("bi", bio), ("rmse", rmo)):
        assert np.max(np.abs(res[0][key] - ref)) < 1e-10, key


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world", [3, 4])
def test_rotation_replay_mid_size_matches_oracle_order(world):
    """A mid-size rotation (20K users x 3K items, 300K ratings, rank 16, FP64,
    N = 3 / 4 virtual ranks, default plans): every epoch equals the oracle's
    sequential sweep over RotationReplay.serial_order; persistent sub-epochs
    are bit-identical to one launch per stratum."""
    import oracle
    from matrix_factorization.distributed import RotationReplay

    rs = np.random.RandomState(5)
    nu, ni, n, k = 20000, 3000, 300000, 16
    keys = rs.choice(nu * ni, n, replace=False)
    u, i = (keys // ni).astype(np.int32), (keys % ni).astype(np.int32)
    r = rs.randint(1, 6, n).astype(np.float64)
    mu = float(r.mean())
    P0, Q0 = rs.normal(0, 0.1, (nu, k)), rs.normal(0, 0.1, (ni, k))
    out = []
    for persistent in (None, False):
        rp = RotationReplay(u, i, r, nu, ni, world, k, "linear", "float64", "cuda:0",
                            min_rating=1, max_rating=5, global_mean=mu)
        rp.load(P0, Q0, np.zeros(nu), np.zeros(ni))
        for ep, d in enumerate((11, 12)):
            rp.epoch(d, 0.01, 0.02, persistent=persistent, epoch=ep)
        out.append(rp.params())
        if persistent is None:
            orders = [rp.serial_order(d, ep) for ep, d in enumerate((11, 12))]
    for a, b in zip(*out):
        assert np.array_equal(a, b)
    Po, Qo, buo, bio = P0.copy(), Q0.copy(), np.zeros(nu), np.zeros(ni)
    for order in orders:
        assert np.array_equal(np.sort(order), np.arange(n))
        oracle.sgd_pass(u, i, r, mu, buo, bio, Po, Qo, lr=0.01, reg=0.02, order=order)
    for got, ref in zip(out[0], (Po, Qo, buo, bio)):
        assert np.max(np.abs(got - ref)) < 1e-10

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
    m = mf.KernelMF(distributed=True, device="cuda:0", **FIT_HP).fit(X, y)
    np.savez(os.path.join(out, f"fit{rank}.npz"), P=m.user_features, Q=m.item_features,
             bu=m.user_biases, bi=m.item_biases, rmse=np.asarray(m.train_rmse),
             pred=np.asarray(m.predict(X.iloc[:50])))
    dist.destroy_process_group()


@pytest.mark.timeout(600)
def test_kernelmf_distributed_fit_on_one_gpu(tmp_path):
    """KernelMF(distributed=True).fit with two gloo ranks sharing cuda:0: the
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

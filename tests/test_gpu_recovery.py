"""Recovery of the persistent strata sweep (a workgroup that gives up waiting
for its neighbour leaves invalid parameters behind; the error word is sticky).

``mf_strata_inject_fail(n)`` starts the next n persistent launches with the
error word set, exactly as a timed-out wait leaves it.  KernelMF.fit then
restores its start snapshot and replays the epochs with the same draws as
per-stratum launches (engine.fit_epochs); in process-group mode every rank
learns of a failure on ANY rank through one MAX all-reduce and all replay
together (distributed.fit_sharded), so no rank is left waiting in a
collective and no stale delta is applied.  The results must equal a clean
fit bit for bit (the replay is the same sequential order)."""

import os
import warnings

import numpy as np
import pandas as pd
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

HP = dict(n_factors=16, n_epochs=3, lr=0.01, reg=0.02, min_rating=1, max_rating=5,
          schedule="strata", dtype="float64", device="cuda:0")


def _frame(seed=4, nu=3000, ni=400, n=40000):
    rs = np.random.RandomState(seed)
    keys = rs.choice(nu * ni, n, replace=False)
    return (pd.DataFrame({"user_id": keys // ni, "item_id": keys % ni}),
            pd.Series(rs.randint(1, 6, n).astype(np.float64)))


def _fit(verbose, inject, **kw):
    import matrix_factorization as mf
    from matrix_factorization import _lib

    X, y = _frame()
    np.random.seed(3)
    _lib.call("mf_strata_inject_fail", inject)
    try:
        with warnings.catch_warnings(record=True) as w:
            warnings.simplefilter("always")
            m = mf.KernelMF(verbose=verbose, **HP, **kw).fit(X, y)
    finally:
        _lib.call("mf_strata_inject_fail", 0)
    replayed = any(issubclass(x.category, RuntimeWarning) and "replayed" in str(x.message)
                   for x in w)
    return m, replayed


@pytest.mark.parametrize("verbose", [0, 1])
def test_fit_replays_after_a_failed_persistent_sweep(verbose):
    clean, r0 = _fit(verbose, 0)
    hurt, r1 = _fit(verbose, 1)
    assert not r0 and r1
    for a in ("user_features", "item_features", "user_biases", "item_biases"):
        assert np.array_equal(getattr(clean, a), getattr(hurt, a)), a
    assert np.array_equal(np.asarray(clean.train_rmse), np.asarray(hurt.train_rmse))


def _rank(rank, world, port, out, exchange, inject_rank):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    m, replayed = _fit(0, 2 if rank == inject_rank else 0, distributed=True, exchange=exchange)
    np.savez(os.path.join(out, f"r{rank}_{inject_rank}.npz"), P=m.user_features,
             Q=m.item_features, bu=m.user_biases, bi=m.item_biases,
             rmse=np.asarray(m.train_rmse), replayed=replayed)
    dist.destroy_process_group()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("exchange", ["rotate", "delta"])
def test_sharded_fit_replays_on_every_rank(tmp_path, exchange):
    """Two gloo ranks on cuda:0; rank 1's first two persistent launches
    'fail'.  Both ranks replay (both warn), nobody hangs, and the model equals
    the clean two-rank fit bit for bit."""
    from test_distributed_cpu import _free_port

    world = 2
    for inject_rank in (-1, 1):
        mp.start_processes(_rank, args=(world, _free_port(), str(tmp_path), exchange,
                                        inject_rank),
                           nprocs=world, join=True, start_method="spawn")
    clean = [dict(np.load(tmp_path / f"r{k}_-1.npz")) for k in range(world)]
    hurt = [dict(np.load(tmp_path / f"r{k}_1.npz")) for k in range(world)]
    assert not any(bool(c["replayed"]) for c in clean)
    assert all(bool(h["replayed"]) for h in hurt)
    for k in range(world):
        for key in ("P", "Q", "bu", "bi", "rmse"):
            assert np.array_equal(clean[k][key], hurt[k][key]), (k, key)

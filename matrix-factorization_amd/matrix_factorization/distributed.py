"""User-sharded data parallelism across the GPUs of one node.

One process per GPU (torch.distributed, backend "nccl" = RCCL on ROCm; "gloo"
for CPU rehearsal of the control flow).  The reference is single-process; this
is the build's multi-GPU extension of the same epoch:

* users are split into contiguous internal-id ranges balanced by rating count;
  a rank owns its users' rows of P and b_u and all of their ratings;
* Q and b_i are replicated and kept in ONE flat buffer [Q | b_i], so the
  exchange is a single collective;
* per epoch (strata): the local persistent sweep runs in delta-out form
  (mf_sgd_epoch_strata_delta: the replica is not written, the slab's update
  lands in a flat delta buffer where the slab would have been written back),
  ``all_reduce(SUM)`` of the delta over xGMI, one element-wise apply
  (replica += scale * sum, scale = min(1/2, 2/world): default_delta_scale)
  -- every rank ends the epoch with the same replica and no snapshot copy is
  taken.  The colored schedule keeps the snapshot form
  (snapshot, sweep, take, all-reduce, apply);
* the training SSE of every epoch stays on the device and is summed across
  ranks once (or per epoch when the caller prints it).

Item updates are thereby delayed by up to one epoch relative to the
sequential sweep and combined with a damped sum (user updates are exact):
RMSE is reported next to the 1-GPU run, not claimed identical.  The plain
sum of the deltas (scale 1, "all-reduce of the gradients") is available but
is not the default: each rank's local epoch moves an item much of the way
toward its local optimum, so N summed moves overshoot and C3 diverges at
N >= 4 (default_delta_scale has the measurements).

``fit_sharded`` is the estimator's process-group mode (KernelMF(...,
distributed=True).fit on every rank with the same data and RNG state).
"""

from __future__ import annotations

from typing import Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist

from . import _lib
from .engine import SGDEngine, _tp


def world_info(group=None) -> Tuple[int, int]:
    """(world size, rank) of the default (or given) process group; (1, 0)
    when torch.distributed is not initialised."""
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(group), dist.get_rank(group)
    return 1, 0


def shard_users(user_ids: np.ndarray, n_users: int, world: int) -> np.ndarray:
    """Contiguous user-id range boundaries (world + 1 values) with about
    equal rating counts per range."""
    deg = np.bincount(user_ids, minlength=n_users).astype(np.int64)
    cum = np.concatenate([[0], np.cumsum(deg)])
    total = cum[-1]
    bounds = [0]
    for r in range(1, world):
        bounds.append(int(np.searchsorted(cum, total * r / world, side="left")))
    bounds.append(n_users)
    return np.maximum.accumulate(np.asarray(bounds, np.int64))


def local_shard(u: np.ndarray, i: np.ndarray, r: np.ndarray, bounds: np.ndarray,
                rank: int) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """The ratings of rank ``rank``'s users, user ids made local."""
    lo, hi = int(bounds[rank]), int(bounds[rank + 1])
    m = (u >= lo) & (u < hi)
    return (u[m] - lo).astype(np.int32), i[m].astype(np.int32), r[m]


def default_delta_scale(world: int) -> float:
    """Weight of the all-reduced sum of the rank-local item deltas:
    min(1/2, 2/world) (1 for one rank).

    Each rank's epoch moves an item part of the way toward the optimum of
    that rank's ratings; the plain sum (1.0) overshoots by up to ~world and
    diverges, plain averaging (1/world) under-steps.  Measured at C3 (lr
    0.01, reg 0.02, final train RMSE after 20 epochs; N = 1: 0.7106;
    DESIGN.md section 6): N = 2: 0.7434 at 1/2, 0.7887 at 1; N = 4: 0.7469 at
    1/2, 0.7974 at 1/4, NaN at 1; N = 8: 0.7977 at 1/4, 0.8706 at 1/8, 2.29
    at 3/8, NaN at 1/2.  2/world sits below the divergence edge (between 2/N
    and 3/N at N = 8) with the best RMSE measured."""
    if world <= 1:
        return 1.0
    return min(0.5, 2.0 / world)


class ReplicaExchange:
    """The per-epoch delta all-reduce of the replicated item parameters.

    ``flat`` is the device buffer holding [Q (n_items*k) | b_i (n_items)];
    the engine's Q and b_i must be views into it (see ``bind``).  ``delta``
    has the same layout (strata: the delta-out target; colored: the
    start-of-epoch snapshot)."""

    def __init__(self, engine: SGDEngine, group=None, scale: Optional[float] = None):
        self.e = engine
        self.group = group
        # weight of the summed deltas (default_delta_scale); 1.0 is the plain
        # gradient-sum form, 1 / world plain model averaging
        self.scale = (default_delta_scale(world_info(group)[0]) if scale is None
                      else float(scale))
        n, k = engine.n_items, engine.k
        self.flat = torch.empty(n * k + n, dtype=engine.tdt, device=engine.dev)
        self.delta = torch.zeros_like(self.flat)
        self.dq = self.delta[: n * k].view(n, k)
        self.dbi = self.delta[n * k:]

    def bind(self, Q, bi) -> None:
        """Upload Q / b_i into the flat buffer and point the engine at it."""
        n, k = self.e.n_items, self.e.k
        self.e.load_params(Q=Q, bi=bi)
        self.flat[: n * k].copy_(self.e.Q.reshape(-1))
        self.flat[n * k:].copy_(self.e.bi)
        self.e.Q = self.flat[: n * k].view(n, k)
        self.e.bi = self.flat[n * k:]

    def _delta(self, mode: int) -> None:
        """mf_replica_delta(flat, delta): TAKE flat -= delta, APPLY flat += delta."""
        e = self.e
        with torch.cuda.device(e.dev):
            _lib.call("mf_replica_delta", _tp(self.flat), _tp(self.delta), self.flat.numel(),
                      e.dcode, mode, e.stream)

    def _reduce(self) -> None:
        dist.all_reduce(self.delta, op=dist.ReduceOp.SUM, group=self.group)

    def _apply(self) -> None:
        """mf_replica_apply: flat += scale * delta."""
        e = self.e
        with torch.cuda.device(e.dev):
            _lib.call("mf_replica_apply", _tp(self.flat), _tp(self.delta), self.flat.numel(),
                      e.dcode, self.scale, e.stream)

    # ---- strata: delta-out sweep, all-reduce, apply
    def strata_epoch(self, seq, seed, lr, reg, update_user=True, update_item=True,
                     timing=False):
        ms = self.e.epoch_strata(seq, seed, lr, reg, update_user, update_item, timing=timing,
                                 delta=(self.dq, self.dbi))
        self.exchange()
        return ms

    def exchange(self) -> None:
        """delta = sum over ranks of the local deltas; flat += scale * delta."""
        self._reduce()
        self._apply()

    # ---- colored (and any in-place sweep): snapshot form
    def begin_epoch(self) -> None:
        self.delta.copy_(self.flat)

    def end_epoch(self) -> None:
        # flat = flat - snapshot (local delta); sum; flat = snapshot + sum
        self._delta(_lib.MF_DELTA_TAKE)
        self.flat, self.delta = self.delta, self.flat       # delta holds the local delta
        self._rebind()
        self._reduce()
        self._apply()                                       # flat (snapshot) += scale * sum

    def _rebind(self) -> None:
        n, k = self.e.n_items, self.e.k
        self.e.Q = self.flat[: n * k].view(n, k)
        self.e.bi = self.flat[n * k:]
        self.dq = self.delta[: n * k].view(n, k)
        self.dbi = self.delta[n * k:]


def epoch_draws(rs: np.random.RandomState, nb: int, strata: bool):
    """Stratum (colour) order and step rotation of one epoch."""
    seq = rs.permutation(nb).astype(np.int32)
    rot = int(rs.randint(0, 2**31 - 1)) if strata else 0
    return seq, rot


def sharded_epochs(engine: SGDEngine, exchange: Optional[ReplicaExchange], n_epochs: int,
                   lr: float, reg: float, seed: int, first_epoch: int = 0,
                   timing: bool = False, schedule: str = "colored",
                   n_blocks: Optional[int] = None) -> list:
    """Run ``schedule`` ("colored" or "strata") epochs on this rank; returns
    per-epoch SGD kernel timings (timing) -- the SSE of epoch j lands in
    engine.sse_buf[first_epoch + j].  Epoch ep draws its colour / stratum
    order (and, for strata, the step rotation) from RandomState(seed, ep), so
    every rank's draws are reproducible on their own.  ``n_blocks``: strata
    B for this rank's plan (default: engine.choose_strata_blocks)."""
    strata = schedule == "strata"
    if schedule not in ("colored", "strata"):
        raise ValueError(f"schedule must be 'colored' or 'strata', got {schedule!r}")
    if strata:
        if engine.strata is None:
            engine.prepare_strata(n_blocks=n_blocks)
        nb = engine.strata.B
    else:
        if engine.colored is None:
            engine.prepare_colored()
        nb = len(engine.colored) - 1
    kms = []
    for j in range(n_epochs):
        ep = first_epoch + j
        seq, rot = epoch_draws(np.random.RandomState((seed * 1000003 + ep) & 0x7FFFFFFF), nb,
                               strata)
        if strata:
            if exchange is not None:
                ms = exchange.strata_epoch(seq, rot, lr, reg, timing=timing)
            else:
                ms = engine.epoch_strata(seq, rot, lr, reg, timing=timing)
        else:
            if exchange is not None:
                exchange.begin_epoch()
            ms = engine.epoch_colored(seq, lr, reg, timing=timing)
            if exchange is not None:
                exchange.end_epoch()
        engine.sse_async(ep)
        kms.append(ms)
    if strata:
        engine.check_strata()
    return kms


def global_rmse(engine: SGDEngine, n_epochs: int, n_total: int, group=None) -> list:
    """Per-epoch training RMSE over all ranks (one all-reduce for all epochs)."""
    engine.sse_join()                     # an overlapped SSE (sse_overlap) has landed
    sse = engine.sse_buf[:n_epochs].clone()
    if dist.is_available() and dist.is_initialized():
        dist.all_reduce(sse, op=dist.ReduceOp.SUM, group=group)
    sse = sse.cpu().numpy()
    return [float(np.sqrt(s / n_total)) if n_total else float("nan") for s in sse]


def _gather_rows(local: torch.Tensor, bounds: np.ndarray, group=None) -> np.ndarray:
    """All ranks' row blocks (rank r holds rows bounds[r]:bounds[r+1]) as one
    host array on every rank (all_gather of equal-size padded blocks)."""
    world = len(bounds) - 1
    sizes = np.diff(bounds)
    m = int(sizes.max())
    tail = local.shape[1:]
    pad = torch.zeros((m,) + tuple(tail), dtype=local.dtype, device=local.device)
    pad[: local.shape[0]] = local
    if dist.get_backend(group) == "gloo":
        pad = pad.cpu()
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad, group=group)
    return np.concatenate([p[: int(s)].cpu().numpy().astype(np.float64)
                           for p, s in zip(parts, sizes)])


def fit_sharded(u: np.ndarray, i: np.ndarray, r: np.ndarray, n_users: int, n_items: int,
                P0: np.ndarray, Q0: np.ndarray, bu0: np.ndarray, bi0: np.ndarray,
                n_epochs: int, kernel: str, n_factors: int, dtype: str, device, gamma: float,
                min_rating: float, max_rating: float, global_mean: float, lr: float,
                reg: float, schedule: str, verbose: int = 0, update_user: bool = True,
                update_item: bool = True, group=None):
    """KernelMF.fit's epochs in process-group mode (every rank calls it with
    the same ratings, initial parameters and NumPy RNG state).

    Each epoch draws ONE integer from NumPy's global RandomState on every
    rank (the same value: same state) and derives the rank's stratum /
    colour order from (that integer, rank).  Returns (P, Q, b_u, b_i,
    train_rmse) as float64 host arrays, identical on every rank."""
    if schedule not in ("strata", "colored"):
        raise ValueError("distributed fit needs schedule='strata' or 'colored' "
                         "(the exact schedule is one sequential order)")
    world, rank = world_info(group)
    bounds = shard_users(u, n_users, world)
    lu, li, lr_ = local_shard(u, i, r, bounds, rank)
    lo, hi = int(bounds[rank]), int(bounds[rank + 1])
    eng = SGDEngine(lu, li, lr_, hi - lo, n_items, n_factors, kernel, dtype, device,
                    gamma=gamma, min_rating=min_rating, max_rating=max_rating,
                    global_mean=global_mean)
    eng.load_params(P=P0[lo:hi], bu=bu0[lo:hi])
    ex = ReplicaExchange(eng, group)
    ex.bind(Q0, bi0)
    strata = schedule == "strata"
    if strata:
        eng.prepare_strata()
        nb = eng.strata.B
    else:
        eng.prepare_colored()
        nb = len(eng.colored) - 1
    n_total = len(u)
    rmse = []
    for epoch in range(n_epochs):
        draw = int(np.random.randint(0, 2**31 - 1))
        seq, rot = epoch_draws(np.random.RandomState([draw, rank]), nb, strata)
        if strata:
            ex.strata_epoch(seq, rot, lr, reg, update_user, update_item)
        else:
            ex.begin_epoch()
            eng.epoch_colored(seq, lr, reg, update_user, update_item)
            ex.end_epoch()
        eng.sse_async(epoch)
        if verbose == 1:
            rm = global_rmse(eng, epoch + 1, n_total, group)[epoch]
            rmse.append(rm)
            if rank == 0:
                print("Epoch ", epoch + 1, "/", n_epochs, " -  train_rmse:", rm)
    if strata:
        eng.check_strata()
    if verbose != 1:
        rmse = global_rmse(eng, n_epochs, n_total, group)
    P = _gather_rows(eng.P, bounds, group)
    bu = _gather_rows(eng.bu.reshape(-1, 1), bounds, group).reshape(-1)
    Q = eng.Q.cpu().numpy().astype(np.float64)
    bi = eng.bi.cpu().numpy().astype(np.float64)
    return P, Q, bu, bi, rmse, eng

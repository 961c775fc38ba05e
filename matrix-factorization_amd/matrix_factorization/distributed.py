"""User-sharded data parallelism across the GPUs of one node.

One process per GPU (torch.distributed, backend "nccl" = RCCL on ROCm; "gloo"
for CPU rehearsal of the control flow).  The reference is single-process; this
is the build's multi-GPU extension of the same epoch:

* users are split into contiguous internal-id ranges balanced by rating count;
  a rank owns its users' rows of P and b_u and all of their ratings;
* Q and b_i are replicated and kept in ONE flat buffer [Q | b_i], so the
  exchange is a single collective;
* per epoch: snapshot the replica, run the local SGD epoch, take the delta,
  ``all_reduce(SUM)`` the deltas over xGMI, apply ``snapshot + sum`` -- every
  rank ends the epoch with the same replica;
* the training SSE of every epoch stays on the device and is summed across
  ranks once, after the last epoch.

Item updates are thereby delayed by up to one epoch relative to the
sequential sweep (user updates are exact): RMSE is reported next to the
1-GPU run, not claimed identical.
"""

from __future__ import annotations

import ctypes
from typing import Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist

from . import _lib
from .engine import SGDEngine, _tp


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


class ReplicaExchange:
    """The per-epoch delta all-reduce of the replicated item parameters.

    ``flat`` is the device buffer holding [Q (n_items*k) | b_i (n_items)];
    the engine's Q and b_i must be views into it (see ``bind``)."""

    def __init__(self, engine: SGDEngine, group=None):
        self.e = engine
        self.group = group
        n, k = engine.n_items, engine.k
        self.flat = torch.empty(n * k + n, dtype=engine.tdt, device=engine.dev)
        self.snap = torch.empty_like(self.flat)

    def bind(self, Q, bi) -> None:
        """Upload Q / b_i into the flat buffer and point the engine at it."""
        n, k = self.e.n_items, self.e.k
        self.e.load_params(Q=Q, bi=bi)
        self.flat[: n * k].copy_(self.e.Q.reshape(-1))
        self.flat[n * k:].copy_(self.e.bi)
        self.e.Q = self.flat[: n * k].view(n, k)
        self.e.bi = self.flat[n * k:]

    def _delta(self, mode: int) -> None:
        e = self.e
        with torch.cuda.device(e.dev):
            _lib.call("mf_replica_delta", _tp(self.flat), _tp(self.snap), self.flat.numel(),
                      e.dcode, mode, e.stream)

    def begin_epoch(self) -> None:
        self.snap.copy_(self.flat)

    def end_epoch(self) -> None:
        self._delta(_lib.MF_DELTA_TAKE)            # flat = local delta
        dist.all_reduce(self.flat, op=dist.ReduceOp.SUM, group=self.group)
        self._delta(_lib.MF_DELTA_APPLY)           # flat = snapshot + sum of deltas


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
        rs_ep = np.random.RandomState((seed * 1000003 + ep) & 0x7FFFFFFF)
        seq = rs_ep.permutation(nb).astype(np.int32)
        if exchange is not None:
            exchange.begin_epoch()
        if strata:
            rot = int(rs_ep.randint(0, 2**31 - 1))
            ms = engine.epoch_strata(seq, rot, lr, reg, timing=timing)
        else:
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
    sse = engine.sse_buf[:n_epochs].clone()
    if dist.is_available() and dist.is_initialized():
        dist.all_reduce(sse, op=dist.ReduceOp.SUM, group=group)
    sse = sse.cpu().numpy()
    return [float(np.sqrt(s / n_total)) if n_total else float("nan") for s in sse]

"""User-sharded data parallelism across the GPUs of one node.

One process per GPU (torch.distributed, backend "nccl" = RCCL on ROCm; "gloo"
for CPU rehearsal of the control flow).  The reference is single-process; this
is the build's multi-GPU extension of the same epoch.
Users are split into contiguous internal-id ranges balanced by rating count;
a rank owns its users' rows of P and b_u and all of their ratings.  Two ways
to keep the item side consistent:

``exchange="rotate"`` (the default; exact).  Items are cut into N contiguous
ranges too, so the ratings form an N x N grid of sub-blocks (user range r x
item range c).  An epoch is N sub-epochs; in sub-epoch s rank r sweeps its
sub-block with item range c = (r + off + s) mod N -- the N sub-blocks of a
sub-epoch share no user and no item -- in place on its rows of Q / b_i (one
persistent strata launch of that item range's plan, engine.epoch_phase), then
hands the range to rank r - 1 and receives range c + 1 from rank r + 1 (ring
send / recv of n_items / N rows over xGMI).  After the last sub-epoch every
range is final on exactly one rank and one all-gather gives every rank the
whole replica (the training-RMSE pass reads it).  Every rating is applied
with the current user AND item rows: the epoch is the sequential sweep of a
stated serial order (sub-epoch by sub-epoch, ranks in any order), the
strata schedule at GPU granularity -- ``RotationReplay`` runs the same order
on one GPU bit for bit, and the oracle replays it (tests).

``exchange="delta"`` (damped; item updates one epoch late):
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

In delta mode item updates are thereby delayed by up to one epoch relative
to the sequential sweep and combined with a damped sum (user updates are
exact): RMSE is reported next to the 1-GPU run, not claimed identical.  The plain
sum of the deltas (scale 1, "all-reduce of the gradients") is available but
is not the default: each rank's local epoch moves an item much of the way
toward its local optimum, so N summed moves overshoot and C3 diverges at
N >= 4 (default_delta_scale has the measurements).

``fit_sharded`` is the estimator's process-group mode (KernelMF(...,
distributed=True).fit on every rank with the same data and RNG state).
"""

from __future__ import annotations

import warnings
from typing import Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist

from . import _lib
from .engine import SGDEngine, _tp, balanced_bounds, stratum_order


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
                     timing=False, persistent=None, exchange=True):
        """Delta-out sweep, then (``exchange``) all-reduce + apply.  With the
        item side frozen there is nothing to exchange: the sweep runs in place."""
        if not update_item:
            return self.e.epoch_strata(seq, seed, lr, reg, update_user, False, timing=timing,
                                       persistent=persistent)
        ms = self.e.epoch_strata(seq, seed, lr, reg, update_user, update_item, timing=timing,
                                 delta=(self.dq, self.dbi), persistent=persistent)
        if exchange:
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


# ------------------------------------------------------------------ rotate
EXCHANGES = ("rotate", "delta")


def item_ranges(item_ids: np.ndarray, n_items: int, world: int) -> np.ndarray:
    """``world`` contiguous item-id ranges (world + 1 int64 bounds) with about
    equal rating counts: the item ranges the rotation schedule passes round
    the ring.  Ranges stay non-empty while n_items >= world."""
    b = balanced_bounds(np.asarray(item_ids, np.int32), n_items, world).astype(np.int64)
    if n_items >= world:                    # no empty range (a degenerate rating skew)
        for c in range(1, world):
            b[c] = min(max(b[c], b[c - 1] + 1), n_items - (world - c))
    return b


def rotation_offset(epoch: int, world: int) -> int:
    """Item range of rank 0 in sub-epoch 0 of epoch ``epoch``: one step back
    per epoch, so every rank opens an epoch on the range it closed the last
    one with (no transfer at the epoch boundary; the other ranges held
    locally are stale until they come round the ring)."""
    return (-int(epoch)) % world


def rotation_range(rank: int, off: int, s: int, world: int) -> int:
    """Item range rank ``rank`` sweeps in sub-epoch ``s``."""
    return (rank + off + s) % world


def rotation_draws(draw: int, rank: int, c: int, nb):
    """Stratum order and step rotation of rank ``rank``'s sub-block with item
    range ``c`` in the epoch with ``draw`` (reproducible per sub-block);
    ``nb`` = the strata plan (or its B)."""
    rs = np.random.RandomState([int(draw) & 0x7FFFFFFF, rank, c])
    return stratum_order(rs, nb), int(rs.randint(0, 2**31 - 1))


class RotationExchange:
    """The ring hand-off of item ranges (``exchange="rotate"``).

    The engine's Q / b_i hold the full item side; at any moment only the
    range this rank holds is current there.  ``pass_range`` sends range
    ``c_send`` to rank - 1 and receives ``c_recv`` from rank + 1 (batched
    point-to-point: one RCCL group, two xGMI transfers per rank);
    ``gather`` all-gathers every rank's final range (into the live replica, or
    into ``into``).  With gloo and device tensors (one-GPU rehearsal) the
    transfers are staged through host memory.

    ``overlap``: the end-of-epoch all-gather and the training-RMSE pass leave
    the critical path (``snapshot_sse``): the rank's P / b_u and its final
    range are copied on the launch stream (two copies of a few MB), then, on
    a side stream, the all-gather fills a snapshot replica and mf_sse_capped
    computes the epoch's SSE from the snapshots with at most ``sse_blocks``
    workgroups, beside the next epoch's sub-epochs (which use B workgroups,
    one per CU, of the chip's CUs).  The live replica is then gathered only
    when the caller needs it whole (``gather`` after the last epoch)."""

    def __init__(self, engine: SGDEngine, ilo: np.ndarray, group=None, overlap: bool = False):
        self.e, self.group = engine, group
        self.ilo = np.asarray(ilo, np.int64)
        self.world, self.rank = world_info(group)
        if len(self.ilo) != self.world + 1:
            raise ValueError("item ranges must be one per rank")
        dev = getattr(engine, "dev", torch.device("cpu"))
        self.stage = (self.world > 1 and dist.get_backend(group) == "gloo"
                      and torch.device(dev).type == "cuda")
        self.rows = int(np.diff(self.ilo).max()) if self.world else 0
        self._gbuf = None
        self.overlap = bool(overlap) and torch.device(dev).type == "cuda"
        self._ov = None
        self.sse_events = []            # (start, end) on the side stream per snapshot_sse

    def _range(self, c: int, Q=None, bi=None):
        lo, hi = int(self.ilo[c]), int(self.ilo[c + 1])
        Q = self.e.Q if Q is None else Q
        bi = self.e.bi if bi is None else bi
        return Q[lo:hi], bi[lo:hi]

    def pass_range(self, c_send: int, c_recv: int) -> None:
        """Send range c_send to rank - 1, receive range c_recv from rank + 1."""
        if self.world == 1:
            return
        to, frm = (self.rank - 1) % self.world, (self.rank + 1) % self.world
        qs, bs = self._range(c_send)
        qr, br = self._range(c_recv)
        if self.stage:
            snd = [qs.cpu(), bs.cpu()]
            rcv = [torch.empty_like(qr, device="cpu"), torch.empty_like(br, device="cpu")]
        else:
            snd, rcv = [qs, bs], [qr, br]
        ops = ([dist.P2POp(dist.isend, t, to, self.group) for t in snd]
               + [dist.P2POp(dist.irecv, t, frm, self.group) for t in rcv])
        for w in dist.batch_isend_irecv(ops):
            w.wait()
        if self.stage:
            qr.copy_(rcv[0])
            br.copy_(rcv[1])

    def _buffers(self):
        e, k, m = self.e, self.e.k, self.rows
        dev = torch.device("cpu") if self.stage else e.Q.device
        if self._gbuf is None:
            self._gbuf = (torch.zeros(m * (k + 1), dtype=e.Q.dtype, device=dev),
                          torch.empty(self.world * m * (k + 1), dtype=e.Q.dtype, device=dev))
        return self._gbuf

    def _pack(self, c: int) -> None:
        """This rank's range c into the gather's send buffer (current stream)."""
        mine, _ = self._buffers()
        k, m = self.e.k, self.rows
        q, b = self._range(c)
        n = q.shape[0]
        mine[: n * k].copy_(q.reshape(-1))
        mine[m * k: m * k + n].copy_(b)

    def _all_gather_unpack(self, c_final: list, Q, bi, skip_own: bool) -> None:
        mine, out = self._buffers()
        k, m = self.e.k, self.rows
        if dist.get_backend(self.group) == "gloo":
            dist.all_gather(list(out.view(self.world, -1).unbind(0)), mine, group=self.group)
        else:
            dist.all_gather_into_tensor(out, mine, group=self.group)
        parts = out.view(self.world, m * (k + 1))
        for r in range(self.world):
            if r == self.rank and skip_own:
                continue
            q, b = self._range(c_final[r], Q, bi)
            n = q.shape[0]
            q.copy_(parts[r, : n * k].view(n, k))
            b.copy_(parts[r, m * k: m * k + n])

    def gather(self, c_final: list) -> None:
        """Every rank's final range (rank r holds c_final[r]) into every rank's
        live replica."""
        if self.world == 1:
            self._whole = "live"
            return
        self.join()
        self._pack(c_final[self.rank])
        self._all_gather_unpack(c_final, None, None, skip_own=True)
        self._whole = "live"

    def snapshot_sse(self, c_final: list, slot: int, sse_blocks: int, timing: bool = False):
        """Epoch end in overlap mode (class docstring): snapshots on the
        launch stream, all-gather + RMSE pass on the side stream."""
        e = self.e
        main = torch.cuda.current_stream(e.dev)
        ov = self._ov
        if ov is None:
            ov = self._ov = dict(side=torch.cuda.Stream(e.dev), done=None,
                                 P=torch.empty_like(e.P), bu=torch.empty_like(e.bu),
                                 Q=torch.empty_like(e.Q), bi=torch.empty_like(e.bi),
                                 ws=torch.empty_like(e.ws))
        if ov["done"] is not None:
            main.wait_event(ov["done"])          # the last pass has read the snapshots
        ov["P"].copy_(e.P)
        ov["bu"].copy_(e.bu)
        own_q, own_b = self._range(c_final[self.rank])
        snap_q, snap_b = self._range(c_final[self.rank], ov["Q"], ov["bi"])
        snap_q.copy_(own_q)
        snap_b.copy_(own_b)
        if self.world > 1:
            self._pack(c_final[self.rank])
        ready = torch.cuda.Event()
        ready.record(main)
        side = ov["side"]
        with torch.cuda.stream(side):
            side.wait_event(ready)
            if timing:
                ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                ev[0].record(side)
            if self.world > 1:
                self._all_gather_unpack(c_final, ov["Q"], ov["bi"], skip_own=True)
            gathered = torch.cuda.Event()
            gathered.record(side)
            e.sse_from(slot, ov["P"], ov["Q"], ov["bu"], ov["bi"], ov["ws"], side, sse_blocks)
            if timing:
                ev[1].record(side)
                self.sse_events.append(ev)
        done = torch.cuda.Event()
        done.record(side)
        ov["done"] = done
        ov["gathered"] = gathered
        self._whole = "snapshot"

    def whole_replica(self):
        """(Q, b_i, event or None): the whole current replica after the last
        epoch -- the live one if the epoch ended with ``gather``, else the
        snapshot of ``snapshot_sse`` with the event after its all-gather on
        the side stream (wait on it before reading; the RMSE pass reads the
        same snapshot meanwhile, read-only)."""
        if getattr(self, "_whole", None) == "snapshot":
            return self._ov["Q"], self._ov["bi"], self._ov["gathered"]
        return self.e.Q, self.e.bi, None

    def join(self) -> None:
        """Make the launch stream wait for the side stream's last pass."""
        if self._ov is not None and self._ov["done"] is not None:
            torch.cuda.current_stream(self.e.dev).wait_event(self._ov["done"])


def sse_blocks_beside(engine: SGDEngine, n_blocks: int) -> int:
    """Workgroups the overlapped RMSE pass may use beside a persistent strata
    launch of ``n_blocks`` workgroups (one per CU): the CUs left over, less a
    margin (at least 8: one per item slice)."""
    cus = engine._cus()
    return max(8, cus - n_blocks - 8)


def rotation_epoch(engine: SGDEngine, rot: RotationExchange, draw: int, lr: float, reg: float,
                   update_user: bool = True, update_item: bool = True, events=None,
                   persistent: Optional[bool] = None, launches: Optional[list] = None,
                   epoch: int = 0, sse_slot: Optional[int] = None,
                   sse_timing: bool = False) -> None:
    """One epoch of the rotation schedule on this rank (module docstring):
    N sub-epochs (engine.epoch_phase on the range held; offset
    rotation_offset(epoch)), N - 1 ring hand-offs, then either the all-gather
    into the live replica or, with ``rot.overlap`` and ``sse_slot``, the
    snapshot + side-stream gather and RMSE pass (RotationExchange.snapshot_sse;
    the caller then gathers the live replica once at the end).  ``events``: a
    list that receives (kind, start, end) timing events ("sgd" / "pass" /
    "gather") recorded on the launch stream.  ``launches``: a list that
    receives each sub-epoch's kernel launch count (1 = persistent;
    synchronises after every sub-epoch)."""
    world, rank = rot.world, rot.rank
    nb = engine.strata
    off = rotation_offset(epoch, world)

    def mark(kind, fn):
        if events is None:
            return fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        out = fn()
        e1.record()
        events.append((kind, e0, e1))
        return out

    for s in range(world):
        c = rotation_range(rank, off, s, world)
        seq, seed = rotation_draws(draw, rank, c, nb)
        out = mark("sgd", lambda: engine.epoch_phase(c, seq, seed, lr, reg, update_user,
                                                     update_item, persistent=persistent,
                                                     timing=launches is not None))
        if launches is not None:
            launches.append(int(out[1]))
        if s + 1 < world:
            mark("pass", lambda: rot.pass_range(c, rotation_range(rank, off, s + 1, world)))
    c_final = [rotation_range(r, off, world - 1, world) for r in range(world)]
    if rot.overlap and sse_slot is not None:
        mark("gather", lambda: rot.snapshot_sse(c_final, sse_slot,
                                                sse_blocks_beside(engine, nb.B), sse_timing))
    else:
        mark("gather", lambda: rot.gather(c_final))


def rotation_final_ranges(epoch: int, world: int) -> list:
    """The range each rank holds at the end of epoch ``epoch``."""
    off = rotation_offset(epoch, world)
    return [rotation_range(r, off, world - 1, world) for r in range(world)]


# ------------------------------------------------- relabelled item ranges
# The rotation over K item relabellings (the frontier's
# "rotrel8"): which items share a range -- and so
# meet a user shard's ratings in the same burst -- changes from epoch to
# epoch.  Relabelling q renames canonical item x to perms[q][x]; its item
# ranges are contiguous ranges of the NEW ids, balanced over all ratings
# (identical on every rank), and each rank sweeps them with an engine over
# its ratings in the new ids.  Measured on one GPU (8 virtual ranks, 8 draws,
# 20 epochs at C3, profiles/r05/frontier_c4_rotation_family_r05o.json): RMSE
# gap to the reference order +1.69e-3 -> +1.40e-3 at the same sweep time.
ROTATE_RELABEL = 8
RELABEL_SEED = 5150           # relabelling q >= 1: RandomState(RELABEL_SEED + q)


def item_relabellings(n_items: int, k: int) -> list:
    """K item relabellings: None (the identity) and K - 1 permutations,
    perms[q][x] = new id of canonical item x.  Drawn from their own
    RandomStates, never the global one (the fit's draws stay one integer per
    epoch)."""
    return [None] + [np.random.RandomState(RELABEL_SEED + q).permutation(n_items)
                     for q in range(1, int(k))]


def relabel_pick(draw: int, k: int) -> int:
    """The relabelling of the epoch with ``draw`` (same on every rank)."""
    if k <= 1:
        return 0
    return int(np.random.RandomState([int(draw) & 0x7FFFFFFF, 77]).randint(0, k))


def relabel_ranges(item_ids: np.ndarray, n_items: int, world: int, perm) -> np.ndarray:
    """item_ranges over the relabelled ids of ALL ratings (``item_ids``:
    canonical ids of every rating of the job)."""
    ids = item_ids if perm is None else perm[item_ids].astype(np.int32)
    return item_ranges(ids, n_items, world)


def _moves(perms: list, dev):
    """Per relabelling: (new id of canonical x, canonical id of new y) as
    device index tensors (None for the identity)."""
    out = []
    for p in perms:
        if p is None:
            out.append((None, None))
            continue
        inv = np.empty_like(p)
        inv[p] = np.arange(len(p))
        out.append((torch.as_tensor(p, dtype=torch.int64, device=dev),
                    torch.as_tensor(inv, dtype=torch.int64, device=dev)))
    return out


def relabel_rows(src: torch.Tensor, dst: torch.Tensor, moves, p: int, q: int) -> None:
    """dst (rows in labelling q) = src (rows in labelling p), exact copies:
    dst[y] = src[perm_p[inv_q[y]]]."""
    fwd_p, _ = moves[p]
    _, inv_q = moves[q]
    if inv_q is None and fwd_p is None:
        dst.copy_(src)
        return
    if inv_q is None:
        idx = fwd_p
    elif fwd_p is None:
        idx = inv_q
    else:
        idx = fwd_p.index_select(0, inv_q)
    torch.index_select(src, 0, idx.to(src.device), out=dst)


class RotationSet:
    """This rank's rotation over K item relabellings.

    ``engine`` (canonical item ids) is relabelling 0; relabelling q >= 1 gets
    an engine over the same ratings with item ids perms[q][i], its own plan
    over its own item ranges and its own item replica, sharing P / b_u (and
    the SSE buffer) with ``engine``.  Each epoch runs in the relabelling its
    draw picks (relabel_pick): when that differs from the last epoch's, the
    whole current replica -- the snapshot the overlapped RMSE pass all-gathered,
    or the live one -- is copied into the new labelling first (one device
    index copy; the main stream waits only for that all-gather, not for the
    RMSE pass).  ``finish`` gathers the last epoch's ranges and leaves the
    canonical replica in ``engine``'s Q / b_i.  ``relabel=1`` is the plain
    rotation (bit for bit the previous product path)."""

    def __init__(self, engine, item_ids: np.ndarray, world: int, relabel: int = ROTATE_RELABEL,
                 group=None, overlap: bool = False, prepare: Optional[dict] = None,
                 make_exchange=None, make_engine=None):
        self.main = engine
        self.world = int(world)
        self.K = max(1, int(relabel))
        n_items = engine.n_items
        prepare = dict(prepare or {})
        self.perms = item_relabellings(n_items, self.K)
        self.ilo = [relabel_ranges(item_ids, n_items, self.world, p) for p in self.perms]
        mk_ex = make_exchange or (lambda e, ilo: RotationExchange(e, ilo, group, overlap=overlap))
        self.engines = [engine]
        if engine.strata is None:
            engine.prepare_strata(item_bounds=self.ilo[0], **prepare)
        make = make_engine or SGDEngine
        for q in range(1, self.K):
            p = self.perms[q]
            e = make(engine.u_host, p[engine.i_host].astype(np.int32), engine.r_host,
                     engine.n_users, n_items, engine.k, getattr(engine, "kernel", "linear"),
                     getattr(engine, "dtype", "float64"), getattr(engine, "dev", None),
                     gamma=getattr(engine, "gamma", 0.0),
                     min_rating=getattr(engine, "min_rating", 0.0),
                     max_rating=getattr(engine, "max_rating", 5.0),
                     global_mean=engine.global_mean)
            e.prepare_strata(item_bounds=self.ilo[q], **prepare)
            self.engines.append(e)
        self.rots = [mk_ex(e, ilo) for e, ilo in zip(self.engines, self.ilo)]
        self.overlap = self.rots[0].overlap
        self.moves = _moves(self.perms, getattr(engine, "dev", torch.device("cpu")))
        self.cur = 0                    # labelling the replica is in
        self.fresh = True               # the current labelling's live replica is whole
        self.B = engine.strata.B
        self.sse_events = []            # (start, end) of each timed side-stream RMSE pass

    # ---- parameters
    def bind(self) -> None:
        """Point every relabelled engine at the main engine's P / b_u and SSE
        buffer, give it an item replica of its own, and start from the main
        engine's (canonical, whole) replica."""
        m = self.main
        for e in self.engines[1:]:
            e.P, e.bu = m.P, m.bu
            if e.Q is None or e.Q.shape != m.Q.shape or e.Q.dtype != m.Q.dtype:
                e.Q, e.bi = torch.empty_like(m.Q), torch.empty_like(m.bi)
            e.sse_buf = m.sse_buf
        self.cur, self.fresh = 0, True

    def ensure_sse_slots(self, n: int) -> None:
        self.main._ensure_sse_slots(n)
        for e in self.engines[1:]:
            e.sse_buf = self.main.sse_buf

    def _to(self, q: int, timed=None) -> None:
        """Move the whole current replica into labelling q."""
        p = self.cur
        if q == p:
            return
        if self.fresh:
            srcQ, srcb, ev = self.engines[p].Q, self.engines[p].bi, None
        else:
            srcQ, srcb, ev = self.rots[p].whole_replica()
        dst = self.engines[q]
        dev = getattr(self.main, "dev", torch.device("cpu"))
        if ev is not None:
            torch.cuda.current_stream(dev).wait_event(ev)
        relabel_rows(srcQ, dst.Q, self.moves, p, q)
        relabel_rows(srcb, dst.bi, self.moves, p, q)
        self.cur, self.fresh = q, True

    # ---- epochs
    def epoch(self, draw: int, lr: float, reg: float, update_user: bool = True,
              update_item: bool = True, events=None, persistent: Optional[bool] = None,
              launches: Optional[list] = None, epoch: int = 0, sse_slot: Optional[int] = None,
              sse_timing: bool = False) -> int:
        """One rotation epoch in the relabelling ``draw`` picks; returns it."""
        q = relabel_pick(draw, self.K)
        if q != self.cur:
            if events is None:
                self._to(q)
            else:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                self._to(q)
                e1.record()
                events.append(("relabel", e0, e1))
        rot = self.rots[q]
        rotation_epoch(self.engines[q], rot, draw, lr, reg, update_user, update_item,
                       events=events, persistent=persistent, launches=launches, epoch=epoch,
                       sse_slot=sse_slot, sse_timing=sse_timing)
        # rotation_epoch ends with rot.gather (live replica whole) or with the
        # snapshot form (live replica current on this rank's range only)
        self.fresh = not (rot.overlap and sse_slot is not None)
        if sse_timing and rot.overlap and sse_slot is not None and rot.sse_events:
            self.sse_events.append(rot.sse_events[-1])
        return q

    def finish(self, last_epoch: int) -> None:
        """The whole replica live on every rank, in canonical ids (main engine)."""
        q = self.cur
        self.rots[q].gather(rotation_final_ranges(last_epoch, self.world))
        self.fresh = True
        self._to(0)
        self.join()

    def join(self) -> None:
        for rot in self.rots:
            rot.join()

    def failed(self) -> bool:
        return any(e.strata is not None and e.strata_failed() for e in self.engines)

    def clear_strata_error(self) -> None:
        for e in self.engines:
            e.clear_strata_error()

    def reset(self) -> None:
        """After restoring the main engine's (canonical) parameters."""
        self.join()
        self.cur, self.fresh = 0, True


class RotationReplay:
    """The N-rank rotation schedule on ONE GPU (rehearsal and check).

    One engine per virtual rank -- the same user shard, item ranges and plans
    a real rank builds -- all pointing at one shared [Q, b_i]; sub-epoch s runs
    every rank's sub-block (r, (r + off + s) mod N) one after another.  The
    sub-blocks of a sub-epoch are disjoint in users and items, so this is bit
    for bit what N GPUs compute (the kernel's arithmetic depends only on the
    plan, the draws and the values), and each rank's sub-epoch time is
    measured alone.  With ``relabel`` K > 1 (the product default,
    ROTATE_RELABEL) each epoch runs in the item relabelling its draw picks,
    as RotationSet does on every rank: one engine set per relabelling, built
    when first drawn, the shared replica copied into the drawn labelling.
    ``serial_order`` lists the epoch's sequential order for the oracle."""

    def __init__(self, u, i, r, n_users: int, n_items: int, world: int, n_factors: int,
                 kernel: str, dtype: str, device, gamma: float = 0.0, min_rating: float = 0.0,
                 max_rating: float = 5.0, global_mean: float = 0.0,
                 n_blocks: Optional[int] = None, waves: Optional[int] = None, engine_cls=None,
                 classes: Optional[int] = None, relabel: int = ROTATE_RELABEL):
        self._make = SGDEngine if engine_cls is None else engine_cls
        self.world = world
        self.bounds = shard_users(u, n_users, world)
        self.n_items, self.n = n_items, len(u)
        self._data = (u, i, r, n_factors, kernel, dtype, device,
                      dict(gamma=gamma, min_rating=min_rating, max_rating=max_rating,
                           global_mean=global_mean))
        self._prep = dict(n_blocks=n_blocks, classes=classes)
        if waves is not None:
            self._prep["waves"] = waves
        self.K = max(1, int(relabel))
        self.perms = item_relabellings(n_items, self.K)
        self.gidx = []
        for rank in range(world):
            lo, hi = int(self.bounds[rank]), int(self.bounds[rank + 1])
            self.gidx.append(np.flatnonzero((u >= lo) & (u < hi)))
        self.sets = [None] * self.K
        self.ilo = relabel_ranges(i, n_items, world, None)
        self.engines = self._set(0)
        self.moves = None
        self.cur = 0
        # one B for every rank (each rank's plans draw their strata from it)
        self.B = [e.strata.B for e in self.engines]

    def _set(self, q: int) -> list:
        """The engines of relabelling q (built once, when first needed)."""
        if self.sets[q] is not None:
            return self.sets[q]
        u, i, r, k, kernel, dtype, device, hyp = self._data
        p = self.perms[q]
        ilo = relabel_ranges(i, self.n_items, self.world, p)
        engs = []
        for rank in range(self.world):
            lo, hi = int(self.bounds[rank]), int(self.bounds[rank + 1])
            m = self.gidx[rank]
            ii = i[m] if p is None else p[i[m]].astype(np.int32)
            e = self._make(u[m] - lo, ii, r[m], hi - lo, self.n_items, k, kernel, dtype, device,
                           **hyp)
            e.prepare_strata(item_bounds=ilo, **self._prep)
            engs.append(e)
        if q > 0:                       # P / b_u and the item replica of set 0's shapes
            base = self.sets[0]
            Q = torch.empty_like(base[0].Q) if base[0].Q is not None else None
            bi = torch.empty_like(base[0].bi) if base[0].bi is not None else None
            for e, b in zip(engs, base):
                e.P, e.bu = b.P, b.bu
                e.Q, e.bi = Q, bi
        self.sets[q] = engs
        return engs

    def load(self, P0, Q0, bu0, bi0) -> None:
        e0 = self.sets[0][0]
        e0.load_params(Q=Q0, bi=bi0)
        for rank, e in enumerate(self.sets[0]):
            lo, hi = int(self.bounds[rank]), int(self.bounds[rank + 1])
            e.load_params(P=P0[lo:hi], bu=bu0[lo:hi])
            e.Q, e.bi = e0.Q, e0.bi
        for q in range(1, self.K):      # relabelled sets built before: re-point P / b_u
            if self.sets[q] is not None:
                for e, b in zip(self.sets[q], self.sets[0]):
                    e.P, e.bu = b.P, b.bu
        self.cur = 0

    def _to(self, q: int) -> None:
        if q == self.cur:
            return
        engs = self._set(q)
        src = self.sets[self.cur][0]
        if engs[0].Q is None:            # built before load(): its replica now
            Q, bi = torch.empty_like(src.Q), torch.empty_like(src.bi)
            for e in engs:
                e.Q, e.bi = Q, bi
        if self.moves is None:
            self.moves = _moves(self.perms, getattr(self.sets[0][0], "dev",
                                                    torch.device("cpu")))
        relabel_rows(src.Q, engs[0].Q, self.moves, self.cur, q)
        relabel_rows(src.bi, engs[0].bi, self.moves, self.cur, q)
        self.cur = q

    def epoch(self, draw: int, lr: float, reg: float, update_user=True, update_item=True,
              timing: bool = False, persistent: Optional[bool] = None, epoch: int = 0):
        """Rotation epoch ``epoch`` (its draw ``draw``); with ``timing`` the
        kernel ms of every (sub-epoch, rank) as a world x world array."""
        W = self.world
        self._to(relabel_pick(draw, self.K))
        engs = self.sets[self.cur]
        off = rotation_offset(epoch, W)
        ms = np.zeros((W, W))
        for s in range(W):
            for rank, e in enumerate(engs):
                c = rotation_range(rank, off, s, W)
                seq, seed = rotation_draws(draw, rank, c, e.strata)
                t = e.epoch_phase(c, seq, seed, lr, reg, update_user, update_item,
                                  timing=timing, persistent=persistent)
                if timing:
                    ms[s, rank] = t[0]
        return ms if timing else None

    def serial_order(self, draw: int, epoch: int = 0) -> np.ndarray:
        """Global rating indices in the order epoch ``epoch`` applies them."""
        W = self.world
        engs = self._set(relabel_pick(draw, self.K))
        off = rotation_offset(epoch, W)
        parts = []
        for s in range(W):
            for rank, e in enumerate(engs):
                c = rotation_range(rank, off, s, W)
                seq, seed = rotation_draws(draw, rank, c, e.strata)
                parts.append(self.gidx[rank][e.strata.phase_order(c, seq, seed)])
        return np.concatenate(parts).astype(np.int64)

    def sse(self, slot: int) -> float:
        tot = 0.0
        for e in self.sets[self.cur]:
            e.sse_async(slot)
            tot += float(e.sse_values(slot + 1)[slot])
        return tot

    def params(self):
        """(P, Q, b_u, b_i) float64 host arrays, users in global order, items
        in canonical ids."""
        self._to(0)
        engs = self.sets[0]
        P = np.concatenate([e.P.cpu().numpy().astype(np.float64) for e in engs])
        bu = np.concatenate([e.bu.cpu().numpy().astype(np.float64) for e in engs])
        e0 = engs[0]
        return (P, e0.Q.cpu().numpy().astype(np.float64), bu,
                e0.bi.cpu().numpy().astype(np.float64))


def epoch_draws(rs: np.random.RandomState, nb, strata: bool):
    """Stratum (colour) order and step rotation of one epoch (``nb``: the
    strata plan, or the colour count)."""
    seq = stratum_order(rs, nb) if strata else rs.permutation(nb).astype(np.int32)
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
        nb = engine.strata
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


def any_rank_failed(engine: SGDEngine, group=None) -> bool:
    """True on every rank if a persistent strata sweep gave up waiting on ANY
    rank since its error word was last cleared (synchronises; one MAX
    all-reduce, so all ranks take the same branch and none is left waiting in
    a collective)."""
    if isinstance(engine, RotationSet):
        bad = 1 if engine.failed() else 0
        engine = engine.main
    else:
        bad = 1 if (engine.strata is not None and engine.strata_failed()) else 0
    if not (dist.is_available() and dist.is_initialized()):
        return bool(bad)
    dev = (torch.device("cpu") if dist.get_backend(group) == "gloo"
           else getattr(engine, "dev", torch.device("cpu")))
    t = torch.tensor([bad], dtype=torch.int32, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return bool(int(t.item()))


def fit_sharded(u: np.ndarray, i: np.ndarray, r: np.ndarray, n_users: int, n_items: int,
                P0: np.ndarray, Q0: np.ndarray, bu0: np.ndarray, bi0: np.ndarray,
                n_epochs: int, kernel: str, n_factors: int, dtype: str, device, gamma: float,
                min_rating: float, max_rating: float, global_mean: float, lr: float,
                reg: float, schedule: str, verbose: int = 0, update_user: bool = True,
                update_item: bool = True, group=None, exchange: str = "rotate",
                relabel: int = ROTATE_RELABEL):
    """KernelMF.fit's epochs in process-group mode (every rank calls it with
    the same ratings, initial parameters and NumPy RNG state).

    Each epoch draws ONE integer from NumPy's global RandomState on every
    rank (the same value: same state).  ``exchange="rotate"`` (strata, item
    updates on): the rotation epoch (module docstring; the draw fixes the
    ranges' order and each sub-block's strata); otherwise the rank's stratum /
    colour order comes from (that integer, rank) and the item deltas are
    all-reduced (``"delta"``; also ``update_item=False``, which needs no
    exchange at all since the item side is frozen).

    No host synchronisation per epoch: the persistent sweeps' error words are
    sticky and checked on all ranks at once (any_rank_failed) where the host
    waits anyway -- the verbose RMSE print or the end; if any rank's sweep gave
    up waiting, every rank restores its start-of-fit snapshot and replays the
    epochs so far with the same draws as per-stratum launches (same result).

    Returns (P, Q, b_u, b_i, train_rmse, engine) with float64 host arrays,
    identical on every rank."""
    if schedule not in ("strata", "colored"):
        raise ValueError("distributed fit needs schedule='strata' or 'colored' "
                         "(the exact schedule is one sequential order)")
    if exchange not in EXCHANGES:
        raise ValueError(f"exchange must be one of {EXCHANGES}, got {exchange!r}")
    world, rank = world_info(group)
    bounds = shard_users(u, n_users, world)
    lu, li, lr_ = local_shard(u, i, r, bounds, rank)
    lo, hi = int(bounds[rank]), int(bounds[rank + 1])
    eng = SGDEngine(lu, li, lr_, hi - lo, n_items, n_factors, kernel, dtype, device,
                    gamma=gamma, min_rating=min_rating, max_rating=max_rating,
                    global_mean=global_mean)
    eng.load_params(P=P0[lo:hi], bu=bu0[lo:hi])
    strata = schedule == "strata"
    rotate = strata and exchange == "rotate" and update_item
    ex = rot = None
    if rotate:
        eng.load_params(Q=Q0, bi=bi0)
        # K item relabellings, one drawn per epoch (RotationSet); the RMSE
        # pass of epoch e beside epoch e+1's sub-epochs (side stream)
        rot = RotationSet(eng, i, world, relabel, group, overlap=True)
        rot.bind()
    else:
        ex = ReplicaExchange(eng, group)
        ex.bind(Q0, bi0)
        if strata:
            # delta-out epochs always run the engine's own plan: no
            # relabelled plans unless items are frozen (update_users runs
            # plain epochs, which do pick them)
            eng.prepare_strata(regroup=None if not update_item else 1)
            nb = eng.strata
        else:
            eng.prepare_colored()
            nb = len(eng.colored) - 1
    n_total = len(u)
    eng._ensure_sse_slots(n_epochs)       # no reallocation under a side-stream pass
    if rot is not None:
        rot.ensure_sse_slots(n_epochs)
    rmse = []
    draws = []
    persistent = None
    snap0 = None
    if strata and eng.strata_persistent:
        snap0 = (eng.snapshot_params(), None if ex is None else ex.flat.clone())

    def run_epoch(epoch, draw, persistent_):
        if rotate:
            rot.epoch(draw, lr, reg, update_user, update_item, persistent=persistent_,
                      epoch=epoch, sse_slot=epoch if rot.overlap else None)
            if rot.overlap:
                return                        # its SSE runs on the side stream
            rot.engines[rot.cur].sse_async(epoch)     # (its labelling's ratings)
            return
        else:
            seq, sd = epoch_draws(np.random.RandomState([draw, rank]), nb, strata)
            if strata:
                ex.strata_epoch(seq, sd, lr, reg, update_user, update_item,
                                persistent=persistent_, exchange=update_item)
            else:
                ex.begin_epoch()
                eng.epoch_colored(seq, lr, reg, update_user, update_item)
                ex.end_epoch()
        eng.sse_async(epoch)

    def replay(upto):
        nonlocal persistent
        warnings.warn(f"a persistent strata sweep could not complete within epochs 1-{upto} "
                      "on some rank (workgroups not co-resident); every rank replayed them "
                      "with the same draws as one launch per stratum", RuntimeWarning,
                      stacklevel=3)
        persistent = False
        if rot is not None:
            rot.join()
        eng.restore_params(snap0[0])
        if ex is not None:
            ex.flat.copy_(snap0[1])
        if rot is not None:
            rot.clear_strata_error()
            rot.reset()                       # the canonical replica is whole again
        else:
            eng.clear_strata_error()
        for ep in range(upto):
            run_epoch(ep, draws[ep], False)

    def check(upto):
        if snap0 is not None and persistent is None and any_rank_failed(
                eng if rot is None else rot, group):
            replay(upto)

    for epoch in range(n_epochs):
        draw = int(np.random.randint(0, 2**31 - 1))
        draws.append(draw)
        run_epoch(epoch, draw, persistent)
        if verbose == 1:
            check(epoch + 1)
            if rot is not None:
                rot.join()
            rm = global_rmse(eng, epoch + 1, n_total, group)[epoch]
            rmse.append(rm)
            if rank == 0:
                print("Epoch ", epoch + 1, "/", n_epochs, " -  train_rmse:", rm)
    check(n_epochs)
    if rot is not None:                   # the whole replica on every rank, all SSEs in
        rot.finish(n_epochs - 1)
    if verbose != 1:
        rmse = global_rmse(eng, n_epochs, n_total, group)
    elif persistent is False:           # a replay re-computed the printed epochs
        rmse = global_rmse(eng, n_epochs, n_total, group)
    P = _gather_rows(eng.P, bounds, group)
    bu = _gather_rows(eng.bu.reshape(-1, 1), bounds, group).reshape(-1)
    Q = eng.Q.cpu().numpy().astype(np.float64)
    bi = eng.bi.cpu().numpy().astype(np.float64)
    return P, Q, bu, bi, rmse, eng

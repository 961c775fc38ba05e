"""Device-side training state: ratings and parameters resident in HBM.

This is the layer the reference implements as numba functions
(``_sgd`` / ``_calculate_rmse`` / ``_predict``,
kernel_matrix_factorization.py:240-541, and their bias-only twins in
baseline_model.py:183-417).  Here the ratings (SoA: int32 user, int32 item,
dtype rating) and the parameters (P, Q, b_u, b_i) live in torch-ROCm tensors
on one GPU and every sweep is a call into libmf_hip.so.

Two epoch schedules:

``exact``    the reference's visit order.  The caller draws the epoch's
             permutation exactly as the reference does (``np.random.shuffle``
             on the rating rows, kernel_matrix_factorization.py:371); the
             host scheduler cuts it into dependency levels and the GPU applies
             level after level -- bit-for-bit the sequential sweep, up to the
             summation order of the k-long dot products.
``colored``  throughput.  Ratings are edge-coloured once per fit (every
             colour is a matching: no shared user or item), stored colour-major
             and item-sorted in HBM; each epoch applies the colours in a fresh
             random order, i.e. a different valid sequential order per epoch.
"""

from __future__ import annotations

import ctypes
from concurrent.futures import ThreadPoolExecutor
import math
import os
import sys
import warnings
from typing import Optional, Sequence, Tuple

import numpy as np
import torch

from . import _lib, _prep

_VOID = ctypes.c_void_p

DTYPES = {
    "float32": (torch.float32, np.float32, _lib.MF_F32),
    "float64": (torch.float64, np.float64, _lib.MF_F64),
}


def canonical_dtype(dtype) -> str:
    name = np.dtype(dtype).name
    if name not in DTYPES:
        raise ValueError(f"dtype must be float32 or float64, got {dtype!r}")
    return name


def resolve_device(device=None) -> torch.device:
    """The GPU the engine runs on.  There is no CPU path."""
    if device is None:
        if not torch.cuda.is_available():
            raise _lib.MFLibraryError(
                "no HIP device visible: matrix_factorization trains on an "
                "AMD Instinct GPU (gfx950) through libmf_hip.so")
        return torch.device("cuda", torch.cuda.current_device())
    dev = torch.device(device)
    if dev.type != "cuda":
        raise ValueError(f"device must be a HIP ('cuda') device, got {device!r}")
    if dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    return dev


_WARMED = set()


def _warm_device(dev: torch.device) -> None:
    """mf_warmup once per device and process: the runtime loads the library's
    code object at the first launch of any of its kernels -- done here, while
    an engine is built (fit() builds it on a worker thread beside the
    initial draws), instead of inside the first training epoch."""
    if dev.type != "cuda" or dev.index in _WARMED:
        return
    with torch.cuda.device(dev):
        # (no cooperative launch under rocprofv3: its interception crashes)
        _lib.call("mf_warmup", _lib.MF_FLAG_NO_COOP if _under_rocprofiler() else 0,
                  _VOID(torch.cuda.current_stream(dev).cuda_stream))
    _WARMED.add(dev.index)


def _tp(t: Optional[torch.Tensor]):
    if t is None or t.numel() == 0:
        return None
    return _VOID(t.data_ptr())


def _np(a: Optional[np.ndarray]):
    if a is None:
        return None
    return a.ctypes.data_as(_VOID)


# ------------------------------------------------------------ schedulers
def sched_levels(u: np.ndarray, i: np.ndarray, order: Optional[np.ndarray],
                 n_users: int, n_items: int, use_user: bool = True,
                 use_item: bool = True) -> Tuple[np.ndarray, np.ndarray]:
    """Exact-order batches: (rating indices grouped by level, level offsets)."""
    n = len(u)
    u = np.ascontiguousarray(u, np.int32)
    i = np.ascontiguousarray(i, np.int32)
    if order is not None:
        order = np.ascontiguousarray(order, np.int64)
    sched = np.empty(n, np.int32)
    offs = np.empty(n + 1, np.int64)
    nl = ctypes.c_int32(0)
    _lib.call("mf_sched_levels", _np(u), _np(i), n, _np(order), n_users,
              n_items, int(use_user), int(use_item), _np(sched), _np(offs),
              n + 1, ctypes.byref(nl))
    return sched, offs[: nl.value + 1].copy()


def sched_levels_chunked(u: np.ndarray, i: np.ndarray, order: np.ndarray,
                         n_users: int, n_items: int, use_user: bool = True,
                         use_item: bool = True, n_chunks: int = 0,
                         out: Optional[np.ndarray] = None) -> Tuple[np.ndarray, np.ndarray]:
    """Exact-order batches built on host threads (mf_sched_levels_chunked):
    the visit order cut into ``n_chunks`` chunks (0 = by size), each levelled
    alone and placed after the earlier chunks' levels -- the same sequential
    sweep as ``sched_levels`` (bit for bit), more levels.  ``order``: 32-bit
    rating indices.  ``out``: optional int32 buffer of n (e.g. pinned memory
    for an asynchronous upload) that receives the schedule."""
    n = len(u)
    u = np.ascontiguousarray(u, np.int32)
    i = np.ascontiguousarray(i, np.int32)
    order = np.ascontiguousarray(order, np.int32)
    if len(order) != n:
        raise ValueError("order and ratings differ in length")
    sched = np.empty(n, np.int32) if out is None else out
    if sched.dtype != np.int32 or len(sched) < n or not sched.flags.c_contiguous:
        raise ValueError("out must be a contiguous int32 array of n entries")
    # a chunk's depth is at most its length: n levels at most
    offs = np.empty(n + 1, np.int64)
    nl = ctypes.c_int32(0)
    _lib.call("mf_sched_levels_chunked", _np(u), _np(i), n, _np(order), n_users,
              n_items, int(use_user), int(use_item), int(n_chunks), _np(sched), _np(offs),
              len(offs), ctypes.byref(nl))
    return sched[:n], offs[: nl.value + 1].copy()


def sched_color(u: np.ndarray, i: np.ndarray, n_users: int,
                n_items: int) -> Tuple[np.ndarray, np.ndarray]:
    """Edge-colouring batches: (rating indices colour-major, colour offsets)."""
    n = len(u)
    u = np.ascontiguousarray(u, np.int32)
    i = np.ascontiguousarray(i, np.int32)
    if n == 0:
        return np.empty(0, np.int32), np.zeros(1, np.int64)
    cap = int(np.bincount(u, minlength=n_users).max()
              + np.bincount(i, minlength=n_items).max() + 1)
    sched = np.empty(n, np.int32)
    offs = np.empty(cap, np.int64)
    nc = ctypes.c_int32(0)
    _lib.call("mf_sched_color", _np(u), _np(i), n, n_users, n_items,
              _np(sched), _np(offs), cap, ctypes.byref(nc))
    return sched, offs[: nc.value + 1].copy()


def sched_slices(u: np.ndarray, i: np.ndarray, n_users: int, n_items: int,
                 n_slices: int = 8) -> Tuple[np.ndarray, np.ndarray]:
    """Evaluation order: rating indices grouped by item slice, then user."""
    n = len(u)
    u = np.ascontiguousarray(u, np.int32)
    i = np.ascontiguousarray(i, np.int32)
    sched = np.empty(n, np.int32)
    offs = np.empty(n_slices + 1, np.int64)
    _lib.call("mf_sched_slices", _np(u), _np(i), n, n_users, n_items, n_slices,
              _np(sched), _np(offs))
    return sched, offs


N_SLICES = 8          # one item slice per XCD (MI355X: 8 XCDs x 4 MiB L2)


def sched_tiles(u: np.ndarray, i: np.ndarray, n_users: int, n_items: int, n_chunks: int,
                n_slices: int) -> Tuple[np.ndarray, np.ndarray]:
    """Evaluation order in tiles (mf_sched_tiles): user chunk x item slice,
    users ascending inside a tile; (1, S) is sched_slices(S)."""
    n = len(u)
    u = np.ascontiguousarray(u, np.int32)
    i = np.ascontiguousarray(i, np.int32)
    sched = np.empty(n, np.int32)
    offs = np.empty(n_chunks * n_slices + 1, np.int64)
    _lib.call("mf_sched_tiles", _np(u), _np(i), n, n_users, n_items, n_chunks, n_slices,
              _np(sched), _np(offs))
    return sched, offs


# the training-RMSE pass's evaluation tiles (user chunks, item slices) per
# dtype; env MF_SSE_TILES="C,S" overrides (probes: tools/sse_tiles_probe.py)
EVAL_TILES = {"float32": (1, N_SLICES), "float64": (1, N_SLICES)}


def eval_tiles(dtype: str) -> Tuple[int, int]:
    env = os.environ.get("MF_SSE_TILES")
    if env:
        c, s_ = (int(x) for x in env.split(","))
        return c, s_
    return EVAL_TILES.get(dtype, (1, N_SLICES))


# ------------------------------------------------------------ strata plan
def strata_mix(seed: int, blk: int) -> int:
    """First colour of block ``blk`` (mod its colour count) in the epoch with
    ``seed`` -- the host mirror of mf_strata.hpp:strata_mix."""
    m = 0xFFFFFFFF
    x = (int(seed) ^ ((int(blk) * 0x9E3779B9) & m)) & m
    x ^= x >> 16
    x = (x * 0x85EBCA6B) & m
    x ^= x >> 13
    x = (x * 0xC2B2AE35) & m
    x ^= x >> 16
    return x


def balanced_bounds(ids: np.ndarray, m: int, n_blocks: int, by_count: bool = True,
                    cum: Optional[np.ndarray] = None) -> np.ndarray:
    """``n_blocks`` contiguous id ranges over [0, m): equal rating counts
    (``by_count``) or equal id counts.  ``cum``: the cumulative rating count
    per id, if already known (SGDEngine.degree_cum)."""
    if not by_count or len(ids) == 0:
        return (np.arange(n_blocks + 1, dtype=np.int64) * m // n_blocks).astype(np.int32)
    if cum is None:
        cum = np.cumsum(np.bincount(ids, minlength=m).astype(np.int64))
    targets = np.arange(1, n_blocks, dtype=np.int64) * cum[-1] // n_blocks
    cuts = np.searchsorted(cum, targets, side="left") + 1
    b = np.concatenate([[0], np.minimum(cuts, m), [m]]).astype(np.int64)
    return np.maximum.accumulate(b).astype(np.int32)


class StrataPlan:
    """Host + device form of a mf_strata_plan: C*B user ranges x B item
    ranges (C = ``classes`` user-range classes, 1 = the plain B x B plan),
    C*B strata of B blocks, each block a grid of ``n_steps`` x ``NS`` rating
    slots (``sched``: rating index per position, -1 = idle slot)."""

    narrow = False      # built for the narrow 4-wave kernels (MF_FLAG_NARROW)
    l2_handoff = False  # run with MF_FLAG_L2_HANDOFF (chosen by prepare_strata)

    def __init__(self, B, NS, ubnd, ibnd, bstep, sched, classes=1):
        self.B, self.NS = int(B), int(NS)
        self.classes = int(classes)
        self.ubnd, self.ibnd, self.bstep, self.sched = ubnd, ibnd, bstep, sched
        self.max_items = int(np.diff(ibnd).max()) if B else 0
        self.max_users = int(np.diff(ubnd).max()) if B else 0

    def to_device(self, u, i, r, dev) -> None:
        """Upload the bounds and the step offsets; lay the triples out in plan
        order (idle slots: user -1, item -1, rating 0).  u / i / r are the
        triples in original order, host arrays or tensors already on ``dev``
        (then the reordering happens on the device)."""
        to = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
        self.d_ubnd, self.d_ibnd, self.d_bstep = to(self.ubnd), to(self.ibnd), to(self.bstep)
        u, i, r = (x if isinstance(x, torch.Tensor) else torch.from_numpy(
            np.ascontiguousarray(x)).to(dev) for x in (u, i, r))
        sched = to(self.sched)
        valid = sched >= 0
        idx = torch.where(valid, sched, 0).long()
        del sched
        self.d_u = torch.where(valid, u.index_select(0, idx), -1).to(torch.int32)
        self.d_i = torch.where(valid, i.index_select(0, idx), -1).to(torch.int32)
        self.d_r = torch.where(valid, r.index_select(0, idx), 0).to(r.dtype)

    @property
    def n_positions(self) -> int:
        return len(self.sched)

    @property
    def n_strata(self) -> int:
        """Strata of one epoch (launches of the per-stratum form)."""
        return self.classes * self.B

    @property
    def n_ratings(self) -> int:
        """Ratings in the plan (positions that are not idle slots)."""
        if getattr(self, "_n_ratings", None) is None:
            self._n_ratings = int(np.count_nonzero(self.sched >= 0))
        return self._n_ratings

    @property
    def n_steps(self) -> np.ndarray:
        return np.diff(self.bstep)

    def stratum_sizes(self) -> np.ndarray:
        """Ratings per stratum (launch)."""
        cnt = np.concatenate([[0], np.cumsum(self.sched >= 0)])
        edges = self.bstep[:: self.B] * self.NS
        return np.diff(cnt[edges])

    # stratum order of the plan's epochs (stratum_order mode): "xcd" for
    # plans run with the L2 hand-off, None = the default (MF_STRATA_ORDER)
    order: Optional[str] = None

    def serial_order(self, seq, seed) -> np.ndarray:
        """Rating indices in the order one epoch (strata ``seq``, ``seed``)
        applies them: a sequential order the GPU result equals."""
        B, NS = self.B, self.NS
        out = []
        for s in seq:
            for w in range(B):
                blk = int(s) * B + w
                st0 = int(self.bstep[blk])
                nst = int(self.bstep[blk + 1]) - st0
                if nst <= 0:
                    continue
                rot = strata_mix(seed, blk) % nst
                steps = (rot + np.arange(nst)) % nst
                grid = self.sched[st0 * NS:(st0 + nst) * NS].reshape(nst, NS)[steps].ravel()
                out.append(grid[grid >= 0])
        return np.concatenate(out).astype(np.int64) if out else np.empty(0, np.int64)


class PhasedStrata:
    """Item phases of one strata epoch: the items are cut into P contiguous
    ranges, and phase p is a whole strata plan over the ratings of range p
    (item ids relative to its start), run as its own persistent launch on
    Q / b_i rows [ilo[p], ilo[p+1]).  For item matrices whose slabs would
    not fit the LDS of one workgroup per CU (C3 at FP64: 52 MB of rows,
    B = 403 > 256 CUs, i.e. one launch per stratum otherwise), P phases of
    B <= CUs keep the sweep persistent.  Every phase uses the same B, so an
    epoch's ``seq`` (a permutation of range(B)) and rotation seed apply to
    each phase; the sequential order is phase 0's, then phase 1's, ... --
    again a plain serial order of all the ratings (``serial_order``)."""

    def __init__(self, phases, idx, ilo):
        self.phases, self.idx = phases, idx
        self.ilo = np.asarray(ilo, np.int64)
        self.B, self.NS = phases[0].B, phases[0].NS
        self.classes = phases[0].classes
        self.narrow = phases[0].narrow
        self.max_items = max(pl.max_items for pl in phases)
        self.max_users = max(pl.max_users for pl in phases)

    @property
    def n_positions(self) -> int:
        return sum(pl.n_positions for pl in self.phases)

    @property
    def n_strata(self) -> int:
        return self.classes * self.B

    @property
    def n_steps(self) -> np.ndarray:
        return np.concatenate([pl.n_steps for pl in self.phases])

    def stratum_sizes(self) -> np.ndarray:
        """Ratings per stratum index, summed over the phases (stratum s of
        every phase runs when ``seq`` lists s)."""
        return np.sum([pl.stratum_sizes() for pl in self.phases], axis=0)

    def serial_order(self, seq, seed) -> np.ndarray:
        parts = [ix[pl.serial_order(seq, seed)] for pl, ix in zip(self.phases, self.idx)]
        return np.concatenate(parts).astype(np.int64) if parts else np.empty(0, np.int64)

    def phase_order(self, p: int, seq, seed) -> np.ndarray:
        """Rating indices (the engine's order) that phase ``p`` alone applies
        with strata ``seq`` and rotation ``seed`` -- one sub-epoch of the
        rotation schedule (distributed.rotation_epoch)."""
        return self.idx[p][self.phases[p].serial_order(seq, seed)].astype(np.int64)


def sched_strata(u: np.ndarray, i: np.ndarray, n_users: int, n_items: int, n_blocks: int,
                 ubnd: np.ndarray, ibnd: np.ndarray, n_slots: int, classes: int = 1):
    """mf_strata_plan_build_classes + fetch: (sched, block step offsets);
    ``ubnd`` has classes * n_blocks + 1 entries."""
    n = len(u)
    u = np.ascontiguousarray(u, np.int32)
    i = np.ascontiguousarray(i, np.int32)
    ubnd = np.ascontiguousarray(ubnd, np.int32)
    ibnd = np.ascontiguousarray(ibnd, np.int32)
    lib = _lib.load()
    handle = ctypes.c_void_p()
    _lib.call("mf_strata_plan_build_classes", _np(u), _np(i), n, n_users, n_items, n_blocks,
              int(classes), _np(ubnd), _np(ibnd), n_slots, ctypes.byref(handle))
    try:
        npos = int(lib.mf_strata_plan_positions(handle))
        sched = np.empty(max(npos, 1), np.int32)
        bstep = np.empty(int(classes) * n_blocks * n_blocks + 1, np.int64)
        _lib.call("mf_strata_plan_fetch", handle, _np(sched), _np(bstep))
    finally:
        lib.mf_strata_plan_free(handle)
    return sched[:npos], bstep


def sched_strata_pick(u: np.ndarray, i: np.ndarray, n_users: int, n_items: int, n_blocks: int,
                      ubnd: np.ndarray, ibnd: np.ndarray, shapes, classes: int = 1,
                      fill_stop: float = 0.0):
    """mf_strata_plan_build_pick + fetch: (sched, block step offsets, index
    of the picked (slots, waves) shape) -- the plan ``sched_strata`` builds
    with the slots of the shape of least steps * waves (the first outright
    when it fills ``fill_stop`` of its positions); the other shapes' step
    counts come without their colouring."""
    n = len(u)
    u = np.ascontiguousarray(u, np.int32)
    i = np.ascontiguousarray(i, np.int32)
    ubnd = np.ascontiguousarray(ubnd, np.int32)
    ibnd = np.ascontiguousarray(ibnd, np.int32)
    slots = np.ascontiguousarray([s for s, _ in shapes], np.int32)
    waves = np.ascontiguousarray([w for _, w in shapes], np.int32)
    lib = _lib.load()
    handle = ctypes.c_void_p()
    picked = ctypes.c_int32(-1)
    _lib.call("mf_strata_plan_build_pick", _np(u), _np(i), n, n_users, n_items, n_blocks,
              int(classes), _np(ubnd), _np(ibnd), _np(slots), _np(waves), len(shapes),
              float(fill_stop), ctypes.byref(picked), ctypes.byref(handle))
    try:
        npos = int(lib.mf_strata_plan_positions(handle))
        sched = np.empty(max(npos, 1), np.int32)
        bstep = np.empty(int(classes) * n_blocks * n_blocks + 1, np.int64)
        _lib.call("mf_strata_plan_fetch", handle, _np(sched), _np(bstep))
    finally:
        lib.mf_strata_plan_free(handle)
    return sched[:npos], bstep, int(picked.value)


def strata_slots(k: int, dcode: int, waves: int = 16) -> int:
    """Rating slots per step of the strata kernel with ``waves`` waves per
    workgroup (16, or 8 for FP32 rows of k <= 64); 0 if that kernel does not
    exist."""
    ns = int(_lib.load().mf_strata_slots_waves(k, dcode, waves))
    if ns <= 0:
        if waves == 16:
            _lib.check(1, "mf_strata_slots")
        return 0
    return ns


# ratings per B^2 of the default plan rule B = sqrt(n / STRATA_PER_B2): the
# single-GPU epoch (C3 caps at 256, C2 gives 69; DESIGN.md section 5 sweeps)
STRATA_PER_B2 = 1024.0
# the same for one rank's sub-block of the rotation schedule (n / N^2 ratings:
# fewer ratings per block pay, DESIGN.md section 6 sweeps)
ROTATE_PER_B2 = 1024.0


def choose_strata_blocks(u, i, n_users, n_items, k, dcode, max_blocks=None,
                         per_b2: float = STRATA_PER_B2, classes: int = 1, cums=(None, None)):
    """B and the user / item bounds: B ~ sqrt(n / per_b2) capped at 256 (one
    workgroup per CU), raised until the largest block's LDS image fits;
    ``classes`` * B user ranges (user-range classes)."""
    lib = _lib.load()
    n = len(u)
    B = int(min(256, max(1, np.sqrt(n / float(per_b2)))))
    if max_blocks is not None:
        B = min(B, int(max_blocks))
    limit = lib.mf_strata_lds_limit()
    while True:
        ub = balanced_bounds(u, n_users, classes * B, cum=cums[0])
        for by_count in (True, False):
            ib = balanced_bounds(i, n_items, B, by_count, cum=cums[1])
            need = lib.mf_strata_lds_bytes(int(np.diff(ib).max()), int(np.diff(ub).max()),
                                           k, dcode)
            if need <= limit:
                return B, ub, ib
        if B >= max(n_items, 1) and B >= max(n_users, 1):
            raise ValueError("strata schedule: a single item row does not fit in LDS")
        B = int(np.ceil(B * 1.25)) + 1


XCD_CLASSES = 8                  # gfx950: workgroups dealt round-robin over 8 XCDs
# MF_FLAG_L2_HANDOFF is chosen automatically (with the XCD-class stratum order
# and B a multiple of 8) when the user rows handed over inside an XCD can stay
# in its 4 MiB L2: P of at most this many bytes (the B/8 ranges an XCD holds
# at a time = P/8).  C2 (100K x 32 FP32 = 12.8 MB): SGD 0.943 -> 0.876 ms
# (B = 69 random order vs B = 72 XCD order + L2, same box);
# C3 / the N = 8 rotation (P 256 / 32 MB): no gain, not chosen.
L2_HANDOFF_P_BYTES = 24 << 20


class _HipBlock:
    """A physically contiguous device allocation, exposed to torch through
    __cuda_array_interface__ (torch keeps this object alive as long as the
    tensor's storage, and the block is freed with it).  The block is not
    torch's: it does not show in torch.cuda.memory_allocated() or the caching
    allocator's statistics."""

    _hip = None

    def __init__(self, shape, dtype, dev):
        if _HipBlock._hip is None:
            _HipBlock._hip = ctypes.CDLL("libamdhip64.so")
        hip = _HipBlock._hip
        self.ptr = ctypes.c_void_p()
        nbytes = int(np.prod(shape)) * torch.tensor([], dtype=dtype).element_size()
        with torch.cuda.device(dev):
            rc = hip.hipExtMallocWithFlags(ctypes.byref(self.ptr), ctypes.c_size_t(nbytes),
                                           ctypes.c_uint(0x4))       # hipDeviceMallocContiguous
        if rc != 0 or not self.ptr.value:
            self.ptr = None
            raise MemoryError(f"hipExtMallocWithFlags(contiguous, {nbytes}) failed: {rc}")
        typestr = {torch.float32: "<f4", torch.float64: "<f8"}[dtype]
        self.__cuda_array_interface__ = {"shape": tuple(shape), "typestr": typestr,
                                         "data": (self.ptr.value, False), "version": 2,
                                         "strides": None}

    def __del__(self):
        # at interpreter shutdown the HIP runtime (or ctypes) may already be
        # gone: the process exit releases the memory then
        if getattr(self, "ptr", None) is None or _HipBlock._hip is None or sys.is_finalizing():
            return
        try:
            _HipBlock._hip.hipFree(self.ptr)
        except Exception:            # noqa: BLE001 -- never raise from a finaliser
            pass
        self.ptr = None


def _contiguous_empty(shape, dtype, dev) -> Optional[torch.Tensor]:
    """A device tensor in physically contiguous memory, or None."""
    if dtype not in (torch.float32, torch.float64):
        return None
    try:
        blk = _HipBlock(shape, dtype, dev)
        t = torch.as_tensor(blk, device=dev)
    except (OSError, MemoryError, RuntimeError, TypeError, KeyError):
        return None
    if t.data_ptr() != blk.ptr.value:            # torch copied instead of wrapping
        return None
    t._mf_block = blk                            # torch's storage deleter holds it too
    return t


AUTO_CLASSES = 4
AUTO_CLASSES_MIN_DEGREE = 2.0


def auto_strata_classes(kernel: str, n: int, n_items: int, B: int) -> int:
    """The automatic user-range classes of a plan of B workgroups over n
    ratings (SGDEngine.auto_classes): AUTO_CLASSES for
    the linear kernel when an item meets at least AUTO_CLASSES_MIN_DEGREE
    ratings per user range of the one-class plan, else 1."""
    if kernel != "linear" or n == 0 or B < 1:
        return 1
    deg = n / float(max(n_items, 1) * B)
    return AUTO_CLASSES if deg >= AUTO_CLASSES_MIN_DEGREE else 1


def stratum_order(rs, nb, mode: Optional[str] = None, classes: Optional[int] = None) -> np.ndarray:
    """The stratum order of one epoch, drawn from ``rs`` (a RandomState or
    the ``np.random`` module).  ``nb``: B, or a strata plan (its B and its
    user-range classes C).

    random: a uniform permutation of the B strata.  With C > 1 user-range
            classes (C*B strata, stratum s of class s mod C): the classes in
            a random order, each class's B strata in a random order, dealt
            round-robin -- position t holds a stratum of class
            cls[t mod C], so a user range is used again only C positions
            later (the persistent kernel's slack).
    xcd:    the strata grouped by s mod 8, the classes in random order and each
            class's strata in random order (B a multiple of 8; else random).
            Stratum t's user range r comes from the workgroup w' = w + s_t -
            s_{t-1} (mod B); inside a class that difference is a multiple of 8,
            so the hand-off stays on one XCD (workgroups are dealt round-robin
            over the XCDs) and the rows come from its L2 -- every order is a
            sequential order, the choice changes which one.
    """
    if hasattr(nb, "B"):
        classes = nb.classes if classes is None else classes
        mode = mode or getattr(nb, "order", None)
        nb = nb.B
    classes = int(classes or 1)
    if classes > 1:
        cls = rs.permutation(classes)
        per = [rs.permutation(nb) for _ in range(classes)]
        t = np.arange(classes * nb)
        c = cls[t % classes]
        j = np.stack(per)[c, t // classes]
        return (c + classes * j).astype(np.int32)
    mode = mode or os.environ.get("MF_STRATA_ORDER", "random")
    if mode == "xcd" and nb % XCD_CLASSES == 0 and nb > XCD_CLASSES:
        cls = rs.permutation(XCD_CLASSES)
        return np.concatenate([rs.permutation(np.arange(c, nb, XCD_CLASSES))
                               for c in cls]).astype(np.int32)
    if mode not in ("random", "xcd"):
        raise ValueError(f"MF_STRATA_ORDER must be 'random' or 'xcd', got {mode!r}")
    return rs.permutation(nb).astype(np.int32)


def _under_rocprofiler() -> bool:
    """True when rocprofv3's tool library is preloaded into this process
    (`rocprofv3 ... -- python ...` puts librocprofiler-sdk-tool in
    LD_PRELOAD).  Profiled runs then launch the persistent strata kernel
    plainly -- the same kernel; the occupancy check stays the co-residency
    guard -- and bench.py labels its line "launch": "plain (profiler)".
    Why ("the r05n abort"): one profiled top-k bench
    exited 139 in its C exit handlers after its JSON line was out; nothing
    ties that fault to the cooperative launch, so this is caution, kept
    narrow: only the preload counts, not any ROCPROF* variable in the
    environment (MF_PROFILER_PLAIN=0 turns it off)."""
    if os.environ.get("MF_PROFILER_PLAIN") == "0":
        return False
    return "librocprofiler" in os.environ.get("LD_PRELOAD", "")


def launch_form_label() -> str:
    """How the persistent sweeps are launched in this process (bench.py's
    line carries it)."""
    if os.environ.get("MF_STRATA_COOP") == "0":
        return "plain (MF_STRATA_COOP=0)"
    return "plain (profiler)" if _under_rocprofiler() else "cooperative"


# the stream kernel's per-position step count is a 16-bit field
STREAM_MAX_STEPS = 0xFFFF


def max_block_steps(pl) -> int:
    """Largest number of steps of one block over every phase of a plan."""
    cached = getattr(pl, "_max_block_steps", None)
    if cached is not None:
        return cached
    subs = pl.phases if hasattr(pl, "phases") else [pl]
    m = 0
    for sub in subs:
        bs = np.asarray(sub.bstep)
        if bs.size > 1:
            m = max(m, int(np.diff(bs).max()))
    try:
        pl._max_block_steps = m
    except AttributeError:
        pass
    return m


def default_sgd_flags() -> int:
    env = os.environ.get("MF_SGD_FLAGS")
    if env is not None:
        return int(env, 0)
    # measured on MI355X (tools/sweep_sgd.py): streaming the user rows
    # non-temporally keeps Q's XCD-local slice in L2 (-6% SGD time)
    return _lib.MF_FLAG_XCD_SWIZZLE | _lib.MF_FLAG_NT_USER


# --------------------------------------------------------------- engine
class SGDEngine:
    """Ratings + factor-model parameters on one GPU.

    ``kernel`` is ``"linear" | "sigmoid" | "rbf"`` (KernelMF) or ``"bias"``
    (BaselineModel: no factor matrices).
    """

    def __init__(self, u: np.ndarray, i: np.ndarray, r: np.ndarray,
                 n_users: int, n_items: int, n_factors: int, kernel: str,
                 dtype="float64", device=None, gamma: float = 0.0,
                 min_rating: float = 0.0, max_rating: float = 5.0,
                 global_mean: float = 0.0, eval_order: bool = True,
                 check_ids: bool = True, device_triples=None):
        self.dev = resolve_device(device)
        _warm_device(self.dev)
        self.dtype = canonical_dtype(dtype)
        self.tdt, self.ndt, self.dcode = DTYPES[self.dtype]
        self.kernel = kernel
        self.bias_only = kernel == "bias"
        if not self.bias_only:
            if kernel not in _lib.KERNEL_CODES:
                raise ValueError(f"unknown kernel {kernel!r}")
            self.kcode = _lib.KERNEL_CODES[kernel]
            kmax = _lib.load().mf_max_factors()
            if not 0 <= n_factors <= kmax:
                raise ValueError(f"n_factors must be in [0, {kmax}], got {n_factors}")
        _lib.load()
        self.n = int(len(u))
        self.n_users, self.n_items = int(n_users), int(n_items)
        self.k = int(n_factors)
        self.gamma = float(gamma)
        self.min_rating, self.max_rating = float(min_rating), float(max_rating)
        self.global_mean = float(global_mean)
        self.u_host = np.ascontiguousarray(u, np.int32)
        self.i_host = np.ascontiguousarray(i, np.int32)
        self.r_host = np.ascontiguousarray(r, self.ndt)
        if check_ids and self.n and (self.u_host.min() < 0 or self.u_host.max() >= n_users
                       or self.i_host.min() < 0 or self.i_host.max() >= n_items):
            raise ValueError("rating ids outside [0, n_users) x [0, n_items)")
        if device_triples is not None:       # (u, i, r) already on the device
            self.u, self.i, self.r = device_triples
        else:
            self._upload_triples(self.u_host, self.i_host, self.r_host)
        if eval_order:
            self._build_eval()
        else:                        # a regrouping's engine: sweeps only, no RMSE pass
            self.eu, self.ei, self.er, self.eval_offs = self.u, self.i, self.r, None
        self.colored = None          # (offsets,) once prepare_colored() ran
        self.strata = None           # StrataPlan once prepare_strata() ran
        self._regroups = []          # relabelled plans: [(engine, user perm, item perm)]
        ws = max(_lib.load().mf_sse_workspace_bytes(self.n), 8)
        self.ws = torch.empty((ws + 7) // 8, dtype=torch.float64, device=self.dev)
        self.sse_buf = torch.zeros(16, dtype=torch.float64, device=self.dev)
        self.P = self.Q = self.bu = self.bi = None
        self._ov = None              # sse_overlap state (side stream, snapshot)

    # ---------------------------------------------------------- plumbing
    @property
    def stream(self):
        return _VOID(torch.cuda.current_stream(self.dev).cuda_stream)

    def _upload_triples(self, u, i, r):
        self.u = torch.from_numpy(u).to(self.dev)
        self.i = torch.from_numpy(i).to(self.dev)
        self.r = torch.from_numpy(r).to(self.dev)

    def _build_eval(self):
        """Second copy of the ratings in evaluation order (mf_sched_slices):
        the training-RMSE pass walks one item slice per XCD, user by user."""
        if self.bias_only or self.n == 0:
            self.eu, self.ei, self.er, self.eval_offs = self.u, self.i, self.r, None
            return
        n_chunks, n_slices = eval_tiles(self.dtype)
        if os.environ.get("MF_EVAL_ORDER") == "host":
            sched, offs = sched_tiles(self.u_host, self.i_host, self.n_users, self.n_items,
                                      n_chunks, n_slices)
            d_sched = torch.from_numpy(sched).to(self.dev).long()
        else:
            d_sched, offs = self._eval_order_device(n_chunks, n_slices)
        # reorder on the device from the uploaded triples
        self.eu = self.u.index_select(0, d_sched)
        self.ei = self.i.index_select(0, d_sched)
        self.er = self.r.index_select(0, d_sched)
        del d_sched
        self.eval_offs = offs

    def _eval_order_device(self, n_chunks: int, n_slices: int):
        """mf_sched_tiles' order computed on the GPU from the uploaded ids:
        a stable sort of key = (user chunk * n_slices + item slice) * n_users
        + user -- the host order exactly (tiles by a stable partition, users
        ascending, ties in rating order), in ~tens of ms instead of the
        host's ~0.4 s at C3 (fit()'s engine build)."""
        with torch.cuda.device(self.dev):
            u = self.u.long()
            i = self.i.long()
            n, nu = self.n, self.n_users
            sl = torch.div(i * n_slices, max(self.n_items, 1), rounding_mode="floor")
            if n_chunks > 1:
                deg = torch.bincount(u, minlength=nu)
                before = torch.cumsum(deg, 0) - deg            # ratings of users < x
                chunk_of = torch.clamp(torch.div(before * n_chunks, n, rounding_mode="floor"),
                                       max=n_chunks - 1)
                tile = chunk_of.index_select(0, u) * n_slices + sl
                del deg, before, chunk_of
            else:
                tile = sl
            key = tile * nu + u
            del sl, i, tile
            skey, order = torch.sort(key, stable=True)
            del key, u
            # tile t starts at the first key >= t * n_users (a search in the
            # sorted keys: a histogram of 10^8 ids into 8 bins is ~4 ms of
            # atomics on one address each)
            T = n_chunks * n_slices
            edges = torch.arange(T + 1, dtype=torch.int64, device=skey.device) * nu
            offs = torch.searchsorted(skey, edges).cpu().numpy().astype(np.int64)
            offs[-1] = n
            return order, offs

    def _dev(self, a, shape) -> torch.Tensor:
        if isinstance(a, torch.Tensor):
            t = a.to(device=self.dev, dtype=self.tdt)
        else:
            t = torch.from_numpy(np.ascontiguousarray(a, self.ndt)).to(self.dev)
        t = t.reshape(shape).contiguous()
        return t

    def _dev_rows(self, a, shape) -> torch.Tensor:
        """P in physically contiguous device memory (hipExtMallocWithFlags,
        hipDeviceMallocContiguous) from 16 MiB up.  Every sweep reads and
        writes the user rows at random; measured at C3 (tools/layout_probe.py,
        profiles/r03/layout_probe_contiguous_r03s31.json)
        the sweep takes 9.45 ms with P contiguous and 10.1 ms when P lands in
        memory the allocator assembled from smaller pieces (most likely the
        address-translation fragment size), which happened in every process
        but bench.py's.  Falls back to an ordinary allocation if the runtime
        refuses; MF_CONTIGUOUS_ROWS=0 turns it off."""
        t = self._dev(a, shape)
        nbytes = t.numel() * t.element_size()
        if (os.environ.get("MF_CONTIGUOUS_ROWS") == "0" or self.dev.type != "cuda"
                or nbytes < (16 << 20)):
            return t
        v = _contiguous_empty(shape, t.dtype, self.dev)
        if v is None:
            return t
        v.copy_(t)
        return v

    def load_params(self, P=None, Q=None, bu=None, bi=None) -> None:
        """Upload parameters (NumPy or torch); None keeps the current one."""
        if P is not None:
            self.P = self._dev_rows(P, (self.n_users, self.k))
        if Q is not None:
            self.Q = self._dev(Q, (self.n_items, self.k))
        if bu is not None:
            self.bu = self._dev(bu, (self.n_users,))
        if bi is not None:
            self.bi = self._dev(bi, (self.n_items,))

    def params_numpy(self):
        """(P, Q, b_u, b_i) as float64 host arrays (synchronises)."""
        out = []
        for t in (self.P, self.Q, self.bu, self.bi):
            out.append(None if t is None else t.cpu().numpy().astype(np.float64))
        return tuple(out)

    def _ensure_sse_slots(self, n):
        if self.sse_buf.numel() < n:
            buf = torch.zeros(max(n, 2 * self.sse_buf.numel()), dtype=torch.float64,
                              device=self.dev)
            buf[: self.sse_buf.numel()] = self.sse_buf
            self.sse_buf = buf

    # ---------------------------------------------------------- schedules
    def prepare_colored(self) -> int:
        """Colour the ratings once and store them colour-major in HBM.

        Returns the number of colours (batches per epoch)."""
        sched, offs = sched_color(self.u_host, self.i_host, self.n_users, self.n_items)
        self.u_host = self.u_host[sched]
        self.i_host = self.i_host[sched]
        self.r_host = self.r_host[sched]
        self._upload_triples(self.u_host, self.i_host, self.r_host)
        self.colored = offs
        return len(offs) - 1

    # user-range classes of the strata plans (StrataPlan.classes): "auto" /
    # None = by the plan (auto_classes), or 1..4; env MF_STRATA_CLASSES
    # overrides
    strata_classes = "auto"

    def _classes(self, classes) -> Optional[int]:
        """The classes asked for, or None for the automatic choice."""
        if classes is None and os.environ.get("MF_STRATA_CLASSES"):
            classes = os.environ["MF_STRATA_CLASSES"]
        if classes is None:
            classes = self.strata_classes
        if classes is None or classes == "auto":
            return None
        classes = int(classes)
        if not 1 <= classes <= _lib.MF_STRATA_MAX_CLASSES:
            raise ValueError(f"strata classes must be in [1, {_lib.MF_STRATA_MAX_CLASSES}], "
                             f"got {classes}")
        return classes

    def prepare_strata(self, n_blocks: Optional[int] = None,
                       waves: Optional[int] = None,
                       phases: Optional[int] = None,
                       item_bounds: Optional[np.ndarray] = None,
                       classes: Optional[int] = None,
                       regroup: Optional[int] = None) -> "StrataPlan":
        """Build the stratified plan once and store a padded copy of the
        ratings in plan order (block-major, step-major, slot-minor).  The
        host arrays keep the original rating order.

        ``waves``: workgroup size of the strata kernels, 16 or 8 (FP32,
        k <= 64), or 4: the 8-wave plan run by the narrow 4-wave kernels
        (MF_FLAG_NARROW; FP32, k a multiple of 4 up to 32).  None = by the plan: when the 16-wave plan fills fewer
        than 70 % of its slots (steps bound by the item degree of the
        blocks, not by the slot count), the 8-wave plan is built too and
        kept if steps * waves -- the per-CU VALU issue of an epoch, which
        bounds such plans (PMC) -- is lower.

        ``phases``: item phases (PhasedStrata).  None = by the plan (env
        MF_STRATA_PHASES overrides): one phase while the default B fits one
        workgroup per CU, else the fewest phases whose B does.

        ``item_bounds``: the phases' item ranges given explicitly (len P + 1
        ascending ids from 0 to n_items) -- the item ranges of the rotation
        schedule (distributed.item_ranges); a PhasedStrata even for P = 1.

        ``classes``: user-range classes C (C*B user ranges, C*B strata per
        epoch; the persistent kernel then hands a user range over with C - 1
        blocks of slack, and an item meets 1/C of a block's ratings per user
        range).  None = ``strata_classes`` / env MF_STRATA_CLASSES; "auto"
        (the default) = ``auto_classes`` for the engine's own B (n_blocks
        None, no item_bounds), else 1.

        ``regroup``: relabelled plans to build (1 = none); None = by
        ``strata_regroup`` / env MF_STRATA_REGROUP.  Engines that only run
        the delta-out form (exchange="delta") pass 1: delta epochs always
        run the engine's own plan, so regroupings would be dead weight (a
        second padded copy of the ratings and of P / Q)."""
        if self.colored is not None or self.strata is not None:
            raise RuntimeError("ratings already permuted by another schedule")
        classes = self._classes(classes)
        auto_classes = classes is None
        if auto_classes:
            classes = 1
        env = os.environ.get("MF_STRATA_WAVES")
        if waves is None and env in ("4", "8", "16"):
            waves = int(env)
        if item_bounds is not None:
            ilo = np.asarray(item_bounds, np.int64)
            if (len(ilo) < 2 or ilo[0] != 0 or ilo[-1] != self.n_items
                    or np.any(np.diff(ilo) < 0)):
                raise ValueError("item_bounds must ascend from 0 to n_items")
            self.strata = self._prepare_phased(len(ilo) - 1, n_blocks, waves, ilo,
                                               per_b2=ROTATE_PER_B2, classes=classes)
            return self.strata
        if phases is None and os.environ.get("MF_STRATA_PHASES"):
            phases = int(os.environ["MF_STRATA_PHASES"])
        bounds = None
        auto_l2 = False
        if phases is None and n_blocks is None:
            phases, n_blocks, bounds = self._item_phases(classes)
            if auto_classes:
                classes = self.auto_classes(n_blocks)
                if classes > 1:
                    phases, n_blocks, bounds = self._item_phases(classes)
            if phases == 1 and classes == 1 and self._l2_handoff_fits():
                B8 = min(self._cus(), -(-n_blocks // XCD_CLASSES) * XCD_CLASSES)
                b8 = self._bounds_for(B8) if B8 >= 2 * XCD_CLASSES else None
                if b8 is not None:
                    n_blocks, bounds, auto_l2 = B8, b8, True
        # the regroupings' plans (same B, classes and phases) are built on a
        # worker thread while this one builds the engine's own: the planner
        # is host code that releases the GIL
        K = self._regroup_count(classes) if regroup is None else int(regroup)
        if not 1 <= K <= self.REGROUP_MAX:
            raise ValueError(f"strata regroupings must be in [1, {self.REGROUP_MAX}], got {K}")
        worker = None
        if K > 1 and n_blocks is not None:
            worker = ThreadPoolExecutor(1)
            fut = worker.submit(self._build_regroups, K, int(n_blocks), phases, classes, waves)
        try:
            if phases is not None and int(phases) > 1:
                plan = self._prepare_phased(int(phases), n_blocks, waves, classes=classes)
            else:
                cums = ((self.degree_cum("user"), self.degree_cum("item"))
                        if bounds is None and n_blocks is not None else (None, None))
                plan = self._build_plan(self.u_host, self.i_host, self.n_items, n_blocks, waves,
                                        bounds, classes, cums)
                plan.to_device(self.u, self.i, self.r, self.dev)
                if auto_l2:
                    plan.l2_handoff, plan.order = True, "xcd"
        finally:
            if worker is not None:
                regroups = fut.result()
                worker.shutdown()
        if K > 1 and worker is None:         # B known only now: after the engine's plan
            regroups = self._build_regroups(
                K, plan.B, len(plan.phases) if isinstance(plan, PhasedStrata) else None,
                classes, waves)
        if K > 1:
            for e, _, _ in regroups:
                if e.strata.n_strata != plan.n_strata or e.strata.B != plan.B:
                    raise RuntimeError("a regrouped plan differs from the engine's in shape")
                self._regroup_buffers(e)
            self._regroups = regroups
        self.strata = plan
        # the persistent sweep's workspace (position counters, error word)
        # now, not in the first epoch
        if self.n:
            self._ensure_strata_ws(plan.B, plan.n_strata)
            self._prime_strata(plan)
        return plan

    def _prime_strata(self, pl) -> None:
        """The launcher's one-time runtime work for this plan's kernels
        (MF_FLAG_PREPARE: kernel attributes, the co-residency query -- no
        launch, the parameters untouched), so that it is not paid inside
        fit()'s first epochs."""
        subs = pl.phases if isinstance(pl, PhasedStrata) else [pl]
        for sub in subs:
            if sub.n_positions == 0:
                continue
            seq = np.arange(sub.n_strata, dtype=np.int32)
            flags = self._strata_flags(sub, None) | _lib.MF_FLAG_PREPARE
            self._run_strata(sub, seq, 0, 0.0, 0.0, True, True, flags, None, None, self.Q,
                             self.bi, self.n_items)

    # relabelled plans, "regroupings" (DESIGN.md section 3.1): K - 1 more
    # plans of the same B and classes over randomly relabelled users and
    # items; every epoch's rotation seed picks one, so which users share a
    # range and which items share a slab is re-drawn epoch to epoch.  C3,
    # 4 classes, 20 epochs: train RMSE +1.18e-5 over the reference's mean
    # with one plan (3.6 SE), +0.73e-5 with two (2.1 SE), +0.79e-5 with four
    # (profiles/r04/seed_spread_c3_20ep_regroup_r04q.json).  "auto" = 2 for
    # the linear kernel's multi-class plans (the order-bias regime), else 1;
    # env MF_STRATA_REGROUP overrides.
    strata_regroup = "auto"
    REGROUP_AUTO = 2
    REGROUP_MAX = 4
    REGROUP_SEED = 0x5EED

    def _regroup_count(self, classes: int) -> int:
        if getattr(self, "_regroup_of", None) is not None:
            return 1                          # a regrouping's own engine: one plan
        k = os.environ.get("MF_STRATA_REGROUP", self.strata_regroup)
        if k in (None, "auto"):
            return (self.REGROUP_AUTO if classes > 1 and self.kernel == "linear"
                    and self.n > 0 else 1)
        k = int(k)
        if not 1 <= k <= self.REGROUP_MAX:
            raise ValueError(f"strata regroupings must be in [1, {self.REGROUP_MAX}], got {k}")
        return k

    def _build_regroups(self, K: int, B: int, phases, classes: int, waves) -> list:
        """Regroupings 1..K-1: engines over relabelled ids (user x -> pu[x],
        item y -> pi[y]) with plans of the same B, classes and phases.  Each
        shares this engine's persistent-sweep workspace (position counters,
        error word) when it runs, so failure detection and recovery see its
        launches too."""
        out = []
        # (runs on a worker thread: the device is set explicitly, the
        # thread's current one need not be this engine's)
        with torch.cuda.device(self.dev):
            for j in range(1, K):
                out.append(self._build_regroup(j, B, phases, classes, waves))
        return out

    def _build_regroup(self, j: int, B: int, phases, classes: int, waves):
        """Regrouping j's engine and its device permutations (pu, pi)."""
        rs = np.random.RandomState(self.REGROUP_SEED + j)
        pu_h = rs.permutation(self.n_users).astype(np.int32)
        pi_h = rs.permutation(self.n_items).astype(np.int32)
        pu = torch.from_numpy(pu_h).to(self.dev)
        pi = torch.from_numpy(pi_h).to(self.dev)
        uj_d = pu.index_select(0, self.u)
        ij_d = pi.index_select(0, self.i)
        # the relabelled ids: on the device for the engine (no upload), and
        # relabelled on the host threads for the planner (no read-back of
        # 2 x 4 bytes per rating); the ratings are this engine's (read-only)
        uj_h = _prep.gather(pu_h, self.u_host)
        ij_h = _prep.gather(pi_h, self.i_host)
        pu, pi = pu.long(), pi.long()
        e = SGDEngine(uj_h, ij_h, self.r_host, self.n_users,
                      self.n_items, self.k, self.kernel, self.dtype, self.dev, self.gamma,
                      self.min_rating, self.max_rating, self.global_mean, eval_order=False,
                      check_ids=False, device_triples=(uj_d, ij_d, self.r))
        e.strata_persistent = self.strata_persistent
        e.strata_deep_pipe = self.strata_deep_pipe
        e.strata_stream = self.strata_stream
        e.strata_regroup = 1
        e._regroup_of = j                 # never regroups itself (env included)
        e.prepare_strata(n_blocks=B, waves=waves,
                         phases=phases if phases is not None and int(phases) > 1 else None,
                         classes=classes)
        return e, pu, pi

    def _regroup_pick(self, seed: int) -> int:
        """Which plan runs the epoch with rotation seed ``seed`` (0 = this
        engine's own): a hash of the seed, so replays pick the same."""
        K = 1 + len(self._regroups)
        if K == 1:
            return 0
        return int((((int(seed) & 0xFFFFFFFF) * 2654435761) & 0xFFFFFFFF) >> 16) % K

    def serial_order(self, seq, seed, delta: bool = False) -> np.ndarray:
        """The rating indices in the order the strata epoch (seq, seed)
        applies them, whichever plan it picks (indices into this engine's
        rating arrays; a regrouping lists the same ratings).  ``delta``: the
        epoch ran in delta-out form, which always runs the engine's own plan
        (epoch_strata with ``delta``)."""
        j = 0 if delta else self._regroup_pick(seed)
        pl = self.strata if j == 0 else self._regroups[j - 1][0].strata
        return pl.serial_order(seq, seed)

    # the automatic choice of user-range classes: the
    # strata order trains measurably slower than the reference's random order
    # when an item meets many ratings of one user range inside a block -- at
    # C3 (linear, rank 64, 3.9 ratings per item and block) train RMSE after 20
    # epochs +4.7e-5 over the reference's mean (12 shuffle seeds, SD 8e-6),
    # +2.0e-5 with 2 classes, +1.1e-5 with 4 (profiles/r04/seed_spread_*);
    # the sigmoid kernel at C2 (7.2 per block, effective step scaled by the
    # sigmoid's derivative) shows none (+1.1e-6, profiles/r04/order_bias_cpu_c2.json)
    AUTO_CLASSES = AUTO_CLASSES
    AUTO_CLASSES_MIN_DEGREE = AUTO_CLASSES_MIN_DEGREE

    def auto_classes(self, B: int) -> int:
        """Classes for the engine's own plan of B workgroups: AUTO_CLASSES for
        the linear kernel when an item meets at least AUTO_CLASSES_MIN_DEGREE
        ratings per user range of the one-class plan, else 1."""
        return auto_strata_classes(self.kernel, self.n, self.n_items, B)

    def _l2_handoff_fits(self) -> bool:
        """MF_FLAG_L2_HANDOFF by the plan (env MF_STRATA_L2=0 / 1 forces it
        off / leaves it to the order): P small enough that the rows an XCD
        hands over stay in its L2, rows of whole 128-B lines."""
        if os.environ.get("MF_STRATA_L2") in ("0", "1") or self.bias_only:
            return False
        ts = np.dtype(self.ndt).itemsize
        return (self.n_users * self.k * ts <= L2_HANDOFF_P_BYTES
                and (self.k * ts) % 128 == 0)

    def _bounds_for(self, B: int):
        """User / item bounds of a B-block plan over all ratings, or None if
        its largest block does not fit the LDS."""
        lib = _lib.load()
        ub = balanced_bounds(self.u_host, self.n_users, B, cum=self.degree_cum("user"))
        icum = self.degree_cum("item")
        for by_count in (True, False):
            ib = balanced_bounds(self.i_host, self.n_items, B, by_count, cum=icum)
            need = lib.mf_strata_lds_bytes(int(np.diff(ib).max()), int(np.diff(ub).max()),
                                           self.k, self.dcode)
            if need <= lib.mf_strata_lds_limit():
                return ub, ib
        return None

    def degree_cum(self, side: str) -> Optional[np.ndarray]:
        """Cumulative rating count per user (or item) id, from a histogram of
        the uploaded ids on the device (np.bincount of 10^8 host ids takes
        a large part of a second; the plan's balanced bounds need it)."""
        ids = self.u if side == "user" else self.i
        m = self.n_users if side == "user" else self.n_items
        if self.n == 0 or ids is None:
            return None
        h = torch.bincount(ids, minlength=m)
        return torch.cumsum(h, 0).cpu().numpy().astype(np.int64)

    def _cus(self) -> int:
        if self.dev.type != "cuda":
            return 256
        return int(torch.cuda.get_device_properties(self.dev).multi_processor_count)

    def _item_phases(self, classes: int = 1):
        """(P, B, bounds): 1 phase and the default B with its user / item
        bounds when the plan's workgroups fit one per CU; else the fewest item
        phases whose common B does (see PhasedStrata), bounds None."""
        cus = self._cus()
        B, ub, ib = choose_strata_blocks(self.u_host, self.i_host, self.n_users, self.n_items,
                                         self.k, self.dcode, classes=classes,
                                         cums=(self.degree_cum("user"), self.degree_cum("item")))
        if B <= cus or self.n == 0:
            return 1, B, (ub, ib)
        icum = self.degree_cum("item")
        for P in range(2, 9):
            ilo = balanced_bounds(self.i_host, self.n_items, P, cum=icum)
            Bp = 0
            for p in range(P):
                # the phase's degree counts on the device; the host arrays are
                # only sized stand-ins (choose_strata_blocks reads their
                # lengths when given the counts)
                lo, hi = int(ilo[p]), int(ilo[p + 1])
                m = (self.i >= lo) & (self.i < hi)
                n_p = int(m.sum())
                cu = torch.cumsum(torch.bincount(self.u[m], minlength=self.n_users),
                                  0).cpu().numpy()
                ci = torch.cumsum(torch.bincount(self.i[m] - lo, minlength=max(hi - lo, 1)),
                                  0).cpu().numpy()
                del m
                stand_in = np.empty(n_p, np.int32)
                b, _, _ = choose_strata_blocks(stand_in, stand_in, self.n_users, hi - lo,
                                               self.k, self.dcode, max_blocks=cus,
                                               classes=classes, cums=(cu, ci))
                Bp = max(Bp, b)
            if Bp <= cus:
                # every phase on all the CUs: B = CUs fits (the LDS image only
                # shrinks as B grows) and is faster than the ratings rule's B
                # (C3 FP64, 2 phases: B = 220 / 240 / 256 -> SGD 21.25 /
                # 20.49 / 19.99 ms, profiles/r04/classes_probe_fp64_blocks_r04d.txt)
                return P, max(Bp, min(cus, 256)), None
        return 1, B, (ub, ib)               # no persistent form: one launch per stratum

    def _build_plan(self, u, i, n_items, n_blocks, waves, bounds=None,
                    classes: int = 1, cums=(None, None)) -> "StrataPlan":
        if bounds is not None:
            B, (ub, ib) = int(n_blocks), bounds
        elif n_blocks is None:
            B, ub, ib = choose_strata_blocks(u, i, self.n_users, n_items, self.k, self.dcode,
                                             classes=classes, cums=cums)
        else:
            B = int(n_blocks)
            ub = balanced_bounds(u, self.n_users, classes * B, cum=cums[0])
            ib = balanced_bounds(i, n_items, B, cum=cums[1])
            need = _lib.load().mf_strata_lds_bytes(int(np.diff(ib).max()), int(np.diff(ub).max()),
                                                   self.k, self.dcode)
            if need > _lib.load().mf_strata_lds_limit():
                ib = balanced_bounds(i, n_items, B, False)   # equal item counts
        cand = [waves] if waves is not None else [16, 8]
        shapes = []
        for wv in cand:
            ns = strata_slots(self.k, self.dcode, wv)
            if ns <= 0:
                if waves is not None:
                    raise ValueError(f"no {wv}-wave strata kernel for n_factors={self.k}, "
                                     f"dtype={self.dtype}")
                continue
            shapes.append((ns, wv))
        if not shapes:
            raise ValueError(f"no strata kernel for n_factors={self.k}, dtype={self.dtype}")
        # the shape of least steps * waves (the per-CU VALU issue of an epoch);
        # the 16-wave plan outright when it fills 70 % of its positions.  Only
        # the pick is coloured (mf_strata_plan_build_pick)
        fill_stop = 0.7 if waves is None and shapes[0][1] == 16 else 0.0
        sched, bstep, j = sched_strata_pick(u, i, self.n_users, n_items, B, ub, ib, shapes,
                                            classes, fill_stop)
        ns = shapes[j][0]
        plan = StrataPlan(B, ns, ub, ib, bstep, sched, classes)
        plan.narrow = waves == 4
        return plan

    def _prepare_phased(self, P: int, n_blocks, waves, ilo=None,
                        per_b2: float = STRATA_PER_B2, classes: int = 1) -> PhasedStrata:
        if ilo is None:
            ilo = balanced_bounds(self.i_host, self.n_items, P,
                                  cum=self.degree_cum("item")).astype(np.int64)
        # each phase's rating indices in rating order, found on the device
        # (10^8 ratings: a host argsort took seconds)
        bnd = torch.from_numpy(np.ascontiguousarray(ilo[1:-1])).to(self.dev, torch.int32)
        ph = torch.bucketize(self.i, bnd, right=True)
        idx_d = [torch.nonzero(ph == p).flatten() for p in range(P)]
        del ph
        # read back as 32-bit indices (half the bytes; serial_order widens)
        narrow = self.n < (1 << 31)
        idx = [(t.to(torch.int32) if narrow else t).cpu().numpy() for t in idx_d]

        def cums(p):
            t = idx_d[p]
            cu = torch.cumsum(torch.bincount(self.u.index_select(0, t), minlength=self.n_users),
                              0).cpu().numpy()
            ci = torch.cumsum(torch.bincount(self.i.index_select(0, t) - int(ilo[p]),
                                             minlength=max(int(ilo[p + 1] - ilo[p]), 1)),
                              0).cpu().numpy()
            return cu, ci

        pcums = [cums(p) for p in range(P)]
        if n_blocks is None:                # one B for every phase: the largest needed
            # (given the counts, choose_strata_blocks reads the id arrays'
            # lengths only: sized stand-ins)
            n_blocks = max(choose_strata_blocks(np.empty(len(ix), np.int32),
                                                np.empty(len(ix), np.int32),
                                                self.n_users, max(int(ilo[p + 1] - ilo[p]), 1),
                                                self.k, self.dcode, per_b2=per_b2,
                                                classes=classes, cums=pcums[p])[0]
                           for p, ix in enumerate(idx))
        plans = []
        for p, ix in enumerate(idx):
            # the phase's ids on the host threads (NumPy's fancy indexing of
            # 5 * 10^7 rows ran on one thread: ~0.2 s per array at C3)
            ui = _prep.gather(self.u_host, ix)
            ii = _prep.gather(self.i_host, ix)
            ii -= np.int32(ilo[p])
            pl = self._build_plan(ui, ii, int(ilo[p + 1] - ilo[p]), n_blocks, waves,
                                  classes=classes, cums=pcums[p])
            if waves is None:               # phase 0 picks the kernel shape for all
                waves = 16 if pl.NS == strata_slots(self.k, self.dcode, 16) else 8
            t = idx_d[p]
            pl.to_device(self.u.index_select(0, t), self.i.index_select(0, t) - int(ilo[p]),
                         self.r.index_select(0, t), self.dev)
            plans.append(pl)
        return PhasedStrata(plans, idx, ilo)

    # one launch per epoch with the item slabs resident (MF_FLAG_PERSISTENT);
    # False: one launch per stratum
    strata_persistent = True
    # user rows two steps ahead in the persistent sweep (MF_FLAG_DEEP_PIPE):
    # None = by the plan, True / False forced; env MF_STRATA_DEEP=0/1 overrides
    strata_deep_pipe: Optional[bool] = None
    # the stream form of the multi-class persistent sweep (MF_FLAG_STREAM:
    # one software pipeline through all positions of a launch, DESIGN.md
    # section 5 "stream"); None = the default, True / False forced; env
    # MF_STRATA_STREAM=0/1 overrides.  Used where it applies: persistent,
    # user-range classes C > 1, the depth-2 pipeline.
    strata_stream: Optional[bool] = None
    # on: C3 FP64 SGD 24.27 -> 20.10 ms, FP32 11.11 -> 10.32 ms on one box
    # (profiles/r05/bench_c3_stream_r05e.json, ..._nostream_same_box_r05e.json)
    STREAM_DEFAULT = True

    def _stream(self) -> bool:
        env = os.environ.get("MF_STRATA_STREAM")
        if env in ("0", "1"):
            return env == "1"
        if self.strata_stream is not None:
            return bool(self.strata_stream)
        return self.STREAM_DEFAULT

    def _deep_pipe(self, pl) -> bool:
        """By the plan: on for plans of few busy slots per step (the 8-wave
        plans, or 16-wave plans filled below 70 %), whose steps wait on the
        per-CU memory round trip rather than on HBM bandwidth; off for
        well-filled plans (C3: 9.25 vs 9.43 ms with it; C2 8-wave 0.925 ->
        0.902 ms, C3 N=8 shard 1.900 -> 1.884 ms)."""
        env = os.environ.get("MF_STRATA_DEEP")
        if env in ("0", "1"):
            return env == "1"
        if self.strata_deep_pipe is not None:
            return bool(self.strata_deep_pipe)
        if pl.narrow:
            return False                       # no depth-2 form of the 4-wave kernels
        n = pl.n_ratings if isinstance(pl, StrataPlan) else self.n
        fill = n / max(pl.n_positions, 1)
        return pl.NS == strata_slots(self.k, self.dcode, 8) or fill < 0.7

    def epoch_strata(self, seq: Optional[np.ndarray], seed: int, lr: float, reg: float,
                     update_user: bool = True, update_item: bool = True, timing=False,
                     persistent: Optional[bool] = None, delta=None):
        """Apply the strata listed in ``seq`` (a permutation of
        range(n_strata) is one epoch; stratum_order draws one) with step
        rotation ``seed``.  ``delta`` = (dQ, db_i)
        device tensors: delta-out form (mf_sgd_epoch_strata_delta) -- Q and
        b_i keep their values, the epoch's item update goes to the deltas."""
        pl = self.strata
        if pl is None:
            raise RuntimeError("call prepare_strata() first")
        seq = (np.arange(pl.n_strata, dtype=np.int32) if seq is None
               else np.ascontiguousarray(seq, np.int32))
        j = self._regroup_pick(seed) if delta is None else 0
        if j > 0:
            return self._epoch_regroup(j - 1, seq, seed, lr, reg, update_user, update_item,
                                       timing, persistent)
        if isinstance(pl, PhasedStrata):
            return self._epoch_phased(pl, seq, seed, lr, reg, update_user, update_item, timing,
                                      persistent, delta)
        ms = (ctypes.c_double * 2)() if timing else None
        flags = self._strata_flags(pl, persistent)
        self._run_strata(pl, seq, seed, lr, reg, update_user, update_item, flags, ms, delta,
                         self.Q, self.bi, self.n_items)
        return (ms[0], int(ms[1])) if timing else None

    def _epoch_regroup(self, j, seq, seed, lr, reg, update_user, update_item, timing,
                       persistent):
        """One epoch on regrouping j: the parameters are gathered into its
        labelling, swept there, and gathered back (device index copies)."""
        e, pu, pi = self._regroups[j]
        e.global_mean, e.gamma = self.global_mean, self.gamma
        e.min_rating, e.max_rating = self.min_rating, self.max_rating
        self._regroup_buffers(e)
        # into the plan's labelling (one launch: P, Q, b_u, b_i scattered by
        # the user / item relabellings), the sweep there, and back (gathered)
        self._permute(e, pu, pi, scatter=True)
        self._ensure_strata_ws(e.strata.B, len(seq))
        e._strata_ws = self._strata_ws           # shared counters and error word
        out = e.epoch_strata(seq, seed, lr, reg, update_user, update_item, timing, persistent)
        self._permute(e, pu, pi, scatter=False)
        return out

    def _regroup_buffers(self, e) -> None:
        """Parameter storage of a relabelled plan's engine (allocated once,
        when the plan is built: an allocation inside the first regrouped
        epoch cost ~20 ms of fit()'s epoch 2)."""
        if self.P is None:
            shapes = ((self.n_users, self.k), (self.n_items, self.k), (self.n_users,),
                      (self.n_items,))
            ref = [torch.empty(sh, dtype=self.tdt, device=self.dev) for sh in shapes]
            if self.bias_only:
                ref[0] = ref[1] = None
        else:
            ref = [self.P, self.Q, self.bu, self.bi]
        have = (e.P, e.Q, e.bu, e.bi)
        if all((a is None) == (b is None) and (a is None or a.shape == b.shape)
               for a, b in zip(have, ref)):
            return
        e.load_params(*(None if t is None else torch.zeros_like(t) for t in ref))

    def _permute(self, e, pu, pi, scatter: bool) -> None:
        """mf_permute_rows: scatter (this engine's parameters -> the plan's
        labelling: e.X[p[x]] = X[x]) or gather (back: X[x] = e.X[p[x]])."""
        jobs = [(e.P, self.P, pu), (e.Q, self.Q, pi), (e.bu, self.bu, pu), (e.bi, self.bi, pi)]
        jobs = [(a, b, p) for a, b, p in jobs if a is not None and b is not None]
        n = len(jobs)
        dst = (ctypes.c_void_p * n)(*[(a if scatter else b).data_ptr() for a, b, _ in jobs])
        src = (ctypes.c_void_p * n)(*[(b if scatter else a).data_ptr() for a, b, _ in jobs])
        idx = (ctypes.c_void_p * n)(*[p.data_ptr() for _, _, p in jobs])
        rows = (ctypes.c_int64 * n)(*[b.shape[0] for _, b, _ in jobs])
        rb = (ctypes.c_int32 * n)(*[b[0].numel() * b.element_size() if b.shape[0] else 4
                                    for _, b, _ in jobs])
        with torch.cuda.device(self.dev):
            _lib.call("mf_permute_rows", n, dst, src, idx, rows, rb, 0 if not scatter else 1,
                      self.stream)

    def _ensure_strata_ws(self, B: int, n_seq: int) -> None:
        wsb = int(_lib.load().mf_strata_workspace_bytes(B, n_seq))
        old = getattr(self, "_strata_ws", None)
        if old is None or old.numel() * 4 < wsb:
            # zeroed once: the error flag (int32 at index B) is sticky until
            # check_strata() raises or clear_strata_error() resets it, and
            # the position counters done[0:B] grow across launches; a grown
            # workspace carries both over
            ws = torch.zeros((wsb + 3) // 4, dtype=torch.int32, device=self.dev)
            if old is not None:
                ws[: B + 1] = old[: B + 1]
            self._strata_ws = ws

    def _strata_flags(self, pl, persistent):
        if persistent is None:
            persistent = self.strata_persistent and os.environ.get("MF_STRATA_PERSISTENT") != "0"
        flags = _lib.MF_FLAG_PERSISTENT if persistent else 0
        if persistent and self._deep_pipe(pl):
            flags |= _lib.MF_FLAG_DEEP_PIPE
            # the stream kernel keeps a block's step count in a 16-bit field
            # of its LDS geometry table: a plan with a longer block runs the
            # per-block form (same order, bit for bit)
            if pl.classes > 1 and self._stream() and max_block_steps(pl) <= STREAM_MAX_STEPS:
                flags |= _lib.MF_FLAG_STREAM
        if os.environ.get("MF_STRATA_COOP") == "0" or _under_rocprofiler():
            flags |= _lib.MF_FLAG_NO_COOP
        if os.environ.get("MF_STRATA_EARLY") == "0":
            flags |= _lib.MF_FLAG_NO_EARLY_POLL
        if pl.narrow:
            flags |= _lib.MF_FLAG_NARROW
        flags |= (pl.classes - 1) << _lib.MF_FLAG_CLASSES_SHIFT
        # user rows handed over inside an XCD through its L2 (needs the
        # XCD-class stratum order; the launcher checks the order, the kernel
        # the placement) -- DESIGN.md section 5
        l2 = os.environ.get("MF_STRATA_L2")
        if persistent and (l2 == "1" or (l2 is None and getattr(pl, "l2_handoff", False))):
            flags |= _lib.MF_FLAG_L2_HANDOFF
        return flags

    def _epoch_phased(self, pl, seq, seed, lr, reg, update_user, update_item, timing,
                      persistent, delta):
        """The phases of one epoch in order, each on its rows of Q / b_i (and
        of the delta buffers)."""
        flags = self._strata_flags(pl, persistent)
        tot_ms, launches = 0.0, 0
        for p, sub in enumerate(pl.phases):
            lo, hi = int(pl.ilo[p]), int(pl.ilo[p + 1])
            ms = (ctypes.c_double * 2)() if timing else None
            d = None if delta is None else (delta[0][lo:hi], delta[1][lo:hi])
            self._run_strata(sub, seq, seed, lr, reg, update_user, update_item, flags, ms, d,
                             self.Q[lo:hi], self.bi[lo:hi] if self.bi is not None else None,
                             hi - lo)
            if timing:
                tot_ms += ms[0]
                launches += int(ms[1])
        return (tot_ms, launches) if timing else None

    def epoch_phase(self, p: int, seq: Optional[np.ndarray], seed: int, lr: float, reg: float,
                    update_user: bool = True, update_item: bool = True, timing=False,
                    persistent: Optional[bool] = None):
        """Phase ``p`` of a PhasedStrata plan alone, in place on its rows of
        Q / b_i: one sub-epoch of the rotation schedule (distributed.py), the
        item range this rank holds at that moment.  ``seq`` is a permutation
        of range(B) (None: 0..B-1)."""
        pl = self.strata
        if not isinstance(pl, PhasedStrata):
            raise RuntimeError("epoch_phase needs prepare_strata(item_bounds=...) or phases")
        seq = (np.arange(pl.n_strata, dtype=np.int32) if seq is None
               else np.ascontiguousarray(seq, np.int32))
        sub = pl.phases[p]
        lo, hi = int(pl.ilo[p]), int(pl.ilo[p + 1])
        ms = (ctypes.c_double * 2)() if timing else None
        if sub.n_positions == 0 or hi == lo:
            return (0.0, 0) if timing else None
        flags = self._strata_flags(sub, persistent)
        self._run_strata(sub, seq, seed, lr, reg, update_user, update_item, flags, ms, None,
                         self.Q[lo:hi], self.bi[lo:hi] if self.bi is not None else None, hi - lo)
        return (ms[0], int(ms[1])) if timing else None

    def _run_strata(self, pl, seq, seed, lr, reg, update_user, update_item, flags, ms, delta,
                    Q, bi, n_items):
        self._ensure_strata_ws(pl.B, len(seq))
        args = (_tp(pl.d_u), _tp(pl.d_i), _tp(pl.d_r),
                pl.n_positions, pl.B, _tp(pl.d_ubnd), _tp(pl.d_ibnd), _tp(pl.d_bstep),
                pl.NS, pl.max_items, pl.max_users, _np(seq), len(seq),
                int(seed) & 0xFFFFFFFF, self.global_mean, _tp(self.bu), _tp(bi),
                _tp(self.P), _tp(Q), self.n_users, n_items, self.k,
                self.kcode, self.dcode, self.gamma, float(lr), float(reg),
                self.min_rating, self.max_rating, int(update_user), int(update_item),
                flags, _tp(self._strata_ws), self._strata_ws.numel() * 4)
        with torch.cuda.device(self.dev):
            if delta is None:
                _lib.call("mf_sgd_epoch_strata", *args, self.stream, ms)
            else:
                _lib.call("mf_sgd_epoch_strata_delta", *args, _tp(delta[0]), _tp(delta[1]),
                          self.stream, ms)

    def check_strata(self) -> None:
        """Synchronise and raise if a persistent strata sweep gave up waiting
        (its parameters would be invalid)."""
        ws = getattr(self, "_strata_ws", None)
        if ws is None:
            return
        with torch.cuda.device(self.dev):
            _lib.call("mf_strata_status", _tp(ws), self.strata.B, self.stream)

    def strata_failed(self) -> bool:
        """Synchronise; True if a persistent sweep gave up waiting since the
        error flag was last cleared (non-raising form of check_strata)."""
        ws = getattr(self, "_strata_ws", None)
        return ws is not None and int(ws[self.strata.B].item()) != 0

    def clear_strata_error(self) -> None:
        """Reset the workspace after a failed persistent sweep: the error word
        and the position counters (they grow across launches and are left
        uneven by workgroups that gave up)."""
        ws = getattr(self, "_strata_ws", None)
        if ws is not None:
            ws.zero_()

    def snapshot_params(self):
        """Device copies of (P, Q, b_u, b_i) (restore_params puts them back)."""
        return tuple(None if t is None else t.clone() for t in (self.P, self.Q, self.bu, self.bi))

    def restore_params(self, snap) -> None:
        for t, s in zip((self.P, self.Q, self.bu, self.bi), snap):
            if t is not None:
                t.copy_(s)

    def epoch_strata_checked(self, seq, seed, lr, reg, update_user=True, update_item=True):
        """One strata epoch that cannot leave invalid parameters behind: the
        persistent sweep runs from a device snapshot of the parameters; if a
        workgroup gave up waiting for its neighbour (another process holding
        CUs, say), the snapshot is restored and the same epoch -- same
        strata, same rotation, hence the same sequential order -- is re-run
        as one launch per stratum.  Returns True if the fallback ran."""
        if not self.strata_persistent:
            self.epoch_strata(seq, seed, lr, reg, update_user, update_item)
            return False
        snap = self.snapshot_params()
        self.epoch_strata(seq, seed, lr, reg, update_user, update_item)
        if not self.strata_failed():
            return False
        self.restore_params(snap)
        self.clear_strata_error()
        self.epoch_strata(seq, seed, lr, reg, update_user, update_item, persistent=False)
        return True

    def epoch_exact(self, order: np.ndarray, lr: float, reg: float,
                    update_user: bool = True, update_item: bool = True,
                    timing=False):
        """One epoch in the given visit order (rating indices).  ``timing``
        (True or a stride S): returns (ms of the bracketed launches, count)."""
        if self.colored is not None or self.strata is not None:
            raise RuntimeError("engine holds permuted ratings; exact order "
                               "needs the original order")
        if order is not None and order.dtype == np.int32 and self.n > 0:
            return self._epoch_exact_chunked(order, lr, reg, update_user, update_item, timing)
        sched, offs = sched_levels(self.u_host, self.i_host, order, self.n_users,
                                   self.n_items, update_user, update_item)
        idx = torch.from_numpy(sched).to(self.dev)
        return self._run(idx, offs, None, lr, reg, update_user, update_item, 0, timing)

    def _epoch_exact_chunked(self, order, lr, reg, update_user, update_item, timing):
        """epoch_exact for a 32-bit visit order: the levels built on host
        threads (sched_levels_chunked, the same bits as the greedy levels)
        straight into one of two pinned buffers, uploaded asynchronously on
        the launch stream (the host builds epoch e+1's levels while the GPU
        still runs epoch e).  Host AND device schedules are double-buffered:
        pair k is rewritten only once the event recorded after epoch k's
        level launches has completed, so a caller that switches streams
        between epochs cannot overwrite a schedule still being read."""
        st = getattr(self, "_exact_bufs", None)
        if st is None or st["host"][0].numel() < self.n:
            st = {"host": [torch.empty(self.n, dtype=torch.int32, pin_memory=True)
                           for _ in range(2)],
                  "ev": [None, None], "flip": 0,
                  "dev": [torch.empty(self.n, dtype=torch.int32, device=self.dev)
                          for _ in range(2)]}
            self._exact_bufs = st
        k = st["flip"]
        st["flip"] ^= 1
        if st["ev"][k] is not None:
            st["ev"][k].synchronize()
        hb, db = st["host"][k], st["dev"][k]
        _, offs = sched_levels_chunked(self.u_host, self.i_host, order, self.n_users,
                                       self.n_items, update_user, update_item,
                                       out=hb.numpy())
        with torch.cuda.device(self.dev):
            stream = torch.cuda.current_stream(self.dev)
            db[: self.n].copy_(hb[: self.n], non_blocking=True)
            out = self._run(db, offs, None, lr, reg, update_user, update_item, 0, timing)
            ev = torch.cuda.Event()
            ev.record(stream)           # after the upload AND the launches reading db
            st["ev"][k] = ev
        return out

    def epoch_colored(self, seq: Optional[np.ndarray], lr: float, reg: float,
                      update_user: bool = True, update_item: bool = True,
                      flags: Optional[int] = None, timing=False):
        """Apply the colours listed in ``seq`` in that order (a permutation of
        all colours is one epoch; a prefix is a partial epoch)."""
        if self.colored is None:
            raise RuntimeError("call prepare_colored() first")
        if seq is not None:
            seq = np.ascontiguousarray(seq, np.int32)
        if flags is None:
            flags = default_sgd_flags()
        return self._run(None, self.colored, seq, lr, reg, update_user,
                         update_item, flags, timing)

    def _claim_ws(self, n_launch):
        """Per-launch tile counters for MF_FLAG_XCD_CLAIM (8 int32 each)."""
        need = 8 * max(n_launch, 1)
        if getattr(self, "_claim", None) is None or self._claim.numel() < need:
            self._claim = torch.zeros(need, dtype=torch.int32, device=self.dev)
        return self._claim

    def _run(self, idx, offs, seq, lr, reg, update_user, update_item, flags, timing):
        nb = len(offs) - 1
        nseq = 0 if seq is None else len(seq)
        ms = (ctypes.c_double * 2)() if timing else None
        if timing and timing is not True:
            flags = int(flags) | (int(timing) << 16)       # timing = stride
        with torch.cuda.device(self.dev):
            if self.bias_only:
                _lib.call("mf_bias_sgd_epoch", _tp(self.u), _tp(self.i), _tp(self.r),
                          self.n, _tp(idx), _np(offs), nb, _np(seq), nseq,
                          self.global_mean, _tp(self.bu), _tp(self.bi), self.dcode,
                          float(lr), float(reg), int(update_user), int(update_item),
                          self.stream)
                return None
            _lib.call("mf_sgd_epoch", _tp(self.u), _tp(self.i), _tp(self.r), self.n,
                      _tp(idx), _np(offs), nb, _np(seq), nseq, self.global_mean,
                      _tp(self.bu), _tp(self.bi), _tp(self.P), _tp(self.Q),
                      self.n_users, self.n_items, self.k, self.kcode, self.dcode,
                      self.gamma, float(lr), float(reg), self.min_rating,
                      self.max_rating, int(update_user), int(update_item), int(flags),
                      _tp(self._claim_ws(nseq or nb)), 8 * 4 * max(nseq or nb, 1),
                      self.stream, ms)
        return (ms[0], int(ms[1])) if timing else None

    # ---------------------------------------------------------- read-only
    def sse_async(self, slot: int) -> None:
        """Enqueue the training SSE into device slot ``slot``."""
        self._ensure_sse_slots(slot + 1)
        out = _VOID(self.sse_buf.data_ptr() + 8 * slot)
        with torch.cuda.device(self.dev):
            if self.bias_only:
                _lib.call("mf_bias_sse", _tp(self.u), _tp(self.i), _tp(self.r), self.n,
                          self.global_mean, _tp(self.bu), _tp(self.bi), self.dcode,
                          _tp(self.ws), out, self.stream)
            else:
                offs = self.eval_offs
                _lib.call("mf_sse", _tp(self.eu), _tp(self.ei), _tp(self.er), self.n,
                          self.global_mean, _tp(self.bu), _tp(self.bi), _tp(self.P),
                          _tp(self.Q), self.n_users, self.n_items, self.k, self.kcode,
                          self.dcode, self.gamma,
                          self.min_rating, self.max_rating, _np(offs),
                          0 if offs is None else len(offs) - 1, _tp(self.ws), out,
                          self.stream)

    def sse_from(self, slot: int, P, Q, bu, bi, ws, stream, max_blocks: int = 0) -> None:
        """The training SSE of the given parameter tensors (this engine's
        ratings) into slot ``slot``, launched on ``stream`` with at most
        ``max_blocks`` workgroups (mf_sse_capped; 0 = mf_sse's own grid).
        ``ws``: an SSE workspace of this engine's size (not shared with a
        concurrently running pass)."""
        self._ensure_sse_slots(slot + 1)
        out = _VOID(self.sse_buf.data_ptr() + 8 * slot)
        offs = self.eval_offs
        with torch.cuda.device(self.dev):
            _lib.call("mf_sse_capped", _tp(self.eu), _tp(self.ei), _tp(self.er), self.n,
                      self.global_mean, _tp(bu), _tp(bi), _tp(P), _tp(Q), self.n_users,
                      self.n_items, self.k, self.kcode, self.dcode, self.gamma,
                      self.min_rating, self.max_rating, _np(offs),
                      0 if offs is None else len(offs) - 1, _tp(ws), int(max_blocks), out,
                      _VOID(stream.cuda_stream))

    def sse_overlap(self, slot: int, timing: bool = False) -> None:
        """The training SSE of the current parameters into slot ``slot``,
        computed off the critical path: the parameters are copied to a device
        snapshot on the main stream (what the next epoch's sweep then
        overwrites), and mf_sse reads the snapshot on a side stream, so the
        next epoch's SGD runs while it does.  Same value as sse_async (the
        same kernel on the same parameter values); sse_values() waits for
        the side stream."""
        if self.bias_only or self.n == 0:
            self.sse_async(slot)
            return
        main = torch.cuda.current_stream(self.dev)
        ov = self._ov
        if ov is None:
            ov = self._ov = dict(side=torch.cuda.Stream(self.dev), done=None,
                                 P=torch.empty_like(self.P), Q=torch.empty_like(self.Q),
                                 bu=torch.empty_like(self.bu), bi=torch.empty_like(self.bi),
                                 ws=torch.empty_like(self.ws))
        if self.sse_buf.numel() < slot + 1:
            ov["side"].synchronize()             # no SSE writes into the old buffer
            self._ensure_sse_slots(slot + 1)
        if ov["done"] is not None:
            main.wait_event(ov["done"])          # the previous SSE has read the snapshot
        for name in ("P", "Q", "bu", "bi"):
            ov[name].copy_(getattr(self, name))
        ready = torch.cuda.Event()
        ready.record(main)
        side = ov["side"]
        side.wait_event(ready)
        if timing:                                 # (start, end) on the side stream
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record(side)
            ov.setdefault("events", []).append(ev)
        out = _VOID(self.sse_buf.data_ptr() + 8 * slot)
        offs = self.eval_offs
        with torch.cuda.device(self.dev):
            _lib.call("mf_sse", _tp(self.eu), _tp(self.ei), _tp(self.er), self.n,
                      self.global_mean, _tp(ov["bu"]), _tp(ov["bi"]), _tp(ov["P"]),
                      _tp(ov["Q"]), self.n_users, self.n_items, self.k, self.kcode,
                      self.dcode, self.gamma, self.min_rating, self.max_rating, _np(offs),
                      0 if offs is None else len(offs) - 1, _tp(ov["ws"]), out,
                      _VOID(side.cuda_stream))
        if timing:
            ov["events"][-1][1].record(side)
        done = torch.cuda.Event()
        done.record(side)
        ov["done"] = done

    def sse_join(self) -> None:
        """Make the main stream wait for an overlapped SSE (sse_overlap)."""
        if self._ov is not None and self._ov["done"] is not None:
            torch.cuda.current_stream(self.dev).wait_event(self._ov["done"])

    def sse_values(self, n_slots: int) -> np.ndarray:
        self.sse_join()
        return self.sse_buf[:n_slots].cpu().numpy().copy()

    def rmse_values(self, n_slots: int) -> list:
        if self.n == 0:
            return [float("nan")] * n_slots
        sse = self.sse_values(n_slots)
        return [float(np.sqrt(s / self.n)) for s in sse]

    def predict(self, u: np.ndarray, i: np.ndarray, bound: bool) -> np.ndarray:
        """Predictions for id pairs (-1 = unknown), float64 host array."""
        n = len(u)
        if n == 0:
            return np.empty(0, np.float64)
        ud = torch.from_numpy(np.ascontiguousarray(u, np.int32)).to(self.dev)
        idd = torch.from_numpy(np.ascontiguousarray(i, np.int32)).to(self.dev)
        out = torch.empty(n, dtype=self.tdt, device=self.dev)
        with torch.cuda.device(self.dev):
            if self.bias_only:
                _lib.call("mf_bias_predict", _tp(ud), _tp(idd), n, self.global_mean,
                          _tp(self.bu), _tp(self.bi), self.dcode, self.min_rating,
                          self.max_rating, int(bound), _tp(out), self.stream)
            else:
                _lib.call("mf_predict", _tp(ud), _tp(idd), n, self.global_mean,
                          _tp(self.bu), _tp(self.bi), _tp(self.P), _tp(self.Q), self.k,
                          self.kcode, self.dcode, self.gamma, self.min_rating,
                          self.max_rating, int(bound), _tp(out), self.stream)
        return out.cpu().numpy().astype(np.float64)

    # workspace of one top-k launch (fused path: the partial lists; two-stage
    # path, amount > 64: n_query * n_items * 8 B of keys); users beyond this
    # budget go in further launches
    topk_ws_budget = 1 << 30
    # recommend_batch through the MFMA candidate filter where supported
    # (mf_topk_mm; env MF_TOPK_MFMA=0 forces the exact kernels)
    topk_mfma = True

    def topk_prepare(self, users: np.ndarray, amount: int,
                     ex_ptr: Optional[np.ndarray] = None,
                     ex_items: Optional[np.ndarray] = None) -> dict:
        """Device-resident top-k batch: query ids, exclusion CSR (each user's
        list sorted, as the fused kernel binary-searches it), workspace and
        outputs, and the users per launch (``topk_ws_budget``)."""
        if self.bias_only:
            raise NotImplementedError("top-k is implemented for factor models")
        users = np.ascontiguousarray(users, np.int32)
        nq = len(users)
        q = {"nq": nq, "amount": int(amount)}
        if nq == 0 or amount == 0:
            return q
        to = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(self.dev)  # noqa: E731
        q["users"] = to(users)
        q["ex_ptr"] = q["ex_items"] = None
        if ex_ptr is not None:
            ex_ptr = np.ascontiguousarray(ex_ptr, np.int64)
            ex_items = np.ascontiguousarray(ex_items, np.int32)
            if len(ex_ptr) != nq + 1:
                raise ValueError("ex_ptr needs n_query + 1 offsets")
            seg = np.repeat(np.arange(nq, dtype=np.int64), np.diff(ex_ptr))
            ex_items = ex_items[np.lexsort((ex_items, seg))]
            q["ex_ptr"] = to(ex_ptr - ex_ptr[0])
            q["ex_items"] = to(ex_items if len(ex_items) else np.zeros(1, np.int32))
        lib = _lib.load()
        q["mm"] = (self.topk_mfma and os.environ.get("MF_TOPK_MFMA") != "0" and
                   bool(lib.mf_topk_mm_supported(self.k, self.kcode, self.dcode, amount)))
        self._topk_workspace(q, q["mm"])
        q["items"] = torch.empty((nq, amount), dtype=torch.int32, device=self.dev)
        q["scores"] = torch.empty((nq, amount), dtype=self.tdt, device=self.dev)
        q["ovf"] = torch.zeros(1, dtype=torch.int32, device=self.dev)
        return q

    def _topk_workspace(self, q: dict, mm: bool) -> None:
        """Users per launch (grid limits, then halved until the workspace fits
        ``topk_ws_budget``) and the workspace, for the MFMA-filter path
        (mf_topk_mm) or the exact one (mf_topk)."""
        lib = _lib.load()
        nq, amount = q["nq"], q["amount"]
        need = ((lambda c: lib.mf_topk_mm_workspace_bytes(c, self.n_items)) if mm else
                (lambda c: lib.mf_topk_workspace_bytes(c, self.n_items, amount)))
        chunk = min(nq, 65535 if amount > 64 else 1 << 20)
        while chunk > 1 and need(chunk) > self.topk_ws_budget:
            chunk = (chunk + 1) // 2
        q["chunk"] = chunk
        q["ws"] = torch.empty(max(need(chunk), 8), dtype=torch.uint8, device=self.dev)

    def topk_launch(self, q: dict, exact: bool = False) -> None:
        """Enqueue the top-k of a prepared batch (results stay on the device):
        mf_topk_mm where supported (its overflow word in q["ovf"]), else, or
        with ``exact``, mf_topk."""
        nq, amount = q["nq"], q["amount"]
        if nq == 0 or amount == 0:
            return
        mm = q["mm"] and not exact
        if not mm and q.get("mm"):
            self._topk_workspace(q, False)        # the exact path's workspace
            q["mm"] = False
        chunk = q["chunk"]
        es_i, es_s = q["items"].element_size(), q["scores"].element_size()
        if mm:
            q["ovf"].zero_()
        with torch.cuda.device(self.dev):
            for q0 in range(0, nq, chunk):
                q1 = min(nq, q0 + chunk)
                # CSR offsets stay absolute: the chunk's ptr array starts at row q0
                dp = None if q["ex_ptr"] is None else _VOID(q["ex_ptr"].data_ptr() + 8 * q0)
                users = _VOID(q["users"].data_ptr() + 4 * q0)
                items = _VOID(q["items"].data_ptr() + es_i * amount * q0)
                scores = _VOID(q["scores"].data_ptr() + es_s * amount * q0)
                if mm:
                    _lib.call("mf_topk_mm", users, q1 - q0, self.global_mean, _tp(self.bu),
                              _tp(self.bi), _tp(self.P), _tp(self.Q), self.n_items, self.k,
                              self.kcode, self.dcode, dp, _tp(q["ex_items"]), amount,
                              _tp(q["ws"]), items, scores, _tp(q["ovf"]), self.stream)
                else:
                    _lib.call("mf_topk", users, q1 - q0,
                              self.global_mean, _tp(self.bu), _tp(self.bi), _tp(self.P),
                              _tp(self.Q), self.n_items, self.k, self.kcode, self.dcode,
                              self.gamma, self.min_rating, self.max_rating, dp,
                              _tp(q["ex_items"]), amount, _tp(q["ws"]), items, scores,
                              self.stream)

    def topk_finish(self, q: dict) -> bool:
        """After topk_launch: if the MFMA filter overflowed, re-run the exact
        path (synchronises).  Returns whether it had to."""
        if not q.get("mm") or q["nq"] == 0 or q["amount"] == 0:
            return False
        if int(q["ovf"].item()) == 0:
            return False
        self.topk_launch(q, exact=True)
        return True

    def topk(self, users: np.ndarray, amount: int, ex_ptr: Optional[np.ndarray] = None,
             ex_items: Optional[np.ndarray] = None) -> Tuple[np.ndarray, np.ndarray]:
        """Best ``amount`` items per internal user id: (item ids, scores).

        ``ex_ptr`` / ``ex_items``: optional CSR exclusions (query q skips
        items ex_items[ex_ptr[q]:ex_ptr[q+1]])."""
        q = self.topk_prepare(users, amount, ex_ptr, ex_items)
        if q["nq"] == 0 or amount == 0:
            return (np.full((q["nq"], amount), -1, np.int32),
                    np.full((q["nq"], amount), np.nan, np.float64))
        self.topk_launch(q)
        self.topk_finish(q)
        return q["items"].cpu().numpy(), q["scores"].cpu().numpy().astype(np.float64)


class BiasALS:
    """CSR lists for the bias-model ALS (baseline_model.py:313-348)."""

    def __init__(self, engine: SGDEngine):
        e = engine
        n = e.n

        def csr(ids, m):
            cnt = np.bincount(ids, minlength=m).astype(np.int64)
            ptr = np.zeros(m + 1, np.int64)
            np.cumsum(cnt, out=ptr[1:])
            lst = np.argsort(ids, kind="stable").astype(np.int32)   # row order kept
            return ptr, lst

        up, ul = csr(e.u_host, e.n_users) if n else (np.zeros(e.n_users + 1, np.int64), np.zeros(0, np.int32))
        ip, il = csr(e.i_host, e.n_items) if n else (np.zeros(e.n_items + 1, np.int64), np.zeros(0, np.int32))
        to = lambda a: torch.from_numpy(a).to(e.dev)  # noqa: E731
        self.e = e
        self.up, self.ul, self.ip, self.il = to(up), to(ul), to(ip), to(il)

    def epoch(self, reg: float) -> None:
        e = self.e
        with torch.cuda.device(e.dev):
            _lib.call("mf_bias_als_epoch", _tp(e.u), _tp(e.i), _tp(e.r), e.global_mean,
                      _tp(e.bu), _tp(e.bi), e.n_users, e.n_items, _tp(self.up),
                      _tp(self.ul), _tp(self.ip), _tp(self.il), e.dcode, float(reg),
                      e.stream)


class FactorALS:
    """Alternating least squares for the factor model (BASELINE config 5;
    mf_als_sweep): CSR lists by user and by item in HBM, one half-sweep per
    side.  Extends the bias ALS (baseline_model.py:283-362) to the latent
    factors; the engine must hold float32 linear-kernel parameters."""

    def __init__(self, engine: SGDEngine):
        e = engine
        if e.dtype != "float32" or e.kernel != "linear":
            raise ValueError("factor ALS runs on float32 linear-kernel parameters")
        kmax = _lib.load().mf_als_max_factors()
        if not 1 <= e.k <= kmax:
            raise ValueError(f"factor ALS needs 1 <= n_factors <= {kmax}, got {e.k}")
        r = e.r_host.astype(np.float32)

        def csr(ent, oth, m):
            order = np.argsort(ent, kind="stable")
            ptr = np.zeros(m + 1, np.int64)
            np.cumsum(np.bincount(ent, minlength=m), out=ptr[1:])
            to = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(e.dev)  # noqa: E731
            return to(ptr), to(oth[order].astype(np.int32)), to(r[order])

        self.e = e
        self.user_csr = csr(e.u_host, e.i_host, e.n_users)
        self.item_csr = csr(e.i_host, e.u_host, e.n_items)

    def _sweep(self, csr, n, ob, oq, b, q, reg):
        e = self.e
        ptr, oth, rr = csr
        with torch.cuda.device(e.dev):
            _lib.call("mf_als_sweep", _tp(ptr), _tp(oth), _tp(rr), n, e.global_mean, _tp(ob),
                      _tp(oq), _tp(b), _tp(q), e.k, e.dcode, float(reg), e.stream)

    def sweep_users(self, reg: float) -> None:
        """User rows and biases from the current item side."""
        e = self.e
        self._sweep(self.user_csr, e.n_users, e.bi, e.Q, e.bu, e.P, reg)

    def sweep_items(self, reg: float) -> None:
        """Item rows and biases from the current user side."""
        e = self.e
        self._sweep(self.item_csr, e.n_items, e.bu, e.P, e.bi, e.Q, reg)

    def epoch(self, reg: float) -> None:
        """Users, then items (the order of baseline_model.py:326-348)."""
        self.sweep_users(reg)
        self.sweep_items(reg)


class _ErrorPoll:
    """Non-blocking look at the persistent sweep's sticky error word: after
    each epoch's launch a copy of the word goes to pinned host memory behind
    an event; ``failed()`` reads the copy only once that event has completed
    (never waits), so a failure in epoch e is seen a few epochs later at most
    instead of at the end of the fit, and no further persistent launches run
    on the uneven position counters a failed sweep leaves."""

    def __init__(self, engine: SGDEngine):
        self.e = engine
        self.host = torch.zeros(1, dtype=torch.int32, pin_memory=True)
        self.ev = None

    def post(self) -> None:
        ws = getattr(self.e, "_strata_ws", None)
        if ws is None or self.ev is not None and not self.ev.query():
            return                                # the last copy is still in flight
        B = self.e.strata.B
        # the copy and its event on the ENGINE's stream (its device's current
        # stream), not the current device's: the engine may live on another
        # device than the caller's current one
        with torch.cuda.device(self.e.dev):
            self.host.copy_(ws[B:B + 1], non_blocking=True)
            self.ev = torch.cuda.Event()
            self.ev.record(torch.cuda.current_stream(self.e.dev))

    def failed(self) -> bool:
        return self.ev is not None and self.ev.query() and int(self.host[0]) != 0


# the exact schedule pipelines its per-epoch shuffle from this many ratings
EXACT_PIPELINE_MIN = 1 << 20
# ... and applies the shuffle's swaps on the GPU from this many
EXACT_GPU_SHUFFLE_MIN = 1 << 22


class ExactShuffler:
    """``np.random.shuffle`` of the exact schedule's 32-bit visit order (the
    reference's per-epoch shuffle, kernel_matrix_factorization.py:371) with
    the draws on the calling thread (mf_legacy_shuffle_draws: the RandomState
    advanced as by the shuffle) and the swaps on the GPU
    (mf_shuffle_swaps_device, rounds of deterministic reservations) on a
    stream of its own, except the last ones (positions below TAIL), applied
    on the host after the read-back -- the same order as NumPy's, bit for bit.
    One host thread made the whole shuffle the exact epoch's bound at C3
    (0.24 s).  The device keeps the order it produced,
    so a call on the previous call's result uploads nothing; the result
    arrays are two pinned buffers used in turn (a result stays valid until
    the second call after it)."""

    TAIL = 1 << 20

    def __init__(self, n: int, dev):
        lib = _lib.load()
        self.n, self.dev = int(n), dev
        self.total = max(self.n - 1, 0)
        # swaps d < d_end have i = total - d >= TAIL; the rest touch [0, TAIL)
        self.d_end = max(0, self.total - self.TAIL + 1)
        m = max(self.total, 1)
        with torch.cuda.device(dev):
            self.tgt_h = torch.empty(m, dtype=torch.int32, pin_memory=True)
            self.tgt_d = torch.empty(m, dtype=torch.int32, device=dev)
            self.res = torch.zeros(max(self.n, 1), dtype=torch.int64, device=dev)
            wsb = int(lib.mf_shuffle_swaps_workspace_bytes(self.n))
            self.ws = torch.empty((wsb + 7) // 8, dtype=torch.int64, device=dev)
            self.ord_d = [torch.empty(max(self.n, 1), dtype=torch.int32, device=dev)
                          for _ in range(2)]
            self.ord_h = [torch.empty(max(self.n, 1), dtype=torch.int32, pin_memory=True)
                          for _ in range(2)]
            self.stream = torch.cuda.Stream(dev)
        self.tag = ctypes.c_uint64(1)
        self.cur = None                  # ord_d / ord_h index of the last result
        self.last = None                 # ... that result (the host array returned)

    def shuffle_from(self, src: np.ndarray) -> np.ndarray:
        """shuffle(copy of src): a new array, src untouched."""
        n = self.n
        if len(src) != n or src.dtype != np.int32:
            raise ValueError("src must hold n int32 entries")
        o = 0 if self.cur != 0 else 1
        tgt = self.tgt_h.numpy().view(np.uint32)
        _prep.legacy_shuffle_draws(n, tgt)
        dst_h = self.ord_h[o].numpy()[:n]
        with torch.cuda.device(self.dev), torch.cuda.stream(self.stream):
            if self.cur is not None and src is self.last:
                base = self.ord_d[self.cur]
            else:                        # an order this shuffler did not make
                base = self.ord_d[o]
                base[:n].copy_(torch.from_numpy(src), non_blocking=False)
            dst = self.ord_d[o]
            if base is not dst:
                dst[:n].copy_(base[:n])
            if self.d_end > 0:
                if self.tag.value > (1 << 30):   # the tags' room: start over
                    self.res.zero_()
                    self.tag.value = 1
                self.tgt_d[: self.total].copy_(self.tgt_h[: self.total], non_blocking=True)
                _lib.call("mf_shuffle_swaps_device", _tp(self.tgt_d), n, self.d_end, _tp(dst),
                          _tp(self.res), _tp(self.ws), ctypes.byref(self.tag),
                          _VOID(self.stream.cuda_stream))
            self.ord_h[o][:n].copy_(dst[:n], non_blocking=True)
            self.stream.synchronize()
            _prep.apply_swaps_i32(tgt, n, self.d_end, dst_h)
            if self.d_end > 0:           # the host's swaps back to the device copy
                t = min(self.TAIL, n)
                dst[:t].copy_(self.ord_h[o][:t], non_blocking=True)
        self.cur, self.last = o, dst_h
        return dst_h


def legacy_permutation_device(n: int, dev) -> np.ndarray:
    """``np.random.permutation(n)`` (int64) with the shuffle's swaps on the
    GPU (ExactShuffler's split, one shot: the draws here, the swaps by
    mf_shuffle_swaps_device on arange(n) on the device, the last ones on
    the host) -- fit()'s ``X.sample(frac=1)`` draw at 10^8 rows, 0.35 s of
    one host thread before.  Same permutation and RandomState as NumPy."""
    lib = _lib.load()
    n = int(n)
    if not 0 < n < (1 << 31):
        raise ValueError("legacy_permutation_device: 0 < n < 2^31")
    total = n - 1
    d_end = max(0, total - ExactShuffler.TAIL + 1)
    tgt = np.empty(max(total, 1), np.uint32)
    _prep.legacy_shuffle_draws(n, tgt)
    with torch.cuda.device(dev):
        stream = torch.cuda.current_stream(dev)
        data = torch.arange(n, dtype=torch.int32, device=dev)
        if d_end > 0:
            tgt_d = torch.from_numpy(tgt.view(np.int32)).to(dev)
            res = torch.zeros(n, dtype=torch.int64, device=dev)
            wsb = int(lib.mf_shuffle_swaps_workspace_bytes(n))
            ws = torch.empty((wsb + 7) // 8, dtype=torch.int64, device=dev)
            _lib.call("mf_shuffle_swaps_device", _tp(tgt_d), n, d_end, _tp(data), _tp(res),
                      _tp(ws), ctypes.byref(ctypes.c_uint64(1)), _VOID(stream.cuda_stream))
            del tgt_d, res, ws
        head = data[: n - d_end].cpu().numpy()            # the swaps left touch these
        _prep.apply_swaps_i32(tgt, n, d_end, head)
        data[: n - d_end].copy_(torch.from_numpy(head))
        return data.to(torch.int64).cpu().numpy()


def exact_shuffler(engine: "SGDEngine"):
    """The engine's ExactShuffler when its ratings are many enough and it is
    on a GPU (env MF_EXACT_GPU_SHUFFLE=0: none, the host shuffle)."""
    if (engine.n < EXACT_GPU_SHUFFLE_MIN or engine.dev.type != "cuda"
            or os.environ.get("MF_EXACT_GPU_SHUFFLE") == "0"):
        return None
    sh = getattr(engine, "_exact_shuffler", None)
    if sh is None or sh.n != engine.n:
        sh = engine._exact_shuffler = ExactShuffler(engine.n, engine.dev)
    return sh


def fit_epochs(engine: SGDEngine, n_epochs: int, schedule: str, lr: float,
               reg: float, update_user: bool = True, update_item: bool = True,
               verbose: int = 0, rng_order: Optional[np.ndarray] = None,
               on_epoch=None) -> list:
    """Run ``n_epochs`` of SGD + training-RMSE exactly as ``_sgd`` does
    (kernel_matrix_factorization.py:367-445).  Returns train_rmse (list).

    exact:   draws ``np.random.shuffle`` on the row order every epoch
             (the reference's RNG stream, :371);
    colored: draws ``np.random.permutation(n_colours)`` every epoch;
    strata:  draws the stratum order (``stratum_order``: np.random.permutation(B)
             for the plain plan) and a 32-bit colour-rotation seed every
             epoch.

    Strata epochs run back to back with no host synchronisation: the
    persistent sweep's error word is sticky, so it is read only where the
    host waits anyway (the per-epoch RMSE print with ``verbose``, or the
    RMSE read-back at the end).  If a workgroup gave up waiting (workgroups
    not co-resident, e.g. another process holding CUs), the parameters are
    restored from the one snapshot taken before epoch 1 and every epoch so
    far is replayed with the same draws as one launch per stratum -- the
    same sequential orders, hence the same result (RuntimeWarning).
    """
    exact_next = None
    if schedule == "exact":
        # the row order as 32-bit indices (np.random.shuffle's draws depend on
        # the length only): half the bytes per swap, and the chunked level
        # builder's input
        narrow = engine.n < (1 << 31)
        dt = np.int32 if narrow else np.int64
        order = (np.arange(engine.n, dtype=dt) if rng_order is None
                 else np.array(rng_order, dtype=dt))
        # epoch e+1's shuffle is drawn on a worker thread while epoch e's
        # levels are built and launched ("exact schedule
        # at scale"); nothing else draws from the global RandomState inside
        # the loop, so the draws are the reference's in the reference's
        # order.  Joined before the end of every epoch; off with an on_epoch
        # callback (it might draw) and for n >= 2^31.
        pipeline = narrow and on_epoch is None and engine.n >= EXACT_PIPELINE_MIN
        if pipeline:
            exact_pool = ThreadPoolExecutor(1)
            exact_spare = np.empty_like(order)
            shuffler = exact_shuffler(engine)

            def shuffled_copy(src, dst):
                if shuffler is not None:          # the swaps on the GPU
                    return shuffler.shuffle_from(src)
                # (torch's CPU copy is threaded: 400 MB at C3 in ~10 ms
                # instead of np.copyto's ~40 ms on the worker's critical path)
                torch.from_numpy(dst).copy_(torch.from_numpy(src))
                _prep.legacy_shuffle_(dst)
                return dst
    elif schedule == "colored":
        if engine.colored is None:
            engine.prepare_colored()
        nb = len(engine.colored) - 1
    elif schedule == "strata":
        if engine.strata is None:
            engine.prepare_strata()
    else:
        raise ValueError(f"schedule must be 'exact', 'colored' or 'strata', got {schedule!r}")
    train_rmse = []
    draws = []                                    # strata: (seq, seed) per epoch
    persistent = None                             # strata: the engine's default
    snap0 = None
    poll = None
    if schedule == "strata" and engine.strata_persistent:
        snap0 = engine.snapshot_params()          # once: the replay's starting point
        poll = _ErrorPoll(engine)

    def replay_failed(upto: int) -> None:
        """Epochs 0..upto-1 again from snap0 as per-stratum launches."""
        nonlocal persistent
        warnings.warn(f"the persistent strata sweep could not complete within epochs 1-{upto} "
                      "(workgroups not co-resident); replayed them with the same draws as one "
                      "launch per stratum", RuntimeWarning, stacklevel=3)
        persistent = False
        engine.restore_params(snap0)
        engine.clear_strata_error()
        for ep, (sq, sd) in enumerate(draws[:upto]):
            engine.epoch_strata(sq, sd, lr, reg, update_user, update_item, persistent=False)
            engine.sse_async(ep)

    try:
        for epoch in range(n_epochs):
            if poll is not None and persistent is None and poll.failed():
                replay_failed(epoch)                  # stop launching persistent sweeps now
            if schedule == "exact":
                if exact_next is not None:            # drawn during the last epoch
                    spare, order = order, exact_next.result()
                    exact_spare, exact_next = spare, None
                else:
                    _prep.legacy_shuffle_(order)      # = np.random.shuffle(order)
                if pipeline and epoch + 1 < n_epochs:
                    exact_next = exact_pool.submit(shuffled_copy, order, exact_spare)
                try:
                    engine.epoch_exact(order, lr, reg, update_user, update_item)
                finally:
                    if exact_next is not None:
                        exact_next.exception()        # joined: RNG consistent at the epoch end
            elif schedule == "colored":
                seq = np.random.permutation(nb).astype(np.int32)
                engine.epoch_colored(seq, lr, reg, update_user, update_item)
            else:
                seq = stratum_order(np.random, engine.strata)
                seed = int(np.random.randint(0, 2**31 - 1))
                draws.append((seq, seed))
                engine.epoch_strata(seq, seed, lr, reg, update_user, update_item,
                                    persistent=persistent)
                if poll is not None and persistent is None:
                    poll.post()
            engine.sse_async(epoch)
            if verbose == 1:
                if snap0 is not None and persistent is None and engine.strata_failed():
                    replay_failed(epoch + 1)
                rmse = engine.rmse_values(epoch + 1)[epoch]
                train_rmse.append(rmse)
                print("Epoch ", epoch + 1, "/", n_epochs, " -  train_rmse:", rmse)
            if on_epoch is not None:
                on_epoch(epoch)
    finally:
        # also on an exception mid-fit: the worker is joined and dropped (a
        # fit aborted in the exact schedule leaves the global RandomState
        # one shuffle past the reference's: epoch e+1's was already drawn)
        if schedule == "exact" and pipeline:
            exact_pool.shutdown(wait=True, cancel_futures=True)
    if snap0 is not None and persistent is None and engine.strata_failed():
        replay_failed(n_epochs)
        if verbose == 1:
            train_rmse = engine.rmse_values(n_epochs)
    if verbose != 1:
        train_rmse = engine.rmse_values(n_epochs)
    return train_rmse

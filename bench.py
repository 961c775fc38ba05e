#!/usr/bin/env python
"""bench.py -- KernelMF SGD throughput on MI355X (BASELINE.json headline).

Workload (BASELINE.json configs[2], the HBM-roofline headline): synthetic
1M users x 100K items, 100M unique ratings (1..5 drawn from the ML-100K
histogram), rank-64 linear-kernel SGD, lr=0.01, reg=0.02, init N(0, 0.1),
FP32 parameters, strata schedule (B x B user/item blocks, item slabs in LDS,
user-owned rating slots; --schedule colored: one launch per edge colour).
With --gpus N the same 100M ratings are user-sharded over N ranks
(configs[3]; total work fixed).

One step = one epoch exactly as the reference's `_sgd` runs it
(kernel_matrix_factorization.py:369-443): the SGD sweep over every rating
plus the training-RMSE pass.  value = ratings * steps / wall time of the
timed steps (inputs resident in HBM, max over ranks).

Also reported (rank 0):
  roofline      SGD-kernel algorithmic HBM bytes / SGD-phase time (one
                hipEvent pair around each timed epoch's launches) against
                8 TB/s.  Algorithmic bytes: SURVEY 8(d)'s 16k+28 B per update
                for the colored kernel; for strata the part of it that must
                cross HBM (user row + triple + user bias per update, the item
                slab per stratum; item rows live in LDS), with the 16k+28 B
                equivalent rate reported beside it.  `traffic` = measured HBM
                bytes per launch from rocprofv3 PMC (profiles/) or null;
  cpu_baseline  the CPU oracle (FP64 C port of the reference loop, 1 core)
                timed on one full epoch (SGD sweep + RMSE pass) of the same
                workload, with the host's CPU model and nproc;
  parity        from the same initial state, after one full epoch: GPU
                (FP32) vs oracle (FP64) in the GPU's serialised order, and the
                oracle in the GPU's order vs the oracle in the reference's own
                np.random.shuffle order, next to the reference's own
                shuffle-seed spread (two shuffle seeds) -- see cpu_leg().
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "matrix-factorization_amd"))

METRIC = "rating-updates/s + final RMSE, rank-64 SGD, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0
ML100K_HIST = np.array([6110, 11370, 27145, 34174, 21201], np.float64)

WORKLOADS = {
    # name: (n_users, n_items, nnz, k, kernel, description)
    "c3": (1_000_000, 100_000, 100_000_000, 64, "linear",
           "synthetic 1Mx100K 100M-nnz rank-64 linear SGD"),
    "c2": (100_000, 10_000, 5_000_000, 32, "sigmoid",
           "synthetic 100Kx10K 5M-nnz rank-32 sigmoid SGD"),
    "small": (100_000, 20_000, 4_000_000, 64, "linear",
              "synthetic 100Kx20K 4M-nnz rank-64 linear SGD (smoke)"),
    "c5": (1_000_000, 100_000, 100_000_000, 128, "als",
           "synthetic 1Mx100K 100M-nnz rank-128 ALS (MFMA Gramian)"),
    "c5_small": (100_000, 10_000, 5_000_000, 128, "als",
                 "synthetic 100Kx10K 5M-nnz rank-128 ALS (smoke)"),
    # probes (not bench lines): one rank's share of C3 at N = 2 / 4 / 8
    # (users sharded), to see the per-GPU epoch of the strong-scaling runs
    "c3_shard2": (500_000, 100_000, 50_000_000, 64, "linear",
                  "probe: C3 user shard at N=2 (500Kx100K 50M-nnz rank-64 linear SGD)"),
    "c3_shard4": (250_000, 100_000, 25_000_000, 64, "linear",
                  "probe: C3 user shard at N=4 (250Kx100K 25M-nnz rank-64 linear SGD)"),
    "c3_shard8": (125_000, 100_000, 12_500_000, 64, "linear",
                  "probe: C3 user shard at N=8 (125Kx100K 12.5M-nnz rank-64 linear SGD)"),
    # recommend_batch (mf_topk) on the C3 model
    "topk": (1_000_000, 100_000, 100_000_000, 64, "topk",
             "C3-shaped model (1Mx100K, rank 64): top-10 of all 100K items for 10K users, "
             "items_known excluded (recommend_batch / mf_topk)"),
    # probes (not bench lines): P that fits the 256 MiB Infinity Cache
    "c3_u250k": (250_000, 100_000, 100_000_000, 64, "linear",
                 "probe: synthetic 250Kx100K 100M-nnz rank-64 linear SGD"),
}


def record_maps_at_exit() -> None:
    """With MF_MAPS_DIR set (tools/gpu.sh sets it per step): this process's
    library map, written by a Python atexit hook -- the last Python code
    before the C exit handlers (HIP's fat-binary unregistration of each
    code object, torch's allocator teardown, rocprofv3's tool finalisation)
    run, so the PCs of a fault there (the r05n abort)
    can be matched to a library.  tools/gpu.sh deletes the file when the
    step exits 0."""
    d = os.environ.get("MF_MAPS_DIR")
    if not d:
        return
    import atexit

    def dump():
        try:
            os.makedirs(d, exist_ok=True)
            with open("/proc/self/maps") as f, open(os.path.join(d, f"maps.{os.getpid()}.txt"),
                                                     "w") as g:
                g.write(f.read())
        except OSError:
            pass

    atexit.register(dump)


def log(msg: str) -> None:
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def synth(n_users: int, n_items: int, nnz: int, seed: int = 20261015):
    """nnz unique (user, item) pairs, uniform; ratings from the ML-100K
    histogram (recommender-evaluation.ipynb:98-102 of the reference)."""
    rs = np.random.RandomState(seed)
    extra = max(1000, int(nnz * 2e-3))
    keys = rs.randint(0, n_users * n_items, size=nnz + extra, dtype=np.int64)
    keys = np.unique(keys)
    while len(keys) < nnz:   # top up (never needed at these densities)
        more = rs.randint(0, n_users * n_items, size=nnz - len(keys) + extra, dtype=np.int64)
        keys = np.unique(np.concatenate([keys, more]))
    keep = np.sort(rs.choice(len(keys), nnz, replace=False)) if len(keys) > nnz else None
    if keep is not None:
        keys = keys[keep]
    keys = keys[rs.permutation(nnz)]
    u = (keys // n_items).astype(np.int32)
    i = (keys % n_items).astype(np.int32)
    del keys
    p = ML100K_HIST / ML100K_HIST.sum()
    r = (rs.choice(5, size=nnz, p=p) + 1).astype(np.float32)
    return u, i, r


def traffic_from_profiles(workload: str, n_gpus: int, schedule: str, dtype: str,
                          kernel: str, emulate: int = 0):
    """HBM bytes per SGD launch measured by rocprofv3 PMC passes for exactly
    this workload, schedule, dtype, kernel and world size, if committed under
    profiles/traffic.json; else None (the line then says `traffic: null`
    rather than borrowing another configuration's counters).  ``emulate``
    (one GPU running rank 0 of an N-rank rotation, --emulate-rank N): the
    key is ``emu{N}``, never the N = 1 run's ``n1`` -- the emulated sub-epochs
    are other launches on other plans."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        world = f"emu{emulate}" if emulate > 1 else f"n{n_gpus}"
        e = d.get(f"{workload}/{schedule}/{dtype}/{world}")
        if e is None or e.get("kernel") != kernel:
            return None
        return float(e["hbm_bytes_per_sgd_launch"])
    except (OSError, ValueError, KeyError, AttributeError):
        return None


MFMA_F32_PEAK_TFS = 157.3      # MI355X dense f32-input MFMA (MI355X_MICROARCH.md)


def run_als(args, u, i, r, nu, ni, nnz, k, desc, mu, P0, Q0, dev) -> int:
    """BASELINE configs[4]: rank-k factor ALS (mf_als_sweep), one step = one
    epoch = user half-sweep + item half-sweep + training-RMSE pass.

    roofline: MFMA-bound.  Algorithmic flops per epoch: the
    Gramian 2k^2 and the right-hand side 2k per rating per half-sweep, plus
    k^3/3 per solved entity; achieved = those flops / ALS-kernel time."""
    import torch

    from matrix_factorization.engine import FactorALS, SGDEngine

    if args.dtype != "float32":
        raise SystemExit("the ALS path is float32 (f32-input MFMA Gramian)")
    reg = 1.0 if args.reg is None else args.reg
    eng = SGDEngine(u, i, r, nu, ni, k, "linear", "float32", dev, min_rating=1.0,
                    max_rating=5.0, global_mean=mu)
    t0 = time.time()
    als = FactorALS(eng)
    log(f"ALS CSR lists in {time.time() - t0:.1f}s")

    def reset():
        eng.load_params(P=P0, Q=Q0, bu=np.zeros(nu), bi=np.zeros(ni))

    # ---- CPU baseline + parity: the user half-sweep for a prefix of users
    cpu_baseline = parity = None
    if args.cpu_sample != 0:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle  # test infrastructure: checker and reported baseline only

        deg = np.bincount(u, minlength=nu)
        want = 1_000_000 if args.cpu_sample < 0 else min(args.cpu_sample, 1_000_000)
        n_s = int(np.searchsorted(np.cumsum(deg), min(want, nnz))) + 1
        n_s = min(n_s, nu)
        sel = u < n_s
        reset()
        als.sweep_users(reg)
        Pg, _, bug, _ = eng.params_numpy()
        S = int(sel.sum())
        log(f"cpu oracle: user half-sweep of {n_s} users = {S} ratings, FP64, 1 thread")
        from threadpoolctl import threadpool_limits

        with threadpool_limits(1), pinned_core() as core:   # one core, as the SGD leg
            t0 = time.perf_counter()
            bo, Po = oracle.als_half_sweep(u[sel], i[sel], r[sel], np.float32(mu),
                                           np.zeros(ni), Q0, n_s, reg)
            t_cpu = time.perf_counter() - t0
        cpu_baseline = {
            "value": S / t_cpu / 2, "unit": "rating-updates/s", "cores": 1, "kind": "port",
            "affinity": core,
            "sample": (f"user half-sweep of the first {n_s} users ({S} ratings, {t_cpu:.1f}s) "
                       f"of the same workload, oracle.als_half_sweep (NumPy FP64, "
                       f"np.linalg.solve per user); value = ratings / (2 x time), an "
                       f"epoch being two half-sweeps"),
        }
        rel = np.abs(Pg[:n_s] - Po) / np.maximum(1.0, np.abs(Po))
        parity = {"what": "user half-sweep from the same state, GPU f32 MFMA vs oracle f64",
                  "max_rel_dP": float(rel.max()),
                  "max_abs_dbu": float(np.max(np.abs(bug[:n_s] - bo)))}
        log(f"cpu {cpu_baseline['value'] / 1e6:.3f} M/s; parity max rel dP "
            f"{parity['max_rel_dP']:.2e}")

    reset()
    events = []

    def epoch(ep, timed):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)] if timed else None
        if ev:
            ev[0].record()
        als.sweep_users(reg)
        if ev:
            ev[1].record()
        als.sweep_items(reg)
        if ev:
            ev[2].record()
        eng.sse_async(ep)
        if ev:
            ev[3].record()
            events.append(ev)

    for ep in range(args.warmup):
        epoch(ep, False)
        log(f"warmup epoch {ep + 1}/{args.warmup}")
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for j in range(args.steps):
        epoch(args.warmup + j, not args.no_phase_timing)
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    rmse = eng.rmse_values(args.warmup + args.steps)
    roofline = phases = None
    if events:
        us = sum(e[0].elapsed_time(e[1]) for e in events) / 1e3
        it = sum(e[1].elapsed_time(e[2]) for e in events) / 1e3
        ss = sum(e[2].elapsed_time(e[3]) for e in events) / 1e3
        flops_epoch = 2 * nnz * (2 * k * k + 2 * k) + (nu + ni) * k ** 3 / 3
        achieved = flops_epoch * len(events) / (us + it) / 1e12
        roofline = {"bound": "mfma", "achieved": achieved, "peak": MFMA_F32_PEAK_TFS,
                    "unit": "TFLOP/s", "frac": achieved / MFMA_F32_PEAK_TFS, "traffic": None,
                    "kernel": "k_als_solve", "launches": 2 * len(events),
                    "avg_launch_us": (us + it) / (2 * len(events)) * 1e6,
                    "flops_per_epoch": flops_epoch,
                    "note": "f32-input MFMA peak (no xf32 on gfx950); flops = 2k^2 + 2k "
                            "per rating per half-sweep + k^3/3 per entity"}
        phases = {"user_sweep_ms": us / len(events) * 1e3,
                  "item_sweep_ms": it / len(events) * 1e3,
                  "rmse_ms": ss / len(events) * 1e3}
    out = {
        "metric": METRIC, "value": nnz * args.steps / elapsed, "unit": "rating-updates/s",
        "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
        "config": {"workload": desc, "n_users": nu, "n_items": ni, "nnz": nnz,
                   "n_factors": k, "reg": reg, "parallelism": "single GPU",
                   "step": "one ALS epoch: user half-sweep + item half-sweep + training RMSE"},
        "final_rmse": rmse[-1], "rmse_per_epoch": rmse, "roofline": roofline,
        "phases": phases, "cpu_baseline": cpu_baseline, "parity": parity,
        "launch": _launch_label(),
    }
    print(json.dumps(out), flush=True)
    return 0


def run_topk(args, u, i, r, nu, ni, nnz, k, desc, mu, P0, Q0, dev) -> int:
    """recommend() for many users at C3 scale.  One step =
    one recommend_batch pass: the top-10 of all n_items for 10K query users
    with their rated items excluded (recommender_base.py:214-271 per user),
    engine.topk_launch with the query ids and the exclusion CSR resident in
    HBM and the results left there: mf_topk_mm (MFMA candidate filter +
    exact rescoring) where supported, else mf_topk.

    value = scores/s (query users x items per second).  roofline: MFMA at
    2k flops per score for the MFMA filter, else HBM at 4k B per score (the
    item row each score reads when nothing is reused)."""
    import torch

    from matrix_factorization.engine import SGDEngine

    n_query, amount = 10_000, 10
    rs = np.random.RandomState(3)
    users = np.sort(rs.choice(nu, n_query, replace=False)).astype(np.int32)
    sel = np.isin(u, users)
    qpos = np.searchsorted(users, u[sel])
    order = np.argsort(qpos, kind="stable")
    ex_items = i[sel][order].astype(np.int32)
    ex_ptr = np.concatenate([[0], np.cumsum(np.bincount(qpos, minlength=n_query))]).astype(np.int64)
    bu0 = rs.normal(0, 0.1, nu)
    bi0 = rs.normal(0, 0.1, ni)
    eng = SGDEngine(np.zeros(0, np.int32), np.zeros(0, np.int32), np.zeros(0), nu, ni, k,
                    "linear", args.dtype, dev, min_rating=1.0, max_rating=5.0, global_mean=mu)
    eng.load_params(P0, Q0, bu0, bi0)
    cpu_baseline = parity = None
    if args.cpu_sample != 0:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle  # test infrastructure: checker and reported baseline only

        ns = 20
        P64, Q64 = P0.astype(np.float64), Q0.astype(np.float64)
        allq = np.arange(ni, dtype=np.int32)
        ref = []
        with pinned_core() as core:
            t0 = time.perf_counter()
            for q in range(ns):
                # recommend(): predict(bound_ratings=False) of every candidate item,
                # sort descending (stable: lower item id first among equal scores)
                pred = oracle.predict(np.full(ni, users[q], np.int32), allq, mu, bu0, bi0, P64,
                                      Q64, min_rating=1.0, max_rating=5.0, bound=False)
                pred[ex_items[ex_ptr[q]:ex_ptr[q + 1]]] = -np.inf
                ref.append(np.argsort(-pred, kind="stable")[:amount])
            t_cpu = time.perf_counter() - t0
        cpu_baseline = {"value": ns * ni / t_cpu, "unit": "scores/s", "cores": 1, "kind": "port",
                        "affinity": core,
                        "sample": f"{ns} of the query users: oracle.predict of all {ni} items "
                                  f"(FP64 C restatement of _predict) + stable argsort, one thread",
                        **host_info()}
        got, _ = eng.topk(users[:ns], amount, ex_ptr[:ns + 1], ex_items[:ex_ptr[ns]])
        parity = {"what": f"top-{amount} item ids of {ns} users, GPU ({args.dtype}) vs oracle FP64",
                  "ids_equal": bool(np.array_equal(got, np.asarray(ref)))}
        log(f"cpu {cpu_baseline['value'] / 1e6:.2f} M scores/s; parity {parity}")
    # inputs resident in HBM (query ids, sorted exclusion CSR), results left
    # on the device: the timed region is the mf_topk launches
    batch = eng.topk_prepare(users, amount, ex_ptr, ex_items)
    for _ in range(args.warmup):
        eng.topk_launch(batch)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        eng.topk_launch(batch)
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    mm = bool(batch["mm"])
    fallback = eng.topk_finish(batch)      # an overflowed filter re-runs exactly (untimed)
    if mm:
        # the whole batch against the exact kernels (untimed): same ids, same scores
        got_i, got_s = batch["items"].clone(), batch["scores"].clone()
        eng.topk_launch(batch, exact=True)
        same = (torch.equal(got_i, batch["items"]) and
                torch.equal(torch.nan_to_num(got_s, nan=-7.0),
                            torch.nan_to_num(batch["scores"], nan=-7.0)))
        parity = dict(parity or {})
        parity["mfma_filter_equals_exact"] = {"users": n_query, "ids_and_scores_equal": bool(same),
                                              "overflow_fallback": bool(fallback)}
    scores = n_query * ni * args.steps
    ts = 4 if args.dtype == "float32" else 8
    achieved = scores * k * ts / elapsed / 1e9
    mmk = "k_topk_mw" if amount <= 16 and os.environ.get("MF_TOPK_MW") != "0" else "k_topk_mm"
    path = (f"MFMA filter ({mmk}{' bf16 hi/lo' if mmk == 'k_topk_mw' and os.environ.get('MF_TOPK_BF16') != '0' else ''}"
            f" + k_topk_mm_merge, exact rescoring)" if mm else
            "two-stage (keys in HBM)" if os.environ.get("MF_TOPK_TWO_STAGE") == "1"
            else "fused (k_topk_fused + k_topk_merge)")
    bf16 = mmk == "k_topk_mw" and os.environ.get("MF_TOPK_BF16") != "0" and \
        os.environ.get("MF_TOPK_MM_PIPE") != "0"
    if mm and bf16:
        # k_topk_mw<.., BF>: three bf16 32x32x16 MFMAs (lo x hi, hi x lo,
        # hi x hi) per 16 columns, so 3 x 2k executed flops per score against
        # the dense bf16 peak; f32_equivalent = the 2k algorithmic flops
        # against the f32 MFMA peak (the round-4 form's roofline)
        tf = scores * 2 * k / elapsed / 1e12
        roof = {"bound": "mfma", "achieved": 3 * tf, "peak": 2500.0, "unit": "TFLOP/s",
                "frac": 3 * tf / 2500.0, "traffic": None, "kernel": mmk,
                "f32_equivalent": {"achieved": tf, "peak": 157.3, "frac": tf / 157.3},
                "note": "6k executed flops per score on v_mfma_f32_32x32x16_bf16 (hi/lo split "
                        "operands; dense bf16 peak); device time of the mf_topk_mm launches "
                        "(inputs resident) incl. the stats / probe / split pre-passes and the "
                        "merge"}
    elif mm:
        tf = scores * 2 * k / elapsed / 1e12
        roof = {"bound": "mfma", "achieved": tf, "peak": 157.3, "unit": "TFLOP/s",
                "frac": tf / 157.3, "traffic": None, "kernel": mmk,
                "note": "2k flops per score on v_mfma_f32_32x32x2_f32 (f32 MFMA peak); device "
                        "time of the mf_topk_mm launches (inputs resident) incl. the merge"}
    else:
        roof = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                "kernel": "k_topk_fused" if "fused" in path else "k_topk_scores + k_topk_select",
                "note": "4k B per score (one item row per score, no reuse); device "
                        "time of the mf_topk launches (inputs resident)"}
    out = {
        "metric": "top-k scores/s (recommend_batch)", "value": scores / elapsed,
        "unit": "scores/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "f32" if ts == 4 else "f64", "data": "synthetic",
        "config": {"workload": desc, "n_users": nu, "n_items": ni, "n_factors": k,
                   "n_query": n_query, "amount": amount, "excluded_pairs": int(ex_ptr[-1]),
                   "chunk_users": batch["chunk"], "path": path},
        "roofline": roof,
        "cpu_baseline": cpu_baseline, "parity": parity,
        "launch": _launch_label(),
    }
    print(json.dumps(out), flush=True)
    return 0


def _launch_label() -> str:
    from matrix_factorization.engine import launch_form_label
    return launch_form_label()


def host_info() -> dict:
    """The host the CPU leg ran on (print nproc and the model)."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        nproc = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        nproc = None
    return {"cpu_model": model, "nproc": nproc, "os_cpu_count": os.cpu_count()}


class pinned_core:
    """Context manager: the calling thread's CPU affinity set to one core (the
    lowest of its current set) for the duration; yields a record of the mask
    actually in force, e.g. {"cpus": [0], "pinned": true}."""

    def __enter__(self):
        try:
            self.old = os.sched_getaffinity(0)
            core = min(self.old)
            os.sched_setaffinity(0, {core})
            return {"cpus": sorted(os.sched_getaffinity(0)), "pinned": True}
        except (AttributeError, OSError) as e:
            self.old = None
            return {"cpus": None, "pinned": False, "error": str(e)}

    def __exit__(self, *exc):
        if self.old is not None:
            os.sched_setaffinity(0, self.old)
        return False


def cpu_leg(args, eng, run, serial, seq_for, rot_for, reset_params, strat_sizes, nb, strata,
            kernel, k, mu, P0, Q0, nu, ni, n_local, shared=None):
    """CPU baseline + parity, untimed, before the timed epochs.

    Full epoch (--cpu-sample -1, the default).  From the same initial state
    (P0, Q0, zero biases) the GPU runs epoch 1 (FP32, strata order), then the
    FP64 oracle (oracle/mf_oracle.c, the reference's per-rating arithmetic)
    runs three full epochs on the host:
      (a) in the GPU's serialised order (StrataPlan.serial_order): GPU vs
          oracle, |dRMSE|, max|dP|, max|dQ|; timed alone = cpu_baseline;
      (b) in the reference's own order, np.random.shuffle of the rows
          (kernel_matrix_factorization.py:369-371, :428-440): |RMSE(a) -
          RMSE(b)| against the north-star 1e-5;
      (c) as (b) with another shuffle seed: the reference's own
          seed-to-seed spread at this size, the yardstick for (b).
    (b) and (c) run concurrently in two threads (ctypes drops the GIL).
    They do not depend on the GPU's dtype (the FP64 and FP32 runs start from
    the same FP32-representable values): computed once per bench run and kept
    in ``shared``.
    --cpu-sample N > 0: the first strata of epoch 1 covering >= N ratings,
    (a) only."""
    import concurrent.futures as cf

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # test infrastructure: checker and reported baseline only

    hyp = dict(kernel=kernel, gamma=1.0 / k, min_rating=1.0, max_rating=5.0)
    unit_name = "strata" if strata else "colours"
    seq0 = seq_for(0)
    full = args.cpu_sample < 0
    if full:
        m = nb
    else:
        sizes = strat_sizes[seq0]
        m = min(int(np.searchsorted(np.cumsum(sizes), min(args.cpu_sample, n_local))) + 1, nb)
    reset_params()
    run(0, seq0[:m])
    eng.sse_async(0)
    rmse_gpu_kernel = eng.rmse_values(1)[0] if full else None
    Pg, Qg, bug, big = eng.params_numpy()
    order = serial(0, seq0[:m])
    S = len(order)
    if full:
        u, i, r = eng.u_host, eng.i_host, eng.r_host.astype(np.float64)
    else:   # the sample's ratings only, in the serialised order
        u, i, r = eng.u_host[order], eng.i_host[order], eng.r_host[order].astype(np.float64)
        order = None

    def state():
        return (np.zeros(nu), np.zeros(ni), P0.astype(np.float64), Q0.astype(np.float64))

    def epoch(order_):
        bu, bi, P, Q = state()
        t0 = time.perf_counter()
        oracle.sgd_pass(u, i, r, mu, bu, bi, P, Q, lr=args.lr, reg=args.reg, order=order_,
                        **hyp)
        t1 = time.perf_counter()
        sse = oracle.sse(u, i, r, mu, bu, bi, P, Q, **hyp)
        t2 = time.perf_counter()
        return (bu, bi, P, Q), float(np.sqrt(sse / len(u))), t1 - t0, t2 - t1

    log(f"cpu oracle (a): {S} ratings ({m} of {nb} {unit_name}, GPU serial order), FP64, "
        f"1 thread")
    # pinned to one core for the timed leg (`taskset -c 0`)
    with pinned_core() as core:
        (bu, bi, P, Q), rm_a, t_sgd, t_sse = epoch(order)
    rm_g = float(np.sqrt(oracle.sse(u, i, r, mu, bug, big, Pg, Qg, **hyp) / len(u)))
    host = host_info()
    what = (f"one full epoch (all {S} ratings)" if full
            else f"first {m} of {nb} {unit_name} of epoch 1 = {S} ratings")
    cpu_baseline = {
        "value": S / (t_sgd + t_sse), "unit": "rating-updates/s", "cores": 1, "kind": "port",
        "sample": (f"{what} of the same workload: FP64 sequential SGD sweep ({t_sgd:.1f}s) "
                   f"+ RMSE pass ({t_sse:.1f}s), oracle/mf_oracle.c, one thread"),
        "sgd_only": S / t_sgd, "affinity": core, **host,
    }
    parity = {
        "what": (f"{what} from the same initial state: (a) GPU "
                 f"{'FP32' if args.dtype == 'float32' else 'FP64'} strata vs CPU oracle "
                 f"FP64 in the GPU's serialised order"
                 + ("; (b) oracle in the reference's np.random.shuffle order; (c) the same, "
                    "another shuffle seed (the reference's own seed spread)" if full else "")),
        "rmse_gpu": rm_g, "rmse_cpu": rm_a, "abs_diff": abs(rm_g - rm_a),
        "max_abs_dP": float(np.max(np.abs(Pg - P))),
        "max_abs_dQ": float(np.max(np.abs(Qg - Q))),
        "max_abs_dbu": float(np.max(np.abs(bug - bu))),
        "max_abs_dbi": float(np.max(np.abs(big - bi))),
    }
    del P, Q, bu, bi
    if full:
        parity["rmse_gpu_kernel"] = rmse_gpu_kernel      # k_sse_owned's own FP64 reduction
        parity["abs_diff_gpu_kernel"] = abs(rmse_gpu_kernel - rm_a)

        def shuffled(seed):
            o = np.arange(len(u), dtype=np.int64)
            np.random.RandomState(seed).shuffle(o)       # = np.random.shuffle(X), :371
            return epoch(o)[1]

        if shared is not None and "ref_order" in shared:
            rm_b, rm_c = shared["ref_order"]
        else:
            log("cpu oracle (b), (c): the same epoch in two np.random.shuffle orders, 2 threads")
            with cf.ThreadPoolExecutor(2) as ex:
                rm_b, rm_c = ex.map(shuffled, (7, 8))
            if shared is not None:
                shared["ref_order"] = (rm_b, rm_c)
        parity.update({
            "rmse_shuffle_order": rm_b, "rmse_shuffle_order_seed2": rm_c,
            "abs_diff_strata_vs_shuffle": abs(rm_a - rm_b),
            "shuffle_seed_spread": abs(rm_b - rm_c),
            "gate_1e5": bool(abs(rm_a - rm_b) <= 1e-5 and abs(rm_g - rm_a) <= 1e-5),
        })
    log(f"cpu {cpu_baseline['value'] / 1e6:.2f} M/s; parity " +
        ", ".join(f"{kk}={vv:.3e}" for kk, vv in parity.items()
                  if isinstance(vv, float) and kk.startswith(("abs", "shuffle"))))
    return cpu_baseline, parity


DRAW_SEED = 12345


def strata_seq(ep: int, nb) -> np.ndarray:
    """Stratum (colour) order of bench epoch ``ep``; ``nb`` = a strata plan
    (its B and user-range classes) or a colour / stratum count."""
    from matrix_factorization.engine import stratum_order
    return stratum_order(np.random.RandomState((DRAW_SEED * 1000003 + ep) & 0x7FFFFFFF), nb)


def strata_rot(ep: int) -> int:
    """Step-rotation seed of bench epoch ``ep`` (rotate: the epoch's draw)."""
    return (DRAW_SEED * 7919 + ep * 104729) & 0x7FFFFFFF


def multi_checks(args, eng, rotate, world, rank, dev, u, i, r, nu, ni, k, kernel, mu, P0, Q0,
                 n_ep, rmse) -> dict:
    """N > 1, after the timed epochs (untimed): is the multi-GPU result
    right?  Every rank takes part in the collectives; rank 0 also re-runs the
    work on its own GPU.

    replicas     a 64-bit fingerprint of each rank's [Q | b_i] replica
                 (mf_fingerprint): all ranks must agree bit for bit;
    replay       rotate: rank 0 runs the same N-rank rotation order on ONE GPU
                 (distributed.RotationReplay: the same shards, item ranges,
                 plans and draws, sub-blocks one after another) for the same
                 epochs from the same start, and compares P, Q, b_u, b_i and
                 the per-epoch RMSE with the N-GPU result (expected: bit-equal
                 parameters -- the order is a sequential one, fixed by the plans
                 and draws);
    n1           rank 0 trains the same data from the same start for the same
                 epochs with the single-GPU default (one strata plan over all
                 ratings) and reports the RMSE gap (north star: RMSE matching
                 the CPU reference to 1e-5; the N=1 run is pinned to the CPU
                 oracle by the N=1 bench line's parity)."""
    import torch
    import torch.distributed as dist

    from matrix_factorization import _lib
    from matrix_factorization.distributed import RotationReplay, _gather_rows, shard_users
    from matrix_factorization.engine import SGDEngine

    t0 = time.time()
    Qh = eng.Q.detach().cpu().numpy()
    bih = eng.bi.detach().cpu().numpy()
    lib = _lib.load()
    fp = [int(lib.mf_fingerprint(np.ascontiguousarray(a).ctypes.data, a.nbytes))
          for a in (Qh, bih)]
    mine = torch.tensor([fp[0] & 0x7FFFFFFFFFFFFFFF, fp[1] & 0x7FFFFFFFFFFFFFFF],
                        dtype=torch.int64, device=dev if args.backend == "nccl" else "cpu")
    allfp = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(allfp, mine)
    allfp = [tuple(int(x) for x in t.cpu()) for t in allfp]
    bounds = shard_users(u, nu, world)
    Pg = _gather_rows(eng.P, bounds)
    bug = _gather_rows(eng.bu.reshape(-1, 1), bounds).reshape(-1)
    out = {"exchange": "rotate" if rotate else "delta",
           "replica_fingerprints": [f"{a:016x}:{b:016x}" for a, b in allfp],
           "replicas_agree": all(f == allfp[0] for f in allfp)}
    if rank == 0 and not args.no_check:
        hyp = dict(gamma=1.0 / k, min_rating=1.0, max_rating=5.0, global_mean=mu)
        if rotate:
            log("check: one-GPU replay of the N-rank rotation order")
            rp = RotationReplay(u, i, r, nu, ni, world, k, kernel, args.dtype, dev,
                                n_blocks=args.blocks, waves=args.waves, relabel=args.relabel,
                                **hyp)
            rp.load(P0, Q0, np.zeros(nu), np.zeros(ni))
            sse = []
            for ep in range(n_ep):
                rp.epoch(strata_rot(ep), args.lr, args.reg, epoch=ep)
                sse.append(rp.sse(ep))
            Pr, Qr, bur, bir = rp.params()
            rm_r = [float(np.sqrt(x / len(u))) for x in sse]
            d = {"dP": float(np.max(np.abs(Pr - Pg))),
                 "dQ": float(np.max(np.abs(Qr - Qh.astype(np.float64)))),
                 "dbu": float(np.max(np.abs(bur - bug))),
                 "dbi": float(np.max(np.abs(bir - bih.astype(np.float64))))}
            out["replay"] = {
                "what": ("rank 0 ran the same N-rank rotation order on one GPU (RotationReplay) "
                         f"for the same {n_ep} epochs from the same start"),
                "max_abs_diff": d, "bit_equal": all(v == 0.0 for v in d.values()),
                "max_abs_rmse_diff": float(np.max(np.abs(np.asarray(rm_r) - np.asarray(rmse)))),
                "rmse_replay_final": rm_r[-1]}
            del rp
            torch.cuda.empty_cache()
        log("check: N=1 leg (single-GPU default schedule, same data, start and epochs)")
        e1 = SGDEngine(u, i, r, nu, ni, k, kernel, args.dtype, dev, **hyp)
        e1.load_params(P=P0, Q=Q0, bu=np.zeros(nu), bi=np.zeros(ni))
        plan1 = e1.prepare_strata()
        for ep in range(n_ep):
            e1.epoch_strata(strata_seq(ep, plan1), strata_rot(ep), args.lr, args.reg)
            e1.sse_async(ep)
        rm1 = e1.rmse_values(n_ep)
        del e1
        torch.cuda.empty_cache()
        out["n1"] = {"what": (f"rank 0: the same {n_ep} epochs on one GPU with the single-GPU "
                              "default schedule (the N=1 bench line's)"),
                     "rmse_n1_final": rm1[-1], "rmse_final": rmse[-1],
                     "rmse_gap_vs_n1": rmse[-1] - rm1[-1],
                     "rmse_per_epoch_n1": rm1}
        out["check_s"] = time.time() - t0
        log(f"checks: replicas agree {out['replicas_agree']}, "
            + (f"replay bit-equal {out['replay']['bit_equal']}, " if rotate else "")
            + f"RMSE gap vs N=1 {out['n1']['rmse_gap_vs_n1']:+.3e}")
    dist.barrier()
    return out


def emulation_fields(args, out, elapsed, emu, nnz, dev, u, i, r, nu, ni, k, kernel, mu, P0,
                     Q0) -> None:
    """--emulate-rank: the line is a per-rank timing probe, not a rate.  The
    measured rank-0 epoch goes to ``projection`` next to the same box's N=1
    epoch (the single-GPU default schedule, same data, dtype and epochs);
    ``value`` is null and ``metric`` names the probe, so no parser can take
    the projection for a measured job rate."""
    import torch

    from matrix_factorization.engine import SGDEngine

    per_rank_ms = elapsed / args.steps * 1e3
    hyp = dict(gamma=1.0 / k, min_rating=1.0, max_rating=5.0, global_mean=mu)
    e1 = SGDEngine(u, i, r, nu, ni, k, kernel, args.dtype, dev, **hyp)
    e1.load_params(P=P0, Q=Q0, bu=np.zeros(nu), bi=np.zeros(ni))
    plan1 = e1.prepare_strata()
    n_ep = args.warmup + args.steps
    for ep in range(args.warmup):
        e1.epoch_strata(strata_seq(ep, plan1), strata_rot(ep), args.lr, args.reg)
        e1.sse_async(ep)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for ep in range(args.warmup, n_ep):
        e1.epoch_strata(strata_seq(ep, plan1), strata_rot(ep), args.lr, args.reg)
        e1.sse_async(ep)
    torch.cuda.synchronize(dev)
    n1_ms = (time.perf_counter() - t0) / args.steps * 1e3
    del e1
    torch.cuda.empty_cache()
    out["metric"] = f"EMULATION probe: rank 0's epoch of a {emu}-rank rotation on one GPU"
    out["value"] = None
    out["unit"] = None
    out["projection"] = {
        "per_rank_epoch_ms": per_rank_ms,
        "n1_epoch_ms_same_box": n1_ms,
        "projected_speedup": n1_ms / per_rank_ms,
        "projected_job_rate": nnz / (per_rank_ms / 1e3),
        "note": ("rank 0's share (its user shard, N sub-epochs, ring hand-offs as device "
                 "copies of the same size) timed alone on one GPU; the N-GPU job would run "
                 "at this rate only if every rank took as long and the xGMI hand-offs cost "
                 "what the copies cost"),
    }


def _emulated_ring_cls():
    from matrix_factorization.distributed import RotationExchange

    class EmulatedRing(RotationExchange):
        """Rank 0 of an N-rank rotation on one GPU (--emulate-rank): the ring
        hand-off copies the range it would send into the rows it would
        receive (a device copy of the same size), the all-gather unpacks this
        rank's range N times (same bytes written); the sweeps, the snapshot
        copies and the overlapped RMSE pass are the real ones."""

        def __init__(self, engine, ilo, n, overlap=True):
            import torch as _t
            self.e, self.group = engine, None
            self.ilo = np.asarray(ilo, np.int64)
            self.world, self.rank = int(n), 0
            self.stage = False
            self.rows = int(np.diff(self.ilo).max())
            self._gbuf = None
            self.overlap = bool(overlap)
            self._ov = None
            self.sse_events = []
            self._t = _t

        def pass_range(self, c_send, c_recv):
            qs, bs = self._range(c_send)
            qr, br = self._range(c_recv)
            n = min(qs.shape[0], qr.shape[0])
            qr[:n].copy_(qs[:n])
            br[:n].copy_(bs[:n])

        def _all_gather_unpack(self, c_final, Q, bi, skip_own):
            mine, out = self._buffers()
            out.view(self.world, -1).copy_(mine.view(1, -1).expand(self.world, -1))
            k, m = self.e.k, self.rows
            parts = out.view(self.world, m * (k + 1))
            for r in range(self.world):
                if r == self.rank and skip_own:
                    continue
                q, b = self._range(c_final[r], Q, bi)
                n = q.shape[0]
                q.copy_(parts[r, : n * k].view(n, k))
                b.copy_(parts[r, m * k: m * k + n])

    return EmulatedRing


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="c3", choices=sorted(WORKLOADS))
    ap.add_argument("--dtype", default="auto", choices=["auto", "float32", "float64"],
                    help="SGD workloads: auto (default) = the reference's FP64 arithmetic "
                         "as the headline line, the FP32 perf layout measured in the same "
                         "run and nested as `fp32_layout`; ALS / top-k: auto = float32")
    ap.add_argument("--lr", type=float, default=0.01)
    ap.add_argument("--reg", type=float, default=None,
                    help="default 0.02 for SGD (project_template/pipeline/train.py:29-36), "
                         "1.0 for ALS (KernelMF's default reg)")
    ap.add_argument("--cpu-sample", type=int, default=-1,
                    help="CPU leg: -1 = one full epoch (default; parity in the strata "
                         "order and in the reference's shuffle order), N > 0 = the first "
                         "strata of epoch 1 covering >= N ratings, 0 = skip")
    ap.add_argument("--no-phase-timing", action="store_true",
                    help="do not bracket the SGD / RMSE phases with hipEvents")
    ap.add_argument("--blocks", type=int, default=None,
                    help="strata: B (probes; default: engine.choose_strata_blocks)")
    ap.add_argument("--waves", type=int, default=None, choices=[4, 8, 16],
                    help="strata: waves per workgroup (default: by the plan's slot fill; "
                         "4 = the 8-wave plan on the narrow 4-wave kernels)")
    ap.add_argument("--schedule", default="strata", choices=["strata", "colored"],
                    help="strata: B x B blocks, item slabs in LDS (mf_strata.hpp); "
                         "colored: one launch per edge colour (mf_rows.hpp)")
    ap.add_argument("--exchange", default="rotate", choices=["rotate", "delta"],
                    help="N > 1 (strata): rotate = item ranges passed round the ring "
                         "between N sub-epochs (exact: a sequential order, DESIGN.md 6); "
                         "delta = item deltas all-reduced once per epoch, applied damped")
    ap.add_argument("--no-delta-leg", action="store_true",
                    help="N > 1, --exchange rotate: skip the nested delta-exchange run")
    ap.add_argument("--relabel", type=int, default=None,
                    help="N > 1, --exchange rotate: item relabellings, one drawn per epoch "
                         "(default distributed.ROTATE_RELABEL = 8; 1 = the plain rotation)")
    ap.add_argument("--delta-scale", type=float, default=None,
                    help="N > 1, --exchange delta: weight of the all-reduced item deltas "
                         "(default min(1/2, 2/N), distributed.default_delta_scale; "
                         "1.0 = plain gradient sum)")
    ap.add_argument("--emulate-rank", type=int, default=0,
                    help="one GPU, N > 1: run rank 0's share of an N-rank rotation run "
                         "(its user shard, N sub-epochs over the N item ranges, the RMSE "
                         "pass overlapped as in the real run); the ring hand-offs and the "
                         "all-gather become device copies of the same sizes (stand-ins: "
                         "no xGMI on one GPU); a per-rank timing probe, not a bench line")
    ap.add_argument("--rotate-no-overlap", action="store_true",
                    help="--exchange rotate: gather the replica and run the RMSE pass on the "
                         "launch stream after every epoch (default: on a side stream beside "
                         "the next epoch's sub-epochs)")
    ap.add_argument("--no-check", action="store_true",
                    help="N > 1: skip the post-timing checks (replica checksums on every "
                         "rank, rank 0's one-GPU replay of the same order, the N=1 RMSE leg)")
    ap.add_argument("--rmse-overlap", action="store_true",
                    help="one GPU: run each epoch's RMSE pass on a side stream from a "
                         "parameter snapshot, beside the next epoch's sweep")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="N>1 process group: nccl (= RCCL, one GPU per rank) or gloo "
                         "(rehearsal: ranks may share a GPU, LOCAL_RANK mod device count)")
    args = ap.parse_args()
    record_maps_at_exit()
    if args.relabel is None:
        from matrix_factorization.distributed import ROTATE_RELABEL
        args.relabel = ROTATE_RELABEL

    import torch
    import torch.distributed as dist

    from matrix_factorization import _lib

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"WORLD_SIZE={world} but --gpus={args.gpus}; using WORLD_SIZE")
    if args.backend == "gloo":
        dev = torch.device("cuda", local_rank % max(torch.cuda.device_count(), 1))
    else:
        dev = torch.device("cuda", local_rank)
    torch.cuda.set_device(dev)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    _lib.load()

    nu, ni, nnz, k, kernel, desc = WORKLOADS[args.workload]
    t0 = time.time()
    u, i, r = synth(nu, ni, nnz)
    log(f"data: {nnz} ratings {nu}x{ni} in {time.time() - t0:.1f}s")
    mu = float(np.mean(r, dtype=np.float64))
    # the initial state: N(0, 0.1) draws (kernel_matrix_factorization.py:97-102)
    # rounded to FP32, so the FP64 and FP32 runs (and the CPU oracle's legs)
    # start from exactly the same values
    rs = np.random.RandomState(7)
    P0 = rs.normal(0.0, 0.1, (nu, k)).astype(np.float32)
    Q0 = rs.normal(0.0, 0.1, (ni, k)).astype(np.float32)
    if kernel in ("als", "topk"):
        if args.dtype == "auto":
            args.dtype = "float32"
        P0, Q0 = P0.astype(args.dtype), Q0.astype(args.dtype)
        if kernel == "als":
            if world > 1:
                raise SystemExit("the ALS workload (configs[4]) is a single-GPU config")
            return run_als(args, u, i, r, nu, ni, nnz, k, desc, mu, P0, Q0, dev)
        return run_topk(args, u, i, r, nu, ni, nnz, k, desc, mu, P0, Q0, dev)
    if args.reg is None:
        args.reg = 0.02
    dtypes = ["float64", "float32"] if args.dtype == "auto" else [args.dtype]
    shared = {}
    outs = []
    for dt in dtypes:
        log(f"---- {dt} run")
        outs.append(run_sgd(args, dt, world, rank, dev, u, i, r, nu, ni, nnz, k, kernel, desc,
                            mu, P0, Q0, shared))
        torch.cuda.empty_cache()
    # N > 1, rotate: the other exchange measured in the same job and nested
    # (`delta_exchange`), so one N-GPU run maps both ends of the frontier
    # (exact order vs damped item deltas)
    delta_leg = None
    if (world > 1 and args.exchange == "rotate" and args.schedule == "strata"
            and not args.no_delta_leg):
        log(f"---- {dtypes[0]} run, exchange delta (nested leg)")
        da = argparse.Namespace(**{**vars(args), "exchange": "delta"})
        delta_leg = run_sgd(da, dtypes[0], world, rank, dev, u, i, r, nu, ni, nnz, k, kernel,
                            desc, mu, P0, Q0, shared)
        torch.cuda.empty_cache()
    if rank == 0:
        out = outs[0]
        if len(outs) > 1:
            out["fp32_layout"] = nested_line(outs[1])
        if delta_leg is not None:
            out["delta_exchange"] = nested_line(delta_leg, fp32=False)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


def nested_line(o: dict, fp32: bool = True) -> dict:
    """A second run nested under the headline line: the FP32 perf layout
    (``fp32``), or at N > 1 the other exchange."""
    keep = ("value", "unit", "ms_per_step", "dtype", "final_rmse", "rmse_per_epoch",
            "roofline", "phases", "parity", "multi_gpu", "projection", "schedule_build_s",
            "launch")
    d = {kk: o.get(kk) for kk in keep if kk in o}
    d["schedule"] = o["config"]["schedule"]
    d["exchange"] = o["config"].get("exchange")
    d["item_delta_scale"] = o["config"].get("item_delta_scale")
    if fp32:
        d["arithmetic"] = ("FP32 parameters; fused multiply-adds, v_exp_f32 / v_rcp_f32 "
                           "(DESIGN.md section 3): not the reference's expression order, "
                           "parity as a tolerance vs the FP64 oracle")
    return d


def run_sgd(args, dtype, world, rank, dev, u, i, r, nu, ni, nnz, k, kernel, desc, mu, P0, Q0,
            shared) -> dict:
    """One SGD bench run in ``dtype`` (float64: the reference's arithmetic,
    float32: the perf layout).  Returns the JSON line (rank 0) or None."""
    import torch
    import torch.distributed as dist

    from matrix_factorization.distributed import (ReplicaExchange, RotationSet,
                                                  any_rank_failed, global_rmse, item_ranges,
                                                  local_shard, shard_users)
    from matrix_factorization.engine import (STREAM_MAX_STEPS, SGDEngine, launch_form_label,
                                             max_block_steps, strata_slots)

    args = argparse.Namespace(**{**vars(args), "dtype": dtype})
    P0, Q0 = P0.astype(dtype), Q0.astype(dtype)
    emu = args.emulate_rank if world == 1 else 0
    if world > 1 or emu > 1:
        nw, rk = (world, rank) if world > 1 else (emu, 0)
        bounds = shard_users(u, nu, nw)
        lu, li, lr_ = local_shard(u, i, r, bounds, rk)
        lo, hi = int(bounds[rk]), int(bounds[rk + 1])
        P_local = P0[lo:hi]
        if emu > 1:
            args.cpu_sample = 0                # the CPU leg needs the whole workload
    else:
        lu, li, lr_, P_local = u, i, r, P0
    n_local = len(lu)
    n_users_local = P_local.shape[0]

    eng = SGDEngine(lu, li, lr_, n_users_local, ni, k, kernel, args.dtype, dev,
                    gamma=1.0 / k, min_rating=1.0, max_rating=5.0, global_mean=mu)
    t0 = time.time()
    strata = args.schedule == "strata"
    rotate = (world > 1 or emu > 1) and strata and args.exchange == "rotate"
    ilo = item_ranges(i, ni, max(world, emu)) if rotate else None
    if strata:
        # (the delta exchange's epochs always run the engine's own plan: no
        # relabelled plans for it)
        plan = eng.prepare_strata(n_blocks=args.blocks, waves=args.waves, item_bounds=ilo,
                                  regroup=1 if (world > 1 and not rotate) else None)
        nb = plan.n_strata                   # strata per epoch (C*B with C user-range classes)
        B = plan.B                           # workgroups / item slabs
        cls = plan.classes
        n_phases = len(getattr(plan, "phases", [plan]))   # item phases (PhasedStrata)
        strat_sizes = plan.stratum_sizes()           # ratings per stratum (launch)
        fill = n_local / max(plan.n_positions, 1)
        sched_desc = ((f"strata rotation ({n_phases} item ranges passed round the ring: "
                       f"{n_phases} sub-epochs x {nb} strata (B={B}"
                       f"{f', {cls} user-range classes' if cls > 1 else ''}) on this rank's "
                       f"sub-block, "
                       if rotate else
                       f"strata ({n_phases} item phases x {nb} strata of B={B}, " if n_phases > 1
                       else f"strata (B={B}: {nb} launches/epoch, ")
                      + (f"{cls} user-range classes ({cls * B} user ranges, {cls - 1} "
                         f"block(s) of slack per hand-off), " if cls > 1 else "")
                      + (f"{1 + len(eng._regroups)} relabelled plans, one drawn per epoch, "
                         if eng._regroups else "")
                      + "item slabs in LDS, "
                      f"{plan.NS} user-owned slots "
                      f"({256 if plan.narrow else plan.NS * 1024 // strata_slots(k, eng.dcode)} "
                      f"threads/workgroup{', narrow lane groups' if plan.narrow else ''}) x "
                      f"{int(plan.n_steps.max())} steps max "
                      f"per block, {fill:.1%} slot fill"
                      f"{', user rows 2 steps ahead' if eng._deep_pipe(plan) else ''}"
                      f"{', one pipeline through all positions (stream)' if (eng._deep_pipe(plan) and cls > 1 and eng._stream()) else ''})")
    else:
        nb = eng.prepare_colored()
        n_phases = 1
        strat_sizes = np.diff(eng.colored)
        sched_desc = f"colored ({nb} conflict-free batches/epoch on rank 0)"
    t_sched = time.time() - t0
    log(f"rank {rank}: {n_local} local ratings, {sched_desc}, scheduled in {t_sched:.1f}s")
    exch = (ReplicaExchange(eng, scale=args.delta_scale) if world > 1 and not rotate
            else None)
    # rotate: epoch e's gather + RMSE pass on a side stream beside epoch e+1,
    # over args.relabel item relabellings (one drawn per epoch; RotationSet)
    rot = None
    if rotate:
        t1 = time.time()
        mk = None
        if emu > 1:
            ring = _emulated_ring_cls()
            mk = lambda e, lo: ring(e, lo, emu, overlap=not args.rotate_no_overlap)  # noqa: E731
        rot = RotationSet(eng, i, max(world, emu), args.relabel,
                          overlap=not args.rotate_no_overlap, make_exchange=mk,
                          prepare=dict(n_blocks=args.blocks, waves=args.waves))
        if rot.K > 1:
            sched_desc = sched_desc.replace(
                "item ranges passed round the ring",
                f"item ranges passed round the ring, {rot.K} item relabellings, one drawn "
                f"per epoch")
        t_sched += time.time() - t1
    rot_overlap = rotate and rot.overlap
    eng._ensure_sse_slots(args.warmup + args.steps + 1)
    if rot is not None:
        rot.ensure_sse_slots(args.warmup + args.steps + 1)

    def reset_params():
        eng.load_params(P=P_local, bu=np.zeros(n_users_local))
        if exch is not None:
            exch.bind(Q0, np.zeros(ni))
        else:
            eng.load_params(Q=Q0, bi=np.zeros(ni))
        if rot is not None:
            rot.bind()

    def seq_for(ep):
        return strata_seq(ep, plan if strata else nb)

    def rot_for(ep):          # colour-rotation seed of a strata epoch (rotate: the epoch draw)
        return strata_rot(ep)

    def run(ep, seq, timing=False, events=None):
        """The local sweep of epoch ep (N > 1, strata: delta-out form -- the
        replica stays put and the item update lands in exch.delta; rotate:
        the whole rotation epoch, hand-offs and final all-gather included)."""
        if rotate:
            launches = [] if timing else None
            rot.epoch(rot_for(ep), args.lr, args.reg, events=events, launches=launches,
                      epoch=ep, sse_slot=ep if rot_overlap else None,
                      sse_timing=events is not None)
            return (None, sum(launches)) if timing else None
        if strata:
            delta = None if exch is None else (exch.dq, exch.dbi)
            return eng.epoch_strata(seq, rot_for(ep), args.lr, args.reg, timing=timing,
                                    delta=delta)
        return eng.epoch_colored(seq, args.lr, args.reg, timing=timing)

    def begin():
        if exch is not None and not strata:
            exch.begin_epoch()               # colored: snapshot form

    def end():
        if exch is not None:
            if strata:
                exch.exchange()              # all_reduce(delta); replica += delta
            else:
                exch.end_epoch()

    def serial(ep, seq):
        if strata:
            return eng.serial_order(seq, rot_for(ep)).astype(np.int64)
        return np.concatenate([np.arange(eng.colored[b], eng.colored[b + 1])
                               for b in seq]).astype(np.int64)

    # ---------------- CPU baseline + parity (rank 0, N=1; untimed)
    cpu_baseline = None
    parity = None
    if world == 1 and args.cpu_sample != 0:
        cpu_baseline, parity = cpu_leg(args, eng, run, serial, seq_for, rot_for, reset_params,
                                       strat_sizes, nb, strata, kernel, k, mu, P0, Q0, nu, ni,
                                       n_local, shared)

    # ---------------- warmup + timed epochs
    reset_params()
    phase = not args.no_phase_timing
    launches_per_epoch = nb if strata else int(np.sum(np.diff(eng.colored) > 0))
    persistent = False
    events = []     # (sgd start, sgd end, exchange end, sse end) per timed epoch
    # --rmse-overlap (one GPU): the RMSE pass of epoch e runs on a side stream
    # from a snapshot of the parameters, beside the SGD sweep of epoch e + 1.
    # Off by default: at C3 the persistent sweep cannot start its workgroups
    # while the RMSE kernel holds the CUs, so the two serialise and the
    # snapshot copy is pure cost (11.83 vs 11.67 ms per epoch; C2 1.125 vs
    # 1.146 ms) -- DESIGN.md section 5
    overlap = world == 1 and args.rmse_overlap

    rot_events = []   # rotate: per timed epoch, the (kind, start, end) events of its parts

    def sse_now(ep):
        # rotate: the SSE of the labelling the epoch ran in (its engine's
        # ratings carry that labelling's item ids; shared SSE buffer)
        (eng if rot is None else rot.engines[rot.cur]).sse_async(ep)

    def epoch(ep, timed):
        # hipEvents on the stream the kernels run on (torch's current stream,
        # which the engine launches on): one pair around the epoch's SGD
        # launches, one more after the RMSE pass -- no host sync in the loop.
        # rotate: every sub-epoch and hand-off bracketed too (rot_events).
        seq = seq_for(ep)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)] if (timed and phase) else None
        begin()
        if ev:
            ev[0].record()
        if rotate and ev:
            rot_events.append([])
            run(ep, seq, events=rot_events[-1])
        else:
            run(ep, seq)
        if ev:
            ev[1].record()
        end()
        if ev:
            ev[2].record()
        if overlap:
            eng.sse_overlap(ep, timing=bool(ev))
        elif not rot_overlap:                # rotate + overlap: ran on the side stream
            sse_now(ep)
        if ev:
            ev[3].record()
            events.append(ev)

    for ep in range(args.warmup):
        if ep == 0 and strata:
            # one synchronised epoch tells whether the persistent kernel ran
            # (one launch) or the per-stratum fallback (B launches)
            begin()
            _, n_launch = run(ep, seq_for(ep), timing=True)
            end()
            if not rot_overlap:
                sse_now(ep)
            persistent = n_launch == n_phases
            if persistent:           # one persistent launch per epoch (per item phase)
                sched_desc = sched_desc.replace(
                    f"B={B}: {nb} launches/epoch", f"B={B}, {nb} strata in 1 persistent launch/epoch")
                if rotate:
                    sched_desc = sched_desc.replace("strata on this rank's sub-block",
                                                    "strata in 1 persistent launch per sub-epoch")
            launches_per_epoch = n_launch
        else:
            epoch(ep, False)
        log(f"warmup epoch {ep + 1}/{args.warmup}")
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for j in range(args.steps):
        epoch(args.warmup + j, True)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    if strata and any_rank_failed(eng if rot is None else rot):   # all ranks raise together
        raise SystemExit("a persistent strata sweep gave up waiting (workgroups not "
                         "co-resident): the timed epochs are invalid")
    n_ep = args.warmup + args.steps
    if rot is not None:       # the live canonical replica whole again (checks), SSEs landed
        rot.finish(n_ep - 1)
    rmse = global_rmse(eng, n_ep, nnz)
    multi = None
    if world > 1:
        multi = multi_checks(args, eng, rotate, world, rank, dev, u, i, r, nu, ni, k, kernel, mu,
                             P0, Q0, n_ep, rmse)

    if rank == 0:
        value = nnz * args.steps / elapsed
        ts = 4 if args.dtype == "float32" else 8
        # 16k+28 B per rating-update = triple + user and item
        # rows read and written + both biases read and written.  The colored
        # kernel moves all of it through HBM / the fabric; the strata kernel
        # keeps item rows and biases in LDS, so its algorithmic HBM bytes are
        # the user row read + write, the triple and the user bias per update,
        # plus per stratum the item slab (+ item biases) in and out and the
        # user-bias slice in and out (mf_strata.hpp) -- DESIGN.md section 4.
        survey_per_update = (16 * k + 28) if ts == 4 else (32 * k + 44)
        if strata:
            # triples of every plan position (idle slots included), user row
            # read + write per update, the user-bias slice in + out per block,
            # the item slab (+ biases) in + out once per epoch (persistent) or
            # once per stratum (per-stratum launches)
            slab_passes = 1 if persistent else nb
            alg_epoch = (plan.n_positions * (8 + ts) + n_local * 2 * k * ts
                         + n_phases * B * 2 * n_users_local * ts
                         + slab_passes * 2 * ni * (k + 1) * ts)
        else:
            alg_epoch = n_local * survey_per_update
        bytes_per_update = alg_epoch / n_local
        roofline = None
        phases = None
        if events:
            sgd_s = sum(e[0].elapsed_time(e[1]) for e in events) / 1e3
            exch_s = sum(e[1].elapsed_time(e[2]) for e in events) / 1e3
            sse_s = sum(e[2].elapsed_time(e[3]) for e in events) / 1e3
            if rotate:      # split the rotation epoch into its sweeps and hand-offs
                part = {"sgd": 0.0, "pass": 0.0, "gather": 0.0, "relabel": 0.0}
                for evs in rot_events:
                    for kind, a, b in evs:
                        part[kind] += a.elapsed_time(b) / 1e3
                sgd_s = part["sgd"]
                exch_s = part["pass"] + part["gather"] + part["relabel"]
            launches = launches_per_epoch * len(events)
            alg = alg_epoch * len(events)                           # algorithmic bytes
            achieved = alg / sgd_s / 1e9
            stream = (strata and persistent and cls > 1 and eng._deep_pipe(plan)
                      and eng._stream() and max_block_steps(plan) <= STREAM_MAX_STEPS)
            kname = ((("k_sgd_strata_stream" if stream else "k_sgd_strata_epoch")
                      if persistent else "k_sgd_strata") if strata else "k_sgd_batch")
            traffic = traffic_from_profiles(args.workload, world, args.schedule
                                            + ("_persistent" if persistent else ""),
                                            args.dtype, kname, emulate=emu)
            roofline = {
                "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                "kernel": kname, "launches": launches,
                "avg_launch_us": sgd_s / launches * 1e6,
                "avg_launch_note": "SGD phase time / launches (hipEvents around each "
                                   "epoch's SGD launches on the launch stream)",
                "alg_bytes_per_launch": alg / launches,
                "bytes_per_update": bytes_per_update,
                "survey_bytes_per_update": survey_per_update,
                "survey_equivalent_gbs": survey_per_update * n_local * len(events) / sgd_s / 1e9,
                "note": "achieved = HBM bytes the schedule must move (item rows live in "
                        "LDS for strata); survey_equivalent_gbs = the 16k+28 B/update "
                        "count of SURVEY 8(d) over the same time",
            }
            phases = {"sgd_ms_per_epoch": sgd_s / len(events) * 1e3,
                      "rmse_ms_per_epoch": sse_s / len(events) * 1e3,
                      "sgd_updates_per_s": n_local * len(events) / sgd_s}
            if overlap:
                side = (eng._ov or {}).get("events", [])
                phases["rmse_ms_per_epoch"] = (sum(a.elapsed_time(b) for a, b in side)
                                               / max(len(side), 1))
                phases["snapshot_ms_per_epoch"] = sse_s / len(events) * 1e3
                phases["rmse_overlapped"] = ("on a side stream, from a device snapshot of "
                                             "the parameters, beside the next epoch's sweep")
            if world > 1:
                phases["exchange_ms_per_epoch"] = exch_s / len(events) * 1e3
                if rotate:
                    phases["ring_pass_ms_per_epoch"] = part["pass"] / len(events) * 1e3
                    phases["gather_ms_per_epoch"] = part["gather"] / len(events) * 1e3
                    phases["relabel_ms_per_epoch"] = part["relabel"] / len(events) * 1e3
                if rot_overlap:
                    side = rot.sse_events[-len(events):]
                    phases["rmse_ms_per_epoch"] = (sum(a.elapsed_time(b) for a, b in side)
                                                   / max(len(side), 1))
                    phases["gather_ms_per_epoch_note"] = (
                        "launch-stream part only (snapshot copies); the all-gather and the "
                        "RMSE pass run on a side stream beside the next epoch: "
                        "rmse_ms_per_epoch is their side-stream time")
        out = {
            "metric": METRIC, "value": value, "unit": "rating-updates/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None,
            "dtype": "f32" if args.dtype == "float32" else "f64",
            "data": "synthetic",
            "config": {"workload": desc, "n_users": nu, "n_items": ni, "nnz": nnz,
                       "n_factors": k, "kernel": kernel, "lr": args.lr, "reg": args.reg,
                       "schedule": sched_desc,
                       "parallelism": (f"user-sharded dp{world}" if world > 1 else
                                       f"EMULATION: rank 0 of a {emu}-rank rotation on one GPU "
                                       f"(hand-offs as device copies); not a measurement of "
                                       f"the N-GPU job: see `projection`" if emu > 1 else
                                       "single GPU"),
                       "exchange": (None if world == 1 else "rotate" if rotate else "delta"),
                       "item_delta_scale": None if exch is None else exch.scale,
                       "step": "one epoch: SGD sweep + training-RMSE pass" +
                               (" (epoch e's RMSE overlapped with epoch e+1's sweep)"
                                if overlap or rot_overlap else "")},
            "final_rmse": rmse[-1], "rmse_per_epoch": rmse,
            "roofline": roofline, "phases": phases,
            "cpu_baseline": cpu_baseline, "parity": parity, "multi_gpu": multi,
            "schedule_build_s": t_sched,
            # how the persistent sweeps were launched in this process: plain
            # under rocprofv3's preload (engine._under_rocprofiler)
            "launch": launch_form_label(),
        }
        if emu > 1:
            emulation_fields(args, out, elapsed, emu, nnz, dev, u, i, r, nu, ni, k, kernel, mu,
                             P0, Q0)
        return out
    return None




if __name__ == "__main__":
    sys.exit(main())

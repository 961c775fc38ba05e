"""Wall time of the public KernelMF.fit() at C3 scale, split by phase.

Synthetic 1M x 100K, 100M ratings (bench.synth), rank 64, linear kernel,
float32 (--dtype), strata schedule (--schedule exact: the reference's own
visit order, np.random.shuffle of the rows every epoch).  Phases are timed by wrapping the functions fit()
calls (preprocessing, normal() initialisation is the remainder, engine
upload + strata plan, SGD epochs incl. the RMSE passes, parameter download).
Usage: python tools/fit_walltime.py [--epochs 20] [--nnz 100000000]
       [--schedule strata|exact] [--dtype float32|float64]
"""

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "matrix-factorization_amd"))

import numpy as np
import pandas as pd
import torch

import bench
from matrix_factorization import KernelMF
from matrix_factorization import kernel_matrix_factorization as kmf
from matrix_factorization import recommender_base as rb
from matrix_factorization.engine import SGDEngine


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=20)
    ap.add_argument("--nnz", type=int, default=100_000_000)
    ap.add_argument("--users", type=int, default=1_000_000)
    ap.add_argument("--items", type=int, default=100_000)
    ap.add_argument("--schedule", default="strata", choices=["strata", "exact"])
    ap.add_argument("--dtype", default="float32", choices=["float32", "float64"])
    ap.add_argument("--pandas-prep", action="store_true",
                    help="force the pandas preprocessing path (reference-shaped)")
    args = ap.parse_args()
    if args.pandas_prep:
        rb.FAST_PREP_MIN_ROWS = 1 << 62
    t0 = time.perf_counter()
    u, i, r = bench.synth(args.users, args.items, args.nnz)
    X = pd.DataFrame({"user_id": u, "item_id": i})
    y = pd.Series(r.astype(np.float64))
    del u, i, r
    t_synth = time.perf_counter() - t0
    phases = {}
    marks = {}                       # wall-clock start / end of each wrapped phase

    def timed(name, fn, sync=True):
        def wrap(*a, **kw):
            if sync:
                torch.cuda.synchronize()
            t = time.perf_counter()
            marks.setdefault(name + "_start", t)
            out = fn(*a, **kw)
            if sync:
                torch.cuda.synchronize()
            marks[name + "_end"] = time.perf_counter()
            phases[name] = phases.get(name, 0.0) + time.perf_counter() - t
            return out
        return wrap

    KernelMF._preprocess_data = timed("preprocess", KernelMF._preprocess_data)
    # the native preprocessing calls (some run on worker threads: wall time of
    # each call, summed per function)
    from matrix_factorization import _prep
    import matrix_factorization.recommender_base as rbm
    calls = {}

    def timed_call(name, fn):
        def wrap(*a, **kw):
            t = time.perf_counter()
            out = fn(*a, **kw)
            calls[name] = calls.get(name, 0.0) + time.perf_counter() - t
            return out
        return wrap

    for name in ("legacy_permutation", "pairs_duplicated", "factorize", "gather"):
        setattr(_prep, name, timed_call(name, getattr(_prep, name)))
    rbm.RecommenderBase._fit_maps_native = timed_call(
        "fit_maps_native", rbm.RecommenderBase._fit_maps_native)
    # since round 4 the engine (upload, evaluation order, strata plan) is built
    # on a worker thread while fit() draws the initial factors
    KernelMF._make_engine = timed("engine_build_worker", KernelMF._make_engine)
    # per-epoch hipEvents on the launch stream (recorded by fit_epochs'
    # on_epoch hook: no synchronisation inside the loop)
    ep_events = []
    inner = kmf.fit_epochs

    def with_events(*a, **kw):
        ev0 = torch.cuda.Event(enable_timing=True)

        def on_epoch(ep):
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            ep_events.append(e)

        ev0.record()                            # the plan is built before fit_epochs
        out = inner(*a, on_epoch=on_epoch, **kw)
        ep_events.insert(0, ev0)
        return out

    exact = args.schedule == "exact"
    ep_wall = []
    if exact:
        # no on_epoch hook here: it would turn off the exact schedule's
        # pipelined shuffle (fit_epochs); the wall clock at each epoch's
        # epoch_exact call instead (no synchronisation)
        inner_ex = SGDEngine.epoch_exact

        def epoch_exact(self, *a, **kw):
            ep_wall.append(time.perf_counter())
            return inner_ex(self, *a, **kw)

        SGDEngine.epoch_exact = epoch_exact
        kmf.fit_epochs = timed("epochs", inner)
    else:
        kmf.fit_epochs = timed("epochs", with_events)
    SGDEngine.prepare_strata = timed("strata_plan", SGDEngine.prepare_strata)
    # the engine build's parts (no synchronisation: wall time of each call as
    # the host sees it, summed per function; the regrouping's run on the
    # worker thread beside the engine's own)
    import matrix_factorization.engine as eng_mod
    ecalls = {}
    timeline = []                    # (name, thread, start, end), seconds from fit()'s start
    import threading

    def timed_e(name, fn):
        def wrap(*a, **kw):
            t = time.perf_counter()
            out = fn(*a, **kw)
            t1 = time.perf_counter()
            ecalls[name] = ecalls.get(name, 0.0) + t1 - t
            timeline.append((name, threading.current_thread().name, t, t1))
            return out
        return wrap

    eng_mod.sched_strata = timed_e("sched_strata", eng_mod.sched_strata)
    eng_mod.sched_slices = timed_e("sched_slices", eng_mod.sched_slices)
    for name in ("normal",):
        setattr(np.random, name, timed_e(name, getattr(np.random, name)))
    eng_mod.StrataPlan.to_device = timed_e("plan_to_device", eng_mod.StrataPlan.to_device)
    for name in ("_build_regroup", "_regroup_buffers", "_prime_strata", "_ensure_strata_ws",
                 "_item_phases", "degree_cum", "__init__", "_upload_triples", "_build_eval"):
        setattr(SGDEngine, name, timed_e(name.strip("_"), getattr(SGDEngine, name)))
    SGDEngine.snapshot_params = timed("start_snapshot", SGDEngine.snapshot_params)
    KernelMF._sync_params = timed("download", KernelMF._sync_params)
    torch.zeros(1, device="cuda:0")
    m = KernelMF(n_factors=64, n_epochs=args.epochs, lr=0.01, reg=0.02, verbose=0,
                 min_rating=1, max_rating=5, dtype=args.dtype, schedule=args.schedule)
    np.random.seed(0)
    t = time.perf_counter()
    m.fit(X, y)
    total = time.perf_counter() - t
    epochs = phases["epochs"] - phases.get("start_snapshot", 0.0)
    # wall time from the end of preprocessing to the first epoch: the normal
    # draws on this thread beside the engine build on the worker
    phases["init_beside_engine_build"] = marks["epochs_start"] - marks["preprocess_end"]
    if exact:
        ep_wall.append(marks["epochs_end"])
        out = {"what": "KernelMF.fit wall time, schedule='exact' (the reference's visit "
                       "order: np.random.shuffle of the rows every epoch)",
               "nnz": args.nnz, "n_users": m.n_users, "n_items": m.n_items,
               "epochs": args.epochs, "dtype": args.dtype,
               "fit_s": round(total, 3), "epochs_s": round(phases["epochs"], 3),
               "epoch_s_mean": round(phases["epochs"] / args.epochs, 4),
               "epoch_wall_s": [round(b - a, 4) for a, b in zip(ep_wall[:-1], ep_wall[1:])],
               "epoch_wall_note": ("wall clock between consecutive epoch_exact calls (the "
                                   "last: to the end of fit_epochs, RMSE read-back "
                                   "included); epoch e+1's shuffle is drawn on a worker "
                                   "thread while epoch e's levels are built and launched"),
               "phases_s": {k: round(v, 3) for k, v in phases.items()},
               "prep_calls_s": {k: round(v, 3) for k, v in calls.items()},
               "engine_calls_s": {k: round(v, 3) for k, v in ecalls.items()},
               "engine_timeline_s": [(a, b, round(c - t, 3), round(d - t, 3)) for a, b, c, d in timeline],
               "final_train_rmse": float(m.train_rmse[-1]),
               "train_rmse": [float(x) for x in m.train_rmse],
               "host_threads": os.environ.get("MF_HOST_THREADS") or min(16, os.cpu_count()),
               "synth_s": round(t_synth, 1)}
        print(json.dumps(out))
        return
    ep_ms = [a.elapsed_time(b) for a, b in zip(ep_events[:-1], ep_events[1:])]
    # the bench's timed loop (bench.py: epoch_strata + sse_async, events
    # around the whole step) on the SAME engine and plan after fit(): tells
    # fit()'s loop apart from the data layout it trains on
    eng = m._pred_engine
    same = []
    for ep in range(10):
        a, m_, b = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        a.record()
        eng.epoch_strata(bench.strata_seq(ep, eng.strata), bench.strata_rot(ep), 0.01, 0.02)
        m_.record()
        eng.sse_async(ep)
        b.record()
        same.append((a, m_, b))
    torch.cuda.synchronize()
    same_ms = [a.elapsed_time(b) for a, _, b in same][1:]
    same_sgd = [a.elapsed_time(m_) for a, m_, _ in same][1:]
    same_sse = [m_.elapsed_time(b) for _, m_, b in same][1:]
    print(json.dumps({"what": "KernelMF.fit wall time", "nnz": args.nnz,
                      "n_users": m.n_users, "n_items": m.n_items, "epochs": args.epochs,
                      "prep_path": "pandas" if args.pandas_prep else "native",
                      "fit_s": round(total, 3),
                      "epochs_s": round(epochs, 4),
                      "epoch_ms": round(epochs / args.epochs * 1e3, 3),
                      "epoch_note": ("fit_epochs minus the one start snapshot: the epochs' SGD "
                                     "sweeps + RMSE passes + the final RMSE read-back, no "
                                     "per-epoch host sync"),
                      "phases_note": ("engine_build_worker (upload, evaluation order, strata_plan "
                                      "inside it) runs on a worker thread beside the initial "
                                      "normal draws; init_beside_engine_build is the wall time "
                                      "of both together"),
                      "phases_s": {k: round(v, 3) for k, v in phases.items()},
                      "prep_calls_s": {k: round(v, 3) for k, v in calls.items()},
                      "engine_calls_s": {k: round(v, 3) for k, v in ecalls.items()},
               "engine_timeline_s": [(a, b, round(c - t, 3), round(d - t, 3)) for a, b, c, d in timeline],
                      "epoch_ms_events": ep_ms,
                      "epoch_ms_events_note": ("hipEvents between consecutive epochs of "
                                               "fit_epochs (SGD sweep + RMSE pass each); "
                                               "epoch 1 includes the first launches"),
                      "epoch_ms_median_2_on": float(np.median(ep_ms[1:])) if len(ep_ms) > 1
                                              else None,
                      "bench_loop_same_engine_ms_median": float(np.median(same_ms)),
                      "bench_loop_sgd_ms_median": float(np.median(same_sgd)),
                      "bench_loop_rmse_ms_median": float(np.median(same_sse)),
                      "plan": {"B": int(eng.strata.B), "positions": int(eng.strata.n_positions),
                               "max_steps": int(np.diff(eng.strata.bstep).max())
                               if hasattr(eng.strata, "bstep") else None},
                      "bench_loop_note": ("bench.py's step (epoch_strata + sse_async) run 10x "
                                          "on fit()'s own engine and plan afterwards, epochs "
                                          "2-10"),
                      "final_train_rmse": float(m.train_rmse[-1]),
                      "P_contiguous": hasattr(eng.P, "_mf_block"),
                      "P_ptr": hex(eng.P.data_ptr()),
                      "synth_s": round(t_synth, 1)}))


if __name__ == "__main__":
    main()

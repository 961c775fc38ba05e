#!/usr/bin/env python
"""Same-process A/B of the strata plan's user-range classes C (DESIGN.md
section 2): with C > 1 the persistent sweep hands a user range over with C - 1
whole blocks of slack instead of waiting for the previous block.

For each dtype and C: engine + plan on the bench workload (bench.synth, the
bench's start and draws), --warmup untimed epochs, then --epochs timed ones:
SGD-phase ms (hipEvents around each epoch's launches), RMSE-pass ms, plan
build seconds, slot fill, steps, and the train RMSE after the epochs.  With
--worlds N: rank 0's rotation sub-epochs at N (distributed.RotationReplay,
every rank's sub-epoch timed alone; sweep = sum over sub-epochs of the
slowest rank).  One JSON document on stdout (or --out).
"""

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "matrix-factorization_amd"))
sys.path.insert(0, ROOT)


def log(msg):
    print(f"[classes_probe {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c3")
    ap.add_argument("--dtypes", nargs="+", default=["float32", "float64"])
    ap.add_argument("--classes", type=int, nargs="+", default=[1, 2, 3])
    ap.add_argument("--blocks", type=int, nargs="*", default=[None],
                    help="B values to sweep (default: the engine's rule)")
    ap.add_argument("--worlds", type=int, nargs="*", default=[])
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--epochs", type=int, default=8)
    ap.add_argument("--reps", type=int, default=1, help="repeat the C sweep (interleaved)")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()

    import torch

    import bench
    from matrix_factorization.distributed import RotationReplay
    from matrix_factorization.engine import SGDEngine

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    nu, ni, nnz, k, kernel, desc = bench.WORKLOADS[args.workload]
    u, i, r = bench.synth(nu, ni, nnz)
    mu = float(np.mean(r, dtype=np.float64))
    rs = np.random.RandomState(7)
    P0 = rs.normal(0.0, 0.1, (nu, k)).astype(np.float32)
    Q0 = rs.normal(0.0, 0.1, (ni, k)).astype(np.float32)
    hyp = dict(gamma=1.0 / k, min_rating=1.0, max_rating=5.0, global_mean=mu)
    doc = {"workload": desc, "warmup": args.warmup, "epochs": args.epochs, "runs": []}

    def ev():
        return torch.cuda.Event(enable_timing=True)

    n_ep = args.warmup + args.epochs
    for rep in range(args.reps):
        for dt in args.dtypes:
            for C, Bq in [(c, b) for c in args.classes for b in args.blocks]:
                t0 = time.time()
                e = SGDEngine(u, i, r, nu, ni, k, kernel, dt, dev, **hyp)
                e.load_params(P=P0, Q=Q0, bu=np.zeros(nu), bi=np.zeros(ni))
                pl = e.prepare_strata(n_blocks=Bq, classes=C)
                t_plan = time.time() - t0
                e._ensure_sse_slots(n_ep)
                ms = []
                for ep in range(n_ep):
                    a, b, c = ev(), ev(), ev()
                    a.record()
                    _, nl = e.epoch_strata(bench.strata_seq(ep, pl), bench.strata_rot(ep), 0.01,
                                           0.02, timing=True)
                    b.record()
                    e.sse_async(ep)
                    c.record()
                    torch.cuda.synchronize()
                    if ep >= args.warmup:
                        ms.append((a.elapsed_time(b), b.elapsed_time(c)))
                e.check_strata()
                rm = e.rmse_values(n_ep)
                ms = np.asarray(ms)
                n_ph = len(getattr(pl, "phases", [pl]))
                run = {"rep": rep, "dtype": dt, "classes": C, "B": pl.B, "phases": n_ph,
                       "l2_handoff": bool(getattr(pl, "l2_handoff", False)),
                       "NS": pl.NS, "launches_per_epoch": nl,
                       "slot_fill": nnz / pl.n_positions,
                       "steps_per_workgroup": float(np.sum(pl.n_steps) / pl.B),
                       "plan_s": t_plan, "sgd_ms": float(ms[:, 0].mean()),
                       "sgd_ms_min": float(ms[:, 0].min()), "rmse_ms": float(ms[:, 1].mean()),
                       "rmse_final": rm[-1]}
                doc["runs"].append(run)
                log(f"{dt} C={C}: B={pl.B} x{n_ph} fill {run['slot_fill']:.3f} steps/wg "
                    f"{run['steps_per_workgroup']:.0f} launches {nl}: SGD {run['sgd_ms']:.3f} ms "
                    f"(min {run['sgd_ms_min']:.3f}) RMSE {run['rmse_ms']:.3f} ms, plan "
                    f"{t_plan:.1f}s, rmse {rm[-1]:.7f}")
                del e
                torch.cuda.empty_cache()
            for W in args.worlds:
                for C in args.classes:
                    rp = RotationReplay(u, i, r, nu, ni, W, k, kernel, dt, dev,
                                        n_blocks=args.blocks[0], classes=C, **hyp)
                    rp.load(P0.astype(dt), Q0.astype(dt), np.zeros(nu), np.zeros(ni))
                    per = []
                    for ep in range(n_ep):
                        m = rp.epoch(bench.strata_rot(ep), 0.01, 0.02, timing=True, epoch=ep)
                        if ep >= args.warmup:
                            per.append(m)
                    sweeps = np.asarray([m.max(axis=1).sum() for m in per])
                    run = {"rep": rep, "dtype": dt, "classes": C, "world": W, "B": rp.B[0],
                           "sweep_ms": float(sweeps.mean()),
                           "sub_epoch_ms_mean": float(np.mean([m.mean() for m in per]))}
                    doc["runs"].append(run)
                    log(f"{dt} N={W} C={C} B={rp.B[0]}: rank sweep {run['sweep_ms']:.3f} ms "
                        f"(sub-epoch {run['sub_epoch_ms_mean']:.3f})")
                    del rp
                    torch.cuda.empty_cache()
    txt = json.dumps(doc)
    if args.out:
        os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
        with open(args.out, "w") as f:
            f.write(txt)
    print(txt)


if __name__ == "__main__":
    main()

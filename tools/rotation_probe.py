#!/usr/bin/env python
"""RMSE-vs-N and per-rank time of the multi-GPU schedules, rehearsed on ONE GPU.

For each N, the rotation schedule (distributed.RotationReplay: N user shards x
N item ranges, sub-epoch s runs every rank's sub-block (r, (r + off + s) mod N)
one after another) trains the bench workload from the bench's start for
--epochs epochs; because the sub-blocks of a sub-epoch share no user and no
item, this is bit for bit what N GPUs compute, and each rank's sub-epoch is
timed alone on the whole GPU, as on its own card.  The N = 1 single-GPU
default schedule runs beside it for the RMSE gap.

Per epoch and N the line reports
  sweep_ms     sum over sub-epochs of the slowest rank's sub-epoch kernel time
               (a real run waits for the slowest rank at every hand-off);
  rmse_ms      the slowest rank's training-RMSE pass (its shard, full replica);
  pass_model_ms / gather_model_ms   the xGMI transfers, NOT measured here (one
               GPU): (N - 1) ring hand-offs of one item range and one
               all-gather, priced at --link-gbs per direction plus
               --latency-us per transfer (the driver's N-GPU bench line
               measures them: phases.ring_pass_ms_per_epoch / gather_ms).
Writes one JSON document (stdout, or --out).
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
    print(f"[rotation_probe {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c3")
    ap.add_argument("--worlds", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--epochs", type=int, default=20)
    ap.add_argument("--blocks", type=int, nargs="*", default=[],
                    help="B values per rank to sweep (none = the default rule)")
    ap.add_argument("--waves", type=int, default=None)
    ap.add_argument("--lr", type=float, default=0.01)
    ap.add_argument("--reg", type=float, default=0.02)
    ap.add_argument("--link-gbs", type=float, default=64.0)
    ap.add_argument("--latency-us", type=float, default=15.0)
    ap.add_argument("--no-n1", action="store_true")
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
    P0 = rs.normal(0.0, 0.1, (nu, k)).astype("float32")
    Q0 = rs.normal(0.0, 0.1, (ni, k)).astype("float32")
    hyp = dict(gamma=1.0 / k, min_rating=1.0, max_rating=5.0, global_mean=mu)
    doc = {"workload": desc, "epochs": args.epochs, "lr": args.lr, "reg": args.reg,
           "link_model": {"gbs_per_direction": args.link_gbs, "latency_us": args.latency_us},
           "runs": []}

    def ev():
        return torch.cuda.Event(enable_timing=True)

    if not args.no_n1:
        log("N=1: single-GPU default schedule")
        e1 = SGDEngine(u, i, r, nu, ni, k, kernel, "float32", dev, **hyp)
        e1.load_params(P=P0, Q=Q0, bu=np.zeros(nu), bi=np.zeros(ni))
        pl = e1.prepare_strata()
        ms, rm = [], []
        for ep in range(args.epochs):
            a, b, c = ev(), ev(), ev()
            a.record()
            e1.epoch_strata(bench.strata_seq(ep, pl.B), bench.strata_rot(ep), args.lr, args.reg)
            b.record()
            e1.sse_async(ep)
            c.record()
            torch.cuda.synchronize()
            ms.append((a.elapsed_time(b), b.elapsed_time(c)))
        rm = e1.rmse_values(args.epochs)
        ms = np.asarray(ms[1:])
        doc["runs"].append({"world": 1, "schedule": "single-GPU default", "B": pl.B,
                            "sweep_ms": float(ms[:, 0].mean()), "rmse_ms": float(ms[:, 1].mean()),
                            "epoch_ms": float(ms.sum(1).mean()), "rmse": rm})
        log(f"N=1 sweep {ms[:, 0].mean():.3f} ms rmse {ms[:, 1].mean():.3f} ms final {rm[-1]:.6f}")
        del e1
        torch.cuda.empty_cache()

    blocks = list(args.blocks) or [None]
    for W in args.worlds:
        for B in blocks:
            t0 = time.time()
            rp = RotationReplay(u, i, r, nu, ni, W, k, kernel, "float32", dev, n_blocks=B,
                                waves=args.waves, **hyp)
            t_plan = time.time() - t0
            rp.load(P0, Q0, np.zeros(nu), np.zeros(ni))
            per_ep, rmse = [], []
            for ep in range(args.epochs):
                m = rp.epoch(bench.strata_rot(ep), args.lr, args.reg, timing=True, epoch=ep)
                sse, sms = 0.0, []
                for e in rp.engines:
                    a, b = ev(), ev()
                    a.record()
                    e.sse_async(ep)
                    b.record()
                    torch.cuda.synchronize()
                    sms.append(a.elapsed_time(b))
                    sse += float(e.sse_values(ep + 1)[ep])
                rmse.append(float(np.sqrt(sse / nnz)))
                per_ep.append((m, sms))
            # drop the first epoch (first-touch of the plans / code objects)
            sweeps = np.asarray([m.max(axis=1).sum() for m, _ in per_ep[1:]])
            rank_sum = np.asarray([m.sum(axis=0) for m, _ in per_ep[1:]])
            rms = np.asarray([max(s) for _, s in per_ep[1:]])
            ts = 4
            rows = int(np.diff(rp.ilo).max())
            slab = rows * (k + 1) * ts
            pass_ms = (W - 1) * (slab / (args.link_gbs * 1e9) * 1e3 + args.latency_us / 1e3)
            gather_ms = ((W - 1) * slab / (args.link_gbs * 1e9 * min(W - 1, 7)) * 1e3
                         + args.latency_us / 1e3)
            pl0 = rp.engines[0].strata
            run = {"world": W, "schedule": "rotate", "B": rp.B, "NS": pl0.NS,
                   "slot_fill": float(sum(e.n for e in rp.engines)
                                      / sum(e.strata.n_positions for e in rp.engines)),
                   "plan_s": t_plan,
                   "sweep_ms": float(sweeps.mean()),
                   "sweep_ms_rank_mean": float(rank_sum.mean()),
                   "sub_epoch_ms_mean": float(np.mean([m.mean() for m, _ in per_ep[1:]])),
                   "rmse_ms": float(rms.mean()),
                   "pass_model_ms": pass_ms, "gather_model_ms": gather_ms,
                   "epoch_ms_est": float(sweeps.mean() + rms.mean() + pass_ms + gather_ms),
                   "rmse": rmse}
            if doc["runs"] and doc["runs"][0]["world"] == 1:
                n1 = doc["runs"][0]
                run["rmse_gap_vs_n1"] = rmse[-1] - n1["rmse"][-1]
                run["speedup_est_vs_n1"] = n1["epoch_ms"] / run["epoch_ms_est"]
            doc["runs"].append(run)
            log(f"N={W} B={rp.B[0]}: sweep {run['sweep_ms']:.3f} ms (sub-epoch "
                f"{run['sub_epoch_ms_mean']:.3f}), rmse {run['rmse_ms']:.3f} ms, est epoch "
                f"{run['epoch_ms_est']:.3f} ms, final rmse {rmse[-1]:.6f}"
                + (f" gap {run['rmse_gap_vs_n1']:+.2e} x{run['speedup_est_vs_n1']:.2f}"
                   if "rmse_gap_vs_n1" in run else ""))
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

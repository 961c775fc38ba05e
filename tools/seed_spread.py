#!/usr/bin/env python
"""How far apart do two equally valid SGD orders end after E epochs?

The reference's own visit order is random every run (numba's shuffle is
seeded from os.urandom: SURVEY 8(c)), so its final training RMSE has a
run-to-run spread; a build's RMSE "matches the reference" only up to that.
This probe measures it on the bench workload, from the bench's start
(bench.synth, RandomState(7) normals, zero biases), all on one GPU in FP32:

  exact    the reference's order: np.random.shuffle of the rating rows every
           epoch (kernel_matrix_factorization.py:369-371), applied exactly
           (level schedule, engine.epoch_exact) -- one run per --shuffle-seeds
           entry (np.random.seed(s) before the first epoch);
  strata   the single-GPU throughput schedule, one run per --draw-seeds entry
           (stratum orders and rotations drawn from that seed);
  rotate   the N-GPU rotation order (distributed.RotationReplay), one run per
           --draw-seeds entry, for each N in --worlds.

Prints / writes one JSON document: per run the RMSE of every epoch; per
family the spread (max - min) of the final RMSE and the mean.
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
    print(f"[seed_spread {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def summarize(runs):
    """Per family and epoch: mean, sample SD, standard error of the mean; per
    non-reference family the difference of means to the reference order
    ("exact") with its standard error sqrt(se_a^2 + se_b^2)."""
    fam = {}
    for run in runs:
        fam.setdefault(run["family"], []).append(run["rmse"])
    stats = {}
    for f, v in fam.items():
        a = np.asarray(v, dtype=np.float64)                 # runs x epochs
        n = a.shape[0]
        sd = a.std(axis=0, ddof=1) if n > 1 else np.full(a.shape[1], np.nan)
        stats[f] = {"n": n, "mean": a.mean(axis=0).tolist(), "sd": sd.tolist(),
                    "se": (sd / np.sqrt(n)).tolist()}
    diff = {}
    if "exact" in stats:
        ref = stats["exact"]
        for f, st in stats.items():
            if f == "exact":
                continue
            d = np.asarray(st["mean"]) - np.asarray(ref["mean"])
            se = np.sqrt(np.asarray(st["se"]) ** 2 + np.asarray(ref["se"]) ** 2)
            diff[f] = {"minus_exact": d.tolist(), "se": se.tolist(),
                       "z": (d / se).tolist()}
    final = {f: {"n": st["n"], "mean_final": st["mean"][-1], "sd_final": st["sd"][-1],
                 "se_final": st["se"][-1],
                 "finals": [r[-1] for r in fam[f]],
                 "spread_final": float(np.max([r[-1] for r in fam[f]]) -
                                       np.min([r[-1] for r in fam[f]]))}
             for f, st in stats.items()}
    for f, d in diff.items():
        final[f].update(minus_exact=d["minus_exact"][-1], se_diff=d["se"][-1],
                        z=d["z"][-1])
    return {"final": final, "per_epoch": stats, "vs_exact": diff}


def merge(paths, out):
    """Combine the runs of several seed_spread outputs (same workload, epochs)."""
    runs, head = [], None
    for p in paths:
        with open(p) as f:
            d = json.load(f)
        head = head or {k: d[k] for k in ("workload", "epochs", "lr", "reg")}
        runs += d["runs"]
    doc = dict(head, summary=summarize(runs), runs=runs, merged_from=paths)
    with open(out, "w") as f:
        json.dump(doc, f)
    print(json.dumps(doc["summary"]["final"], indent=1))


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--merge":
        return merge(sys.argv[3:], sys.argv[2])
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c3")
    ap.add_argument("--epochs", type=int, default=20)
    ap.add_argument("--shuffle-seeds", type=int, nargs="*", default=[7, 8])
    ap.add_argument("--draw-seeds", type=int, nargs="*", default=[0, 1, 2])
    ap.add_argument("--worlds", type=int, nargs="*", default=[8])
    ap.add_argument("--lr", type=float, default=0.01)
    ap.add_argument("--reg", type=float, default=0.02)
    ap.add_argument("--out", default=None)
    ap.add_argument("--dtype", default="float32")
    ap.add_argument("--variants", nargs="*", default=["C1"],
                    help="strata plan variants (the engine's relabelled plans apply as in the "
                         "product: 2 with C > 1 and the linear kernel unless "
                         "MF_STRATA_REGROUP=1): C<n> = n user-range classes, B<n> = n "
                         "blocks, joined with '_' (C2_B128); family strata_<variant> "
                         "(C1: family 'strata')")
    args = ap.parse_args()

    import torch

    import bench
    from matrix_factorization import _prep
    from matrix_factorization.distributed import RotationReplay
    from matrix_factorization.engine import SGDEngine, stratum_order

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    nu, ni, nnz, k, kernel, desc = bench.WORKLOADS[args.workload]
    u, i, r = bench.synth(nu, ni, nnz)
    mu = float(np.mean(r, dtype=np.float64))
    rs = np.random.RandomState(7)
    P0 = rs.normal(0.0, 0.1, (nu, k)).astype("float32")
    Q0 = rs.normal(0.0, 0.1, (ni, k)).astype("float32")
    hyp = dict(gamma=1.0 / k, min_rating=1.0, max_rating=5.0, global_mean=mu)
    E = args.epochs
    runs = []

    def fresh():
        e = SGDEngine(u, i, r, nu, ni, k, kernel, args.dtype, dev, **hyp)
        e.load_params(P=P0, Q=Q0, bu=np.zeros(nu), bi=np.zeros(ni))
        return e

    for s in args.shuffle_seeds:
        t0 = time.time()
        e = fresh()
        np.random.seed(s)
        order = np.arange(nnz, dtype=np.int32)     # (32-bit: the chunked level builder)
        for ep in range(E):
            _prep.legacy_shuffle_(order)           # = np.random.shuffle(order), :371
            e.epoch_exact(order, args.lr, args.reg)
            e.sse_async(ep)
            if ep % 5 == 4:
                log(f"exact seed {s}: epoch {ep + 1}/{E} ({time.time() - t0:.0f}s)")
        rm = e.rmse_values(E)
        runs.append({"family": "exact", "seed": s, "rmse": rm, "s": time.time() - t0,
                     "dtype": args.dtype})
        log(f"exact seed {s}: final {rm[-1]:.7f} in {time.time() - t0:.0f}s")
        del e
        torch.cuda.empty_cache()

    def regrouped(opt, fam):
        """K groupings: K engines over randomly relabelled users and items
        (engine 0: the identity), each with its own strata plan; every epoch
        draws which one runs, and the parameters move to its labelling
        (device gathers) -- a probe of re-drawing which users and items share
        a block, before any product support."""
        K = opt["K"]
        rk = np.random.RandomState(424242)
        perms = [(np.arange(nu), np.arange(ni))] + [(rk.permutation(nu), rk.permutation(ni))
                                                    for _ in range(K - 1)]
        engines = []
        for pu, pi in perms:
            e = SGDEngine(pu[u].astype(np.int32), pi[i].astype(np.int32), r, nu, ni, k, kernel,
                          args.dtype, dev, **hyp)
            e.prepare_strata(n_blocks=opt["B"], classes=opt["C"])
            e.load_params(P=P0, Q=Q0, bu=np.zeros(nu), bi=np.zeros(ni))
            engines.append(e)
        dperm = [(torch.from_numpy(pu).to(dev), torch.from_numpy(pi).to(dev)) for pu, pi in perms]
        out = []
        for s in args.draw_seeds:
            e0 = engines[0]
            e0.load_params(P=P0, Q=Q0, bu=np.zeros(nu), bi=np.zeros(ni))
            cur, rm = 0, []
            for ep in range(E):
                rsd = np.random.RandomState([s, ep])
                kk = int(rsd.randint(0, K))
                if kk != cur:      # row of original user x: pu_cur[x] -> pu_kk[x]
                    a, b = engines[cur], engines[kk]
                    (pu_a, pi_a), (pu_b, pi_b) = dperm[cur], dperm[kk]
                    b.P[pu_b] = a.P[pu_a]
                    b.bu[pu_b] = a.bu[pu_a]
                    b.Q[pi_b] = a.Q[pi_a]
                    b.bi[pi_b] = a.bi[pi_a]
                    cur = kk
                e = engines[cur]
                e.epoch_strata(stratum_order(rsd, e.strata), int(rsd.randint(0, 2**31 - 1)),
                               args.lr, args.reg)
                e.sse_async(ep)
                rm.append(e.rmse_values(ep + 1)[ep])
            out.append({"family": fam, "seed": s, "rmse": rm, "dtype": args.dtype, "K": K,
                        "B": engines[0].strata.B, "classes": engines[0].strata.classes})
            log(f"{fam} (K={K}) seed {s}: final {rm[-1]:.7f}")
        del engines
        torch.cuda.empty_cache()
        return out

    for var in args.variants:
        opt = {"C": 1, "B": None, "K": 1}
        for part in var.split("_"):
            opt[part[0]] = int(part[1:])
        fam = "strata" if var == "C1" else f"strata_{var}"
        if opt["K"] > 1:
            runs += regrouped(opt, fam)
            continue
        for s in args.draw_seeds:
            e = fresh()
            pl = e.prepare_strata(n_blocks=opt["B"], classes=opt["C"])
            for ep in range(E):
                rsd = np.random.RandomState([s, ep])
                e.epoch_strata(stratum_order(rsd, pl),
                               int(rsd.randint(0, 2**31 - 1)), args.lr, args.reg)
                e.sse_async(ep)
            rm = e.rmse_values(E)
            runs.append({"family": fam, "seed": s, "rmse": rm, "dtype": args.dtype,
                         "B": pl.B, "classes": pl.classes})
            log(f"{fam} (B={pl.B}, C={pl.classes}) seed {s}: final {rm[-1]:.7f}")
            del e
            torch.cuda.empty_cache()

    for W in args.worlds:
        rp = RotationReplay(u, i, r, nu, ni, W, k, kernel, "float32", dev, **hyp)
        for s in args.draw_seeds:
            rp.load(P0, Q0, np.zeros(nu), np.zeros(ni))
            rm = []
            for ep in range(E):
                rp.epoch(int(np.random.RandomState([s, ep, W]).randint(0, 2**31 - 1)),
                         args.lr, args.reg, epoch=ep)
                rm.append(float(np.sqrt(rp.sse(ep) / nnz)))
            runs.append({"family": f"rotate_n{W}", "seed": s, "rmse": rm})
            log(f"rotate N={W} seed {s}: final {rm[-1]:.7f}")
        del rp
        torch.cuda.empty_cache()

    doc = {"workload": desc, "epochs": E, "lr": args.lr, "reg": args.reg,
           "summary": summarize(runs), "runs": runs}
    txt = json.dumps(doc)
    if args.out:
        with open(args.out, "w") as f:
            f.write(txt)
    print(txt)
    log(json.dumps(doc["summary"]["final"]))


if __name__ == "__main__":
    main()

#!/usr/bin/env python
"""Does the strata schedule's visit order bias the training RMSE against the
reference's random order?  A CPU study with the FP64 oracle (the reference's
per-rating arithmetic, oracle/mf_oracle.c -- test infrastructure, run here
only as the thing being studied, not as a product path).

A C3-like problem scaled down 10x in users and items -- 100K users, 10K
items, 10M ratings (100 per user, 1000 per item, as at C3), rank 64, lr 0.01,
reg 0.02 -- so that a strata plan with B = 256 has C3's per-block statistics
(~3.9 ratings per item and ~0.4 per user in a block).  Each arm trains from
the same start for --epochs epochs, one run per seed, orders:
  shuffle        np.random.shuffle of the rows every epoch (the reference,
                 kernel_matrix_factorization.py:369-371)
  strata         the product's plan (engine.sched_strata, built once) in
                 StrataPlan.serial_order of stratum_order + rotation draws
  strata_Bn      the same with B = n
  strata_regrid  a fresh plan every epoch over randomly relabelled users and
                 items (so the blocks group different users / items each epoch)
  strata_Cn      n user-range classes
  strata_Kn      n plans over n fixed random relabellings of users and items,
                 one drawn per epoch
  strata_affine  the fixed plan, but each block's steps in a random affine
                 order (a t + b) mod n_steps per epoch instead of a rotation
Runs go to a process pool (one thread each).  Writes per run the RMSE of the
--record epochs; the summary has per arm and epoch mean, SD, SE and the
difference to shuffle with its SE.
"""

import argparse
import json
import os
import sys
import time
from concurrent.futures import ProcessPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "matrix-factorization_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, ROOT)

G = {}


def log(msg):
    print(f"[order_bias {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def setup(nu, ni, nnz, k, kernel="linear"):
    import bench
    u, i, r = bench.synth(nu, ni, nnz)
    rs = np.random.RandomState(7)
    G.update(u=u, i=i, r=r.astype(np.float64), nu=nu, ni=ni, k=k, kernel=kernel,
             P0=rs.normal(0, 0.1, (nu, k)), Q0=rs.normal(0, 0.1, (ni, k)),
             mu=float(np.mean(r, dtype=np.float64)))


def plan_for(u, i, nu, ni, B, C=1):
    from matrix_factorization.engine import StrataPlan, balanced_bounds, sched_strata
    ub = balanced_bounds(u, nu, C * B)
    ib = balanced_bounds(i, ni, B)
    sched, bstep = sched_strata(u, i, nu, ni, B, ub, ib, 128, C)
    return StrataPlan(B, 128, ub, ib, bstep, sched, C)


def affine_order(plan, seq, rs):
    """plan.serial_order with each block's steps in the order (a t + b) mod
    n, a coprime to n, drawn per block."""
    from math import gcd
    B, NS = plan.B, plan.NS
    out = []
    for s in seq:
        for w in range(B):
            blk = int(s) * B + w
            st0 = int(plan.bstep[blk])
            nst = int(plan.bstep[blk + 1]) - st0
            if nst <= 0:
                continue
            while True:
                a = int(rs.randint(1, nst + 1))
                if gcd(a, nst) == 1:
                    break
            b = int(rs.randint(0, nst))
            steps = (a * np.arange(nst) + b) % nst
            grid = plan.sched[st0 * NS:(st0 + nst) * NS].reshape(nst, NS)[steps].ravel()
            out.append(grid[grid >= 0])
    return np.concatenate(out).astype(np.int64)


def run(job):
    import oracle
    from matrix_factorization.engine import stratum_order
    arm, seed, epochs, record, lr, reg = job
    u, i, r, nu, ni = G["u"], G["i"], G["r"], G["nu"], G["ni"]
    P, Q = G["P0"].copy(), G["Q0"].copy()
    bu, bi = np.zeros(nu), np.zeros(ni)
    mu = G["mu"]
    B, C, K = G.get("B", 256), 1, 0
    for part in arm.split("_")[1:]:
        if part[0] == "B":
            B = int(part[1:])
        elif part[0] == "C":
            C = int(part[1:])
        elif part[0] == "K":
            K = int(part[1:])
    plan = None
    if arm.startswith("strata") and "regrid" not in arm and not K:
        plan = plan_for(u, i, nu, ni, B, C)
    plans = []
    if K:
        rk = np.random.RandomState(1000 + seed)
        for _ in range(K):
            pu, pi = rk.permutation(nu).astype(np.int32), rk.permutation(ni).astype(np.int32)
            plans.append(plan_for(pu[u], pi[i], nu, ni, B, C))
    out = {}
    order = np.arange(len(u), dtype=np.int64)
    rs = np.random.RandomState(seed)
    t0 = time.time()
    for ep in range(epochs):
        if arm == "shuffle":
            rs.shuffle(order)
            o = order
        elif K:
            pl = plans[int(rs.randint(0, K))]
            o = pl.serial_order(stratum_order(rs, pl), int(rs.randint(0, 2**31 - 1)))
        elif "affine" in arm:
            rsd = np.random.RandomState([seed, ep])
            o = affine_order(plan, stratum_order(rsd, plan), rsd)
        elif "regrid" in arm:
            pu, pi = rs.permutation(nu).astype(np.int32), rs.permutation(ni).astype(np.int32)
            pl = plan_for(pu[u], pi[i], nu, ni, B, C)
            o = pl.serial_order(stratum_order(rs, pl), int(rs.randint(0, 2**31 - 1)))
        else:
            rsd = np.random.RandomState([seed, ep])
            o = plan.serial_order(stratum_order(rsd, plan), int(rsd.randint(0, 2**31 - 1)))
        hyp = dict(kernel=G["kernel"], gamma=1.0 / G["k"], min_rating=1.0, max_rating=5.0)
        oracle.sgd_pass(u, i, r, mu, bu, bi, P, Q, lr=lr, reg=reg, order=o, **hyp)
        if ep + 1 in record:
            out[ep + 1] = oracle.rmse(u, i, r, mu, bu, bi, P, Q, **hyp)
    return {"arm": arm, "seed": seed, "rmse": out, "s": time.time() - t0}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arms", nargs="+", default=["shuffle", "strata"])
    ap.add_argument("--seeds", type=int, default=8)
    ap.add_argument("--seed0", type=int, default=0, help="first seed")
    ap.add_argument("--epochs", type=int, default=20)
    ap.add_argument("--record", type=int, nargs="+", default=[1, 5, 10, 15, 20])
    ap.add_argument("--users", type=int, default=100_000)
    ap.add_argument("--items", type=int, default=10_000)
    ap.add_argument("--nnz", type=int, default=10_000_000)
    ap.add_argument("--k", type=int, default=64)
    ap.add_argument("--kernel", default="linear")
    ap.add_argument("--blocks", type=int, default=256, help="B of the strata arms")
    ap.add_argument("--workers", type=int, default=8)
    ap.add_argument("--out", default=None)
    ap.add_argument("--merge", nargs="*", default=None,
                    help="summarise these outputs together instead of running")
    args = ap.parse_args()
    if args.merge:
        runs = []
        for f in args.merge:
            with open(f) as fh:
                runs += json.load(fh)["runs"]
        args.arms = sorted({x["arm"] for x in runs}, key=lambda a: (a != "shuffle", a))
        for x in runs:
            x["rmse"] = {int(k): v for k, v in x["rmse"].items()}
        return summarize(args, runs)
    setup(args.users, args.items, args.nnz, args.k, args.kernel)
    G["B"] = args.blocks
    import oracle
    oracle.lib()                                   # build / load before forking
    jobs = [(a, s, args.epochs, set(args.record), 0.01, 0.02)
            for s in range(args.seed0, args.seed0 + args.seeds) for a in args.arms]
    runs = []
    with ProcessPoolExecutor(args.workers) as ex:
        for res in ex.map(run, jobs):
            runs.append(res)
            log(f"{res['arm']} seed {res['seed']}: {res['rmse'][args.epochs]:.7f} "
                f"({res['s']:.0f}s)")
    summarize(args, runs)


def summarize(args, runs):
    summ = {}
    for a in args.arms:
        rows = [[x["rmse"][e] for e in args.record] for x in runs if x["arm"] == a]
        m = np.asarray(rows)
        summ[a] = {"n": len(rows), "mean": m.mean(0).tolist(),
                   "sd": m.std(0, ddof=1).tolist() if len(rows) > 1 else None,
                   "se": (m.std(0, ddof=1) / np.sqrt(len(rows))).tolist() if len(rows) > 1
                   else None}
    ref = summ.get("shuffle")
    if ref is not None:
        for a, st in summ.items():
            if a == "shuffle" or st["se"] is None:
                continue
            d = np.asarray(st["mean"]) - np.asarray(ref["mean"])
            se = np.sqrt(np.asarray(st["se"]) ** 2 + np.asarray(ref["se"]) ** 2)
            st["minus_shuffle"] = d.tolist()
            st["z"] = (d / se).tolist()
    doc = {"what": __doc__.split("\n")[0], "users": args.users, "items": args.items,
           "nnz": args.nnz, "k": args.k, "epochs": args.epochs, "record": args.record,
           "summary": summ, "runs": runs}
    txt = json.dumps(doc)
    if args.out:
        with open(args.out, "w") as f:
            f.write(txt)
    for a, st in summ.items():
        log(f"{a}: mean {['%.6f' % x for x in st['mean']]} "
            + (f"minus shuffle {['%+.1e' % x for x in st['minus_shuffle']]} "
               f"z {['%+.1f' % x for x in st['z']]}" if "z" in st else ""))


if __name__ == "__main__":
    main()

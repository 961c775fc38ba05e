#!/usr/bin/env python
"""C4 (8 GPUs) speed / RMSE frontier of the multi-GPU exchange designs,
rehearsed on ONE GPU.

Every design runs N virtual ranks one after another on the one GPU -- the
same user shards, plans and draws real ranks would use, sharing one item
replica -- so the RMSE after each epoch is what N GPUs would compute, and
each rank's sweep is timed alone (its own GPU's kernel time).  Workload,
start and hyper-parameters are seed_spread.py's (bench.synth C3, N(0, 0.1)
RandomState(7) FP32 start, lr 0.01, reg 0.02, FP32), so the final RMSE
compares with the reference-order runs of profiles/r04/seed_spread_*
(family "exact", passed with --ref).

Designs (--designs, any of):
  rotate              the product's default (distributed.RotationReplay): items
                      cut into N ranges passed round the ring, N sub-epochs,
                      every update sees current rows (a sequential order);
  rotcls<M>           the rotation with M rounds over user classes: each
                      shard's users cut into M contiguous classes; round j
                      runs the N sub-epochs over class j only, so an item
                      meets its ratings in M*N bursts instead of N;
  rotrel<K>           the rotation over K item relabellings, one drawn per
                      epoch (which items share a range changes epoch to
                      epoch; the ranges are all-gathered anyway);
  rotcls<M>rel<K>     both of the above;
  rotprod<K>          the PRODUCT path: distributed.RotationReplay with K item
                      relabellings (relabel_pick of each epoch's draw, the
                      replica moved between labellings) -- the bench / fit
                      default since round 6 is rotprod8;
  rotc<C>[b<B>]       the rotation with sub-block plans of C user-range classes
                      (and B blocks): the stream kernel applies from C = 2;
  delta<M>s<S>        user-sharded replicas, the stratum order of each rank's
                      epoch cut into M rounds; after every round the item
                      deltas of all ranks are summed (all_reduce) and added
                      to the replica scaled by S (S = d: the product's default
                      min(1/2, 2/N)).  Items lag by 1/M epoch.

Per-rank time = the sum over the design's sequential steps (rounds,
sub-epochs) of the slowest rank's sweep (hipEvents, measured), plus the
exchange priced by a model (no xGMI here): a ring all-reduce of the
n_items x (k+1) FP32 replica at --busbw GB/s bus bandwidth + 25 us per
collective, a ring pass of n_items/N rows at --linkbw GB/s + 15 us, the
all-gather of the final ranges likewise; plus the RMSE pass over the rank's
shard (measured, rank 0).  The N = 1 default epoch (SGD + RMSE) is measured
in the same process: projected x = N1 epoch / per-rank epoch.

Usage: python tools/frontier_probe.py --designs rotate delta1sd delta4s1 ...
       [--draw-seeds 0 1 ... 7] [--epochs 20] [--ref a.json b.json] [--out f.json]
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
    print(f"[frontier {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c3")
    ap.add_argument("--epochs", type=int, default=20)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--draw-seeds", type=int, nargs="*", default=list(range(8)))
    ap.add_argument("--designs", nargs="*", default=["rotate", "delta1sd", "delta4s1"])
    ap.add_argument("--busbw", type=float, default=300.0,
                    help="all-reduce bus bandwidth, GB/s (model)")
    ap.add_argument("--linkbw", type=float, default=64.0,
                    help="one xGMI link, one direction, GB/s (model)")
    ap.add_argument("--ref", nargs="*", default=[],
                    help="seed_spread outputs holding 'exact' (reference-order) runs")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()

    import torch

    import bench
    from matrix_factorization.distributed import (RotationReplay, default_delta_scale,
                                                  item_ranges, rotation_draws,
                                                  rotation_offset, rotation_range,
                                                  shard_users)
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
    W, E, lr, reg = args.world, args.epochs, 0.01, 0.02
    replica_mb = ni * (k + 1) * 4 / 1e6

    def t_allreduce():
        return 2 * (W - 1) / W * replica_mb / 1e3 / args.busbw * 1e3 + 0.025     # ms

    def t_pass(rows):
        return rows * (k + 1) * 4 / 1e9 / args.linkbw * 1e3 + 0.015               # ms

    def ev():
        return torch.cuda.Event(enable_timing=True)

    # ---- N = 1: the default single-GPU epoch (SGD + RMSE), for the projection
    e1 = SGDEngine(u, i, r, nu, ni, k, kernel, "float32", dev, **hyp)
    pl = e1.prepare_strata()
    e1.load_params(P=P0, Q=Q0, bu=np.zeros(nu), bi=np.zeros(ni))
    ts = []
    for ep in range(6):
        a, b = ev(), ev()
        a.record()
        rsd = np.random.RandomState([99, ep])
        e1.epoch_strata(stratum_order(rsd, pl), int(rsd.randint(0, 2**31 - 1)), lr, reg)
        e1.sse_async(ep)
        b.record()
        ts.append((a, b))
    torch.cuda.synchronize()
    n1_ms = float(np.median([a.elapsed_time(b) for a, b in ts[2:]]))
    log(f"N=1 default epoch {n1_ms:.3f} ms (B={pl.B}, C={pl.classes})")
    del e1
    torch.cuda.empty_cache()

    bounds = shard_users(u, nu, W)
    ilo = item_ranges(i, ni, W)
    runs, timing = [], {}

    def shard_engines(sub=1):
        """(rank, class) -> engine over that part of the rank's users (sub
        contiguous classes per shard, balanced by ratings)."""
        out = {}
        for rank in range(W):
            lo, hi = int(bounds[rank]), int(bounds[rank + 1])
            m = (u >= lo) & (u < hi)
            us, is_, rs_ = u[m] - lo, i[m], r[m]
            cb = shard_users(us, hi - lo, sub)
            for j in range(sub):
                a, b = int(cb[j]), int(cb[j + 1])
                mm = (us >= a) & (us < b)
                out[(rank, j)] = (lo + a, lo + b, us[mm] - a, is_[mm], rs_[mm])
        return out

    # ------------------------------------------------------------- designs
    def run_rotate(name, sub=1, relabel=1, classes=None, blocks=None):
        parts = shard_engines(sub)
        perms = [np.arange(ni)] + [np.random.RandomState(5150 + q).permutation(ni)
                                   for q in range(relabel - 1)]
        sets = []                       # per relabelling: {(rank, j): engine}
        for q, pi in enumerate(perms):
            engs = {}
            for key, (a, b, us, is_, rs_) in parts.items():
                e = SGDEngine(us, pi[is_].astype(np.int32), rs_, b - a, ni, k, kernel, "float32",
                              dev, **hyp)
                e.prepare_strata(n_blocks=blocks,
                                 item_bounds=item_ranges(pi[i].astype(np.int32), ni, W),
                                 classes=classes)
                engs[key] = e
            sets.append(engs)
        dpi = [torch.from_numpy(p).to(dev) for p in perms]
        e00 = sets[0][(0, 0)]
        for q in range(1, relabel):      # every set shares the P / b_u tensors of set 0
            for key, e in sets[q].items():
                e.P, e.bu = sets[0][key].P, sets[0][key].bu
        Qc = torch.empty((ni, k), dtype=torch.float32, device=dev)
        bic = torch.empty(ni, dtype=torch.float32, device=dev)
        sweep = []
        for s in args.draw_seeds:
            for key, (a, b, *_ ) in parts.items():
                sets[0][key].load_params(P=P0[a:b], bu=np.zeros(b - a))
                for q in range(1, relabel):
                    sets[q][key].P, sets[q][key].bu = sets[0][key].P, sets[0][key].bu
            Qc.copy_(torch.from_numpy(Q0))
            bic.zero_()
            rm = []
            for ep in range(E):
                draw = int(np.random.RandomState([s, ep, W]).randint(0, 2**31 - 1))
                q = int(np.random.RandomState([s, ep, 77]).randint(0, relabel))
                engs = sets[q]
                e0 = engs[(0, 0)]
                if e0.Q is None:
                    e0.load_params(Q=Q0, bi=np.zeros(ni))
                e0.Q[dpi[q]] = Qc
                e0.bi[dpi[q]] = bic
                for e in engs.values():
                    e.Q, e.bi = e0.Q, e0.bi
                off = rotation_offset(ep, W)
                t_ep = 0.0
                for j in range(sub):
                    dj = int(np.random.RandomState([draw, j]).randint(0, 2**31 - 1)) if sub > 1 \
                        else draw
                    for st in range(W):
                        worst = 0.0
                        for rank in range(W):
                            e = engs[(rank, j)]
                            c = rotation_range(rank, off, st, W)
                            seq, seed = rotation_draws(dj, rank, c, e.strata)
                            ms = e.epoch_phase(c, seq, seed, lr, reg, timing=True)
                            worst = max(worst, ms[0])
                        t_ep += worst
                sweep.append(t_ep)
                Qc.copy_(e0.Q[dpi[q]])
                bic.copy_(e0.bi[dpi[q]])
                tot = 0.0
                for e in engs.values():
                    e.sse_async(ep)
                    tot += float(e.sse_values(ep + 1)[ep])
                rm.append(float(np.sqrt(tot / nnz)))
            runs.append({"family": name, "seed": s, "rmse": rm})
            log(f"{name} seed {s}: final {rm[-1]:.7f}")
        # per-rank epoch: the sweeps + (M*N - 1) ring passes + 1 all-gather
        # of the final ranges (RMSE pass beside the next epoch: not counted)
        rows = ni // W
        xch = (sub * W - 1) * t_pass(rows) + (W - 1) * t_pass(rows)
        timing[name] = {"sweep_ms": float(np.median(sweep)), "exchange_ms_model": xch}
        del sets
        torch.cuda.empty_cache()

    def run_prod(name, relabel):
        rp = RotationReplay(u, i, r, nu, ni, W, k, kernel, "float32", dev, relabel=relabel, **hyp)
        sweep = []
        for s in args.draw_seeds:
            rp.load(P0, Q0, np.zeros(nu), np.zeros(ni))
            rm = []
            for ep in range(E):
                draw = int(np.random.RandomState([s, ep, W]).randint(0, 2**31 - 1))
                ms = rp.epoch(draw, lr, reg, timing=True, epoch=ep)
                sweep.append(float(ms.max(axis=1).sum()))      # per sub-epoch: slowest rank
                rm.append(float(np.sqrt(rp.sse(ep) / nnz)))
            runs.append({"family": name, "seed": s, "rmse": rm})
            log(f"{name} seed {s}: final {rm[-1]:.7f}")
        rows = ni // W
        xch = (W - 1) * t_pass(rows) + (W - 1) * t_pass(rows)
        timing[name] = {"sweep_ms": float(np.median(sweep)), "exchange_ms_model": xch,
                        "relabel": relabel}
        del rp
        torch.cuda.empty_cache()

    def run_delta(name, rounds, scale):
        parts = shard_engines(1)
        engs = []
        for rank in range(W):
            a, b, us, is_, rs_ = parts[(rank, 0)]
            e = SGDEngine(us, is_, rs_, b - a, ni, k, kernel, "float32", dev, **hyp)
            e.prepare_strata(regroup=1)
            e.dq = torch.zeros((ni, k), dtype=torch.float32, device=dev)
            e.dbi = torch.zeros(ni, dtype=torch.float32, device=dev)
            engs.append(e)
        C = engs[0].strata.classes
        sweep, sse_ms = [], []
        for s in args.draw_seeds:
            for rank, e in enumerate(engs):
                a, b = parts[(rank, 0)][:2]
                e.load_params(P=P0[a:b], bu=np.zeros(b - a))
            engs[0].load_params(Q=Q0, bi=np.zeros(ni))
            for e in engs[1:]:
                e.Q, e.bi = engs[0].Q, engs[0].bi
            rm = []
            for ep in range(E):
                cuts = []
                for rank, e in enumerate(engs):
                    rsd = np.random.RandomState([s, ep, rank])
                    seq = stratum_order(rsd, e.strata)
                    seed = int(rsd.randint(0, 2**31 - 1))
                    n = len(seq) // C                     # class-cycle groups
                    b = [C * (n * j // rounds) for j in range(rounds + 1)]
                    b[-1] = len(seq)
                    cuts.append([(seq[b[j]:b[j + 1]], seed) for j in range(rounds)])
                t_ep = 0.0
                for j in range(rounds):
                    worst = 0.0
                    for rank, e in enumerate(engs):
                        sq, seed = cuts[rank][j]
                        if len(sq) == 0:
                            continue
                        ms = e.epoch_strata(sq, seed, lr, reg, timing=True,
                                            delta=(e.dq, e.dbi))
                        worst = max(worst, ms[0])
                    t_ep += worst
                    dq = sum(e.dq for e in engs)
                    db = sum(e.dbi for e in engs)
                    engs[0].Q.add_(dq, alpha=scale)
                    engs[0].bi.add_(db, alpha=scale)
                sweep.append(t_ep)
                tot = 0.0
                for rank, e in enumerate(engs):
                    if rank == 0:
                        a0, b0 = ev(), ev()
                        a0.record()
                    e.sse_async(ep)
                    if rank == 0:
                        b0.record()
                    tot += float(e.sse_values(ep + 1)[ep])
                torch.cuda.synchronize()
                sse_ms.append(a0.elapsed_time(b0))
                rm.append(float(np.sqrt(tot / nnz)))
            runs.append({"family": name, "seed": s, "rmse": rm})
            log(f"{name} seed {s}: final {rm[-1]:.7f}")
        timing[name] = {"sweep_ms": float(np.median(sweep)),
                        "exchange_ms_model": rounds * (t_allreduce() + 0.01),
                        "rmse_ms": float(np.median(sse_ms)), "scale": scale, "rounds": rounds,
                        "classes": C, "B": engs[0].strata.B}
        del engs
        torch.cuda.empty_cache()

    for d in args.designs:
        if d == "rotate":
            run_rotate(d)
        elif d.startswith("rotcls") and "rel" in d:       # rotcls<M>rel<K>: both
            m, kk = d[6:].split("rel")
            run_rotate(d, sub=int(m), relabel=int(kk))
        elif d.startswith("rotcls"):
            run_rotate(d, sub=int(d[6:]))
        elif d.startswith("rotprod"):
            run_prod(d, int(d[7:]))
        elif d.startswith("rotrel"):
            run_rotate(d, relabel=int(d[6:]))
        elif d.startswith("rotc"):                 # rotc<C>[b<B>]: sub-block plans of C classes
            cc, _, bb = d[4:].partition("b")
            run_rotate(d, classes=int(cc), blocks=int(bb) if bb else None)
        elif d.startswith("delta"):
            m, sc = d[5:].split("s")
            run_delta(d, int(m), default_delta_scale(W) if sc == "d" else float(sc))
        else:
            raise SystemExit(f"unknown design {d}")

    # RMSE pass of one rank (the rotation runs it beside the next epoch on a
    # side stream; the delta designs after the exchange) -- from the delta runs
    rmse_rank = next((t["rmse_ms"] for t in timing.values() if "rmse_ms" in t), None)
    ref = []
    for p in args.ref:
        try:
            with open(p) as f:
                ref += [x for x in json.load(f)["runs"] if x["family"] == "exact"]
        except OSError as e:                   # (not on the GPU box: compare offline)
            log(f"reference file {p}: {e}")
    ref_final = np.array([x["rmse"][-1] for x in ref]) if ref else None
    table = {}
    fams = {}
    for x in runs:
        fams.setdefault(x["family"], []).append(x["rmse"][-1])
    for f, v in fams.items():
        v = np.array(v)
        t = timing[f]
        per_rank = t["sweep_ms"] + t["exchange_ms_model"] + (
            t.get("rmse_ms", 0.0) if f.startswith("delta") else 0.0)
        row = {"n": len(v), "mean_final": float(v.mean()),
               "sd_final": float(v.std(ddof=1)) if len(v) > 1 else None,
               "per_rank_epoch_ms": per_rank, "projected_x": n1_ms / per_rank, **t}
        if ref_final is not None and len(v) > 1:
            se = np.sqrt(v.var(ddof=1) / len(v) + ref_final.var(ddof=1) / len(ref_final))
            row.update(minus_reference=float(v.mean() - ref_final.mean()), se=float(se),
                       z=float((v.mean() - ref_final.mean()) / se))
        table[f] = row
    doc = {"what": "C4 frontier on one GPU: RMSE after E epochs vs projected per-rank speed-up",
           "workload": desc, "world": W, "epochs": E, "n1_epoch_ms": n1_ms,
           "model": {"busbw_GBs": args.busbw, "linkbw_GBs": args.linkbw,
                     "replica_MB": replica_mb, "allreduce_ms": t_allreduce()},
           "reference": None if ref_final is None else {
               "n": len(ref_final), "mean_final": float(ref_final.mean()),
               "sd_final": float(ref_final.std(ddof=1))},
           "table": table, "runs": runs}
    txt = json.dumps(doc)
    if args.out:
        with open(args.out, "w") as f:
            f.write(txt)
    print(txt)
    log(json.dumps(table, indent=1))


if __name__ == "__main__":
    main()

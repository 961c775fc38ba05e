#!/usr/bin/env python
"""Which users does the MFMA-filter top-k (mf_topk_mm) get wrong at the bench's
C3 top-k workload, and how: for each mismatching user, the exact top-k
(mf_topk) against the filter's, with the scores of the items one list has
and the other lacks.  Same model and queries as bench.py --workload topk.
Usage: python tools/topk_mismatch_probe.py [--show 5]"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "matrix-factorization_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--show", type=int, default=5)
    ap.add_argument("--splits", type=int, default=6, help="k_topk_mw's item splits (C3: 6)")
    args = ap.parse_args()
    import torch

    import bench
    from matrix_factorization.engine import SGDEngine

    nu, ni, nnz, k, _, _ = bench.WORKLOADS["topk"]
    u, i, r = bench.synth(nu, ni, nnz)
    mu = float(np.mean(r, dtype=np.float64))
    rs0 = np.random.RandomState(7)             # bench.main's start (P0, Q0)
    P0 = rs0.normal(0.0, 0.1, (nu, k)).astype(np.float32)
    Q0 = rs0.normal(0.0, 0.1, (ni, k)).astype(np.float32)
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
                    "linear", "float32", torch.device("cuda", 0), min_rating=1.0,
                    max_rating=5.0, global_mean=mu)
    eng.load_params(P0, Q0, bu0, bi0)
    batch = eng.topk_prepare(users, amount, ex_ptr, ex_items)
    eng.topk_launch(batch)
    torch.cuda.synchronize()
    ws = batch["ws"].cpu().numpy().copy()
    fb = eng.topk_finish(batch)
    fi, fs = batch["items"].cpu().numpy(), batch["scores"].cpu().numpy()
    ns = args.splits
    o = 16
    stats = ws[:16].view(np.float32)
    marg = ws[o:o + 4 * n_query].view(np.float32); o += 4 * n_query
    part_n = ws[o:o + 4 * n_query * ns].view(np.int32).reshape(n_query, ns); o += 4 * n_query * ns
    part_s = ws[o:o + 4 * n_query * ns * 256].view(np.float32).reshape(n_query, ns, 256)
    o += 4 * n_query * ns * 256
    part_id = ws[o:o + 4 * n_query * ns * 256].view(np.int32).reshape(n_query, ns, 256)
    o += 4 * n_query * ns * 256
    probe = ws[o:o + 4 * 512].view(np.int32)
    print("stats", stats, "probe[:8]", probe[:8], "part_n total mean", part_n.sum(1).mean())
    eng.topk_launch(batch, exact=True)
    ei, es = batch["items"].cpu().numpy(), batch["scores"].cpu().numpy()
    bad = np.nonzero(~np.all((fi == ei) & ((fs == es) | (np.isnan(fs) & np.isnan(es))), axis=1))[0]
    print(f"fallback {fb}; users differing: {len(bad)} of {n_query}")
    Pd = P0.astype(np.float64)
    Qd = Q0.astype(np.float64)
    for q in bad[: args.show]:
        uu = users[q]
        miss = sorted(set(ei[q]) - set(fi[q]))
        extra = sorted(set(fi[q]) - set(ei[q]))
        def sc(it):
            return mu + bu0[uu] + bi0[it] + Pd[uu] @ Qd[it]
        print(f"user {uu} (query {q}): |p| {np.linalg.norm(Pd[uu]):.4f}")
        print("  exact  ", list(zip(ei[q].tolist(), np.round(es[q], 7).tolist())))
        print("  filter ", list(zip(fi[q].tolist(), np.round(fs[q], 7).tolist())))
        print("  missed ", [(it, round(sc(it), 7)) for it in miss],
              " extra ", [(it, round(sc(it), 7)) for it in extra])
        print(f"  M {marg[q]:.3e}  part_n {part_n[q].tolist()}  missed in probe set: "
              f"{[int(it) in set(probe.tolist()) for it in miss]}")
        for sp in range(ns):
            nn = part_n[q, sp]
            print(f"   split {sp}: " + ", ".join(f"{part_id[q, sp, j]}:{part_s[q, sp, j]:.5f}"
                                                for j in range(min(nn, 12))))


if __name__ == "__main__":
    main()

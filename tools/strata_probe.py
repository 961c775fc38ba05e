#!/usr/bin/env python
"""Phase stamps of the persistent strata kernel (mf_strata_set_probe):
per (position t, workgroup w) the wait for the user range, the block's
steps, the hand-off signal; mean and spread over one epoch.
Usage: python tools/strata_probe.py [--workload c2] [--blocks B] [--rotate N]
--rotate N: one sub-epoch of the N-rank rotation schedule instead -- rank 0's
users x item range 0 (distributed.shard_users / item_ranges), i.e. one
launch of engine.epoch_phase."""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "matrix-factorization_amd"))

import numpy as np
import torch

import bench
from matrix_factorization import _lib
from matrix_factorization.engine import SGDEngine, stratum_order


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c2")
    ap.add_argument("--blocks", type=int, default=None)
    ap.add_argument("--rotate", type=int, default=0)
    ap.add_argument("--dtype", default="float32")
    ap.add_argument("--classes", default="auto", help="user-range classes: auto or 1..4")
    args = ap.parse_args()
    nu, ni, nnz, k, kernel, _ = bench.WORKLOADS[args.workload]
    u, i, r = bench.synth(nu, ni, nnz)
    mu = float(r.mean())
    if args.rotate:
        from matrix_factorization.distributed import item_ranges, local_shard, shard_users
        bounds = shard_users(u, nu, args.rotate)
        ilo = item_ranges(i, ni, args.rotate)
        u, i, r = local_shard(u, i, r, bounds, 0)
        nu = int(bounds[1])
    dt = np.float64 if args.dtype == "float64" else np.float32
    eng = SGDEngine(u, i, r, nu, ni, k, kernel, args.dtype, "cuda:0", gamma=1.0 / k,
                    min_rating=1, max_rating=5, global_mean=mu)
    eng.strata_classes = args.classes if args.classes == "auto" else int(args.classes)
    plan = eng.prepare_strata(n_blocks=args.blocks,
                              item_bounds=ilo if args.rotate else None)
    B = plan.B
    rs = np.random.RandomState(0)
    eng.load_params(rs.normal(0, 0.1, (nu, k)).astype(dt),
                    rs.normal(0, 0.1, (ni, k)).astype(dt),
                    np.zeros(nu, dt), np.zeros(ni, dt))

    def run(seq, seed):
        if args.rotate:
            eng.epoch_phase(0, seq, seed, 0.01, 0.02)
        else:
            eng.epoch_strata(seq, seed, 0.01, 0.02)

    for ep in range(2):
        run(stratum_order(rs, plan), ep)
    torch.cuda.synchronize()
    NSQ = plan.n_strata                   # positions per launch (C*B with user-range classes)
    probe = torch.zeros(4 * NSQ * B, dtype=torch.int64, device="cuda:0")
    _lib.call("mf_strata_set_probe", ctypes.c_void_p(probe.data_ptr()))
    t0 = torch.cuda.Event(enable_timing=True)
    t1 = torch.cuda.Event(enable_timing=True)
    t0.record()
    run(stratum_order(rs, plan), 7)
    t1.record()
    torch.cuda.synchronize()
    _lib.call("mf_strata_set_probe", None)
    eng.check_strata()
    st = probe.cpu().numpy().reshape(NSQ, B, 4).astype(np.float64) * 10.0 / 1000.0   # us
    if not np.all(st[:, :, 3] > 0):
        print("probe incomplete (per-stratum fallback ran?)")
        return
    wait = st[:, :, 1] - st[:, :, 0]
    block = st[:, :, 2] - st[:, :, 1]
    sig = st[:, :, 3] - st[:, :, 2]
    gap = st[1:, :, 0] - st[:-1, :, 3]
    span = st[:, :, 3].max() - st[:, :, 0].min()
    # the probe keeps the stamps of the last launch: phase 0 of the rotation,
    # the last item phase of a phased plan
    pl0 = plan.phases[0] if args.rotate else (plan.phases[-1] if hasattr(plan, "phases") else plan)
    steps = np.diff(pl0.bstep).reshape(NSQ, B)           # [s, w]
    print(f"{args.workload}{' rotate N=%d sub-epoch' % args.rotate if args.rotate else ''}: "
          f"B={B} C={plan.classes} NS={plan.NS} epoch kernel {t0.elapsed_time(t1):.3f} ms, "
          f"stamp span {span / 1e3:.3f} ms, per position {span / NSQ:.2f} us")
    for name, a in (("wait", wait), ("block", block), ("signal", sig), ("gap", gap)):
        print(f"  {name:6s} mean {a.mean():7.2f} us  p50 {np.median(a):7.2f}  p90 "
              f"{np.percentile(a, 90):7.2f}  max {a.max():7.2f}")
    print(f"  steps per block: mean {steps.mean():.2f} max {steps.max()}; "
          f"block us per step {block.sum() / max(steps.sum(), 1):.2f}")
    busy = (block + sig).sum(axis=0)                      # per workgroup
    print(f"  per-workgroup busy (block+signal) mean {busy.mean() / 1e3:.3f} ms "
          f"(min {busy.min() / 1e3:.3f}, max {busy.max() / 1e3:.3f}), "
          f"wait total mean {wait.sum(axis=0).mean() / 1e3:.3f} ms")
    xcd = np.array([busy[w::8].mean() for w in range(min(8, B))]) / 1e3
    print("  busy by XCD (w % 8), ms: " + " ".join(f"{x:.3f}" for x in xcd))
    bt = block.T                                          # [w, t]
    rel = bt / bt.mean(axis=1, keepdims=True)
    print(f"  block time / its workgroup's mean: p10 {np.percentile(rel, 10):.2f} "
          f"p90 {np.percentile(rel, 90):.2f}; workgroup means p10 "
          f"{np.percentile(bt.mean(axis=1), 10):.1f} p90 {np.percentile(bt.mean(axis=1), 90):.1f} us")


if __name__ == "__main__":
    main()

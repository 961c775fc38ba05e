#!/usr/bin/env python
"""Stamps of the stream form of the persistent strata kernel
(k_sgd_strata_stream, MF_STRATA_STREAM=1; mf_strata_set_probe): per
(position t, workgroup w) when the apply cursor entered the position, wave
0's spin waiting for the NEXT position's user range (inside this position),
and the drain + barrier of a hand-off publication (in this position's second
step).  Prints per-position time, its split, and the per-step time.
Usage: python tools/stream_probe.py [--workload c3] [--dtype float64]"""
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
from matrix_factorization.engine import PhasedStrata, SGDEngine, stratum_order


def main():
    os.environ.setdefault("MF_STRATA_STREAM", "1")
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c3")
    ap.add_argument("--dtype", default="float64")
    ap.add_argument("--blocks", type=int, default=None)
    args = ap.parse_args()
    nu, ni, nnz, k, kernel, _ = bench.WORKLOADS[args.workload]
    u, i, r = bench.synth(nu, ni, nnz)
    dt = np.float64 if args.dtype == "float64" else np.float32
    eng = SGDEngine(u, i, r, nu, ni, k, kernel, args.dtype, "cuda:0", gamma=1.0 / k,
                    min_rating=1, max_rating=5, global_mean=float(r.mean()))
    eng.strata_regroup = 1
    plan = eng.prepare_strata(n_blocks=args.blocks)
    rs = np.random.RandomState(0)
    eng.load_params(rs.normal(0, 0.1, (nu, k)).astype(dt), rs.normal(0, 0.1, (ni, k)).astype(dt),
                    np.zeros(nu, dt), np.zeros(ni, dt))
    for ep in range(2):
        eng.epoch_strata(stratum_order(rs, plan), ep, 0.01, 0.02)
    torch.cuda.synchronize()
    B, NSQ = plan.B, plan.n_strata
    sub = plan.phases[-1] if isinstance(plan, PhasedStrata) else plan   # stamps of the last phase
    probe = torch.zeros(4 * NSQ * B, dtype=torch.int64, device="cuda:0")
    _lib.call("mf_strata_set_probe", ctypes.c_void_p(probe.data_ptr()))
    seq = stratum_order(rs, plan)
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    eng.epoch_strata(seq, 7, 0.01, 0.02)
    t1.record()
    torch.cuda.synchronize()
    _lib.call("mf_strata_set_probe", None)
    eng.check_strata()
    st = probe.cpu().numpy().reshape(NSQ, B, 4)
    if not np.all(st[:, :, 3] > 0):
        print("probe incomplete (not the stream kernel?)")
        return
    tick = 0.01                                           # us per s_memrealtime tick (100 MHz)
    enter = st[:, :, 0].astype(np.int64)
    tend = st[0, :, 3].astype(np.int64)
    nxt = np.vstack([enter[1:], tend[None, :]])
    pos = ((nxt - enter) % (1 << 32)) * tick              # us per position (32-bit stamps)
    spin = st[:, :, 1] * tick                             # spin for position t, spent in t-1
    drain = st[:, :, 2] * tick
    spin_in = np.vstack([spin[1:], np.zeros((1, B))])     # spin spent inside position t
    steps = np.diff(sub.bstep).reshape(NSQ, B)[np.asarray(seq)] if hasattr(sub, "bstep") else None
    nv = np.maximum(steps, 4) if steps is not None else None
    ms = t0.elapsed_time(t1)
    print(f"{args.workload} {args.dtype}: B={B} C={plan.classes} NS={plan.NS} epoch {ms:.3f} ms "
          f"({'2 phases, stamps of the last' if isinstance(plan, PhasedStrata) else '1 launch'})")

    def stat(name, a):
        a = np.asarray(a, np.float64).ravel()
        print(f"  {name:28s} mean {a.mean():7.3f}  p50 {np.percentile(a, 50):7.3f}  "
              f"p90 {np.percentile(a, 90):7.3f}  max {a.max():8.3f}")
    stat("position (us)", pos)
    stat("spin for next range (us)", spin_in)
    d = drain[drain > 0]
    stat("drain + barrier (us, when)", d if d.size else [0])
    print(f"  drains per position {d.size / drain.size:.3f}, spins > 0.05 us: "
          f"{(spin_in > 0.05).mean():.3f} of positions")
    if nv is not None:
        body = pos - spin_in - drain
        stat("steps per position", steps)
        stat("us per step (excl. spin/drain)", (body / nv)[nv > 0])

    print(f"  per-workgroup sum of positions (ms): mean {pos.sum(0).mean() / 1e3:.3f} "
          f"min {pos.sum(0).min() / 1e3:.3f} max {pos.sum(0).max() / 1e3:.3f}")


if __name__ == "__main__":
    main()

#!/usr/bin/env python
"""Where fit()'s first epochs spend their time: the C3 engine built as fit()
builds it (SGDEngine + prepare_strata with the default classes and relabelled
plans), then the first epochs one call at a time, each synchronised and
wall-clocked (host + device), with the plan each epoch picked.
Usage: python tools/warmup_probe.py [--dtype float32] [--epochs 5]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "matrix-factorization_amd"))

import numpy as np
import torch

import bench
from matrix_factorization.engine import SGDEngine, _ErrorPoll, stratum_order


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="float32")
    ap.add_argument("--epochs", type=int, default=5)
    ap.add_argument("--workload", default="c3")
    args = ap.parse_args()
    nu, ni, nnz, k, kernel, _ = bench.WORKLOADS[args.workload]
    u, i, r = bench.synth(nu, ni, nnz)
    dt = np.dtype(args.dtype)
    t = time.perf_counter()
    eng = SGDEngine(u, i, r, nu, ni, k, kernel, args.dtype, "cuda:0", gamma=1.0 / k,
                    min_rating=1, max_rating=5, global_mean=float(r.mean()))
    plan = eng.prepare_strata()
    torch.cuda.synchronize()
    print(f"engine + plan {time.perf_counter() - t:.3f} s", flush=True)
    rs = np.random.RandomState(0)
    eng.load_params(rs.normal(0, 0.1, (nu, k)).astype(dt), rs.normal(0, 0.1, (ni, k)).astype(dt),
                    np.zeros(nu, dt), np.zeros(ni, dt))
    torch.cuda.synchronize()

    def clock(name, fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = fn()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"  {name:24s} host {1e3 * (t1 - t0):8.3f} ms   host+device {1e3 * (t2 - t0):8.3f} ms",
              flush=True)
        return out

    snap = clock("snapshot_params", eng.snapshot_params)
    poll = clock("_ErrorPoll()", lambda: _ErrorPoll(eng))
    for ep in range(args.epochs):
        seq = stratum_order(np.random, eng.strata)
        seed = int(np.random.randint(0, 2**31 - 1))
        print(f"epoch {ep + 1}: plan {eng._regroup_pick(seed)}", flush=True)
        clock("epoch_strata", lambda: eng.epoch_strata(seq, seed, 0.01, 0.02))
        clock("poll.post", poll.post)
        clock("sse_async", lambda: eng.sse_async(ep))
    del snap


if __name__ == "__main__":
    main()

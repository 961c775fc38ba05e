#!/usr/bin/env python
"""Where an exact-schedule epoch (fit(schedule="exact")) spends its time at
C3, component by component, each timed alone on this host / GPU:
  shuffle   np.random.shuffle of the 32-bit row order (native, one thread)
  gather    order[perm] on the host threads (mf_gather_i32)
  levels    the exact-order batches (sched_levels_chunked, host threads)
  gpu       one epoch of level launches (epoch_exact, synchronised)
  epoch     epoch_exact end to end (levels + upload + launches), synchronised
  gpu_shuffle  the same shuffle with its swaps on the GPU (ExactShuffler)
Usage: python tools/exact_probe.py [--nnz 100000000] [--reps 3]"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "matrix-factorization_amd"))

import torch  # noqa: E402

import bench  # noqa: E402
from matrix_factorization import _prep  # noqa: E402
from matrix_factorization.engine import (ExactShuffler, SGDEngine,  # noqa: E402
                                         sched_levels_chunked)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nnz", type=int, default=100_000_000)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    nu, ni, k = 1_000_000, 100_000, 64
    u, i, r = bench.synth(nu, ni, args.nnz)
    n = len(u)
    eng = SGDEngine(u, i, r, nu, ni, k, "linear", "float64", "cuda:0",
                    global_mean=float(r.mean()))
    rs = np.random.RandomState(1)
    eng.load_params(rs.normal(0, 0.1, (nu, k)), rs.normal(0, 0.1, (ni, k)),
                    np.zeros(nu), np.zeros(ni))
    out = {"nnz": n}
    order = np.arange(n, dtype=np.int32)
    np.random.seed(5)

    def timed(fn):
        ts = []
        for _ in range(args.reps):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        return ts

    out["shuffle_s"] = timed(lambda: _prep.legacy_shuffle_(order))
    sh = ExactShuffler(n, torch.device("cuda:0"))
    cur = [sh.shuffle_from(order)]

    def gpu_shuffle():
        cur[0] = sh.shuffle_from(cur[0])

    out["gpu_shuffle_s"] = timed(gpu_shuffle)
    tg = np.empty(n - 1, np.uint32)
    out["draws_s"] = timed(lambda: _prep.legacy_shuffle_draws(n, tg))
    perm = order.copy()
    out["gather_s"] = timed(lambda: _prep.gather(order, perm))
    hb = np.empty(n, np.int32)
    out["levels_s"] = timed(lambda: sched_levels_chunked(eng.u_host, eng.i_host, order, nu, ni,
                                                         out=hb))
    _, offs = sched_levels_chunked(eng.u_host, eng.i_host, order, nu, ni)
    out["levels"] = len(offs) - 1
    eng.epoch_exact(order, 0.01, 0.02)
    torch.cuda.synchronize()

    def epoch():
        eng.epoch_exact(order, 0.01, 0.02)
        torch.cuda.synchronize()

    out["epoch_s"] = timed(epoch)
    ms = []
    for _ in range(args.reps):
        torch.cuda.synchronize()
        m, _ = eng.epoch_exact(order, 0.01, 0.02, timing=True)
        torch.cuda.synchronize()
        ms.append(m / 1e3)
    out["gpu_launches_s"] = ms
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

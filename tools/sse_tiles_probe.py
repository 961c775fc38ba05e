#!/usr/bin/env python
"""Time the training-SSE pass (mf_sse) at C3 over evaluation tilings:
user chunks x item slices (mf_sched_tiles), walked in phases by a resident
grid (k_sse_phased) or, with a trailing 'd', by the dispatch-ordered grid.
Usage: python tools/sse_tiles_probe.py [--dtype float64] CxS[d] ...
(1x8 = the round-5 default evaluation order)"""

import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "matrix-factorization_amd"))

import numpy as np
import torch

import bench
from matrix_factorization.engine import SGDEngine


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="float64")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("tiles", nargs="*", default=["1x8"])
    args = ap.parse_args()
    nu, ni, nnz, k = 1_000_000, 100_000, 100_000_000, 64
    u, i, r = bench.synth(nu, ni, nnz)
    dt = args.dtype
    os.environ["MF_SSE_TILES"] = args.tiles[0].rstrip("d").replace("x", ",")
    eng = SGDEngine(u, i, r, nu, ni, k, "linear", dt, "cuda:0",
                    global_mean=float(r.mean()), min_rating=1, max_rating=5)
    rs = np.random.RandomState(0)
    eng.load_params(rs.normal(0, 0.1, (nu, k)).astype(dt),
                    rs.normal(0, 0.1, (ni, k)).astype(dt),
                    np.zeros(nu, dt), np.zeros(ni, dt))
    ref = None
    for t in args.tiles:
        os.environ["MF_SSE_TILES"] = t.rstrip("d").replace("x", ",")
        os.environ["MF_SSE_PHASED"] = "0" if t.endswith("d") else "1"
        eng._build_eval()
        for _ in range(3):
            eng.sse_async(0)
        torch.cuda.synchronize()
        t0 = torch.cuda.Event(enable_timing=True)
        t1 = torch.cuda.Event(enable_timing=True)
        t0.record()
        for s in range(args.reps):
            eng.sse_async(s)
        t1.record()
        torch.cuda.synchronize()
        ms = t0.elapsed_time(t1) / args.reps
        sse = eng.sse_values(1)[0]
        ref = sse if ref is None else ref
        print(f"dtype={dt} tiles={t} sse_ms={ms:.3f} sse={sse:.10f} "
              f"rel_to_first={abs(sse - ref) / ref:.2e}", flush=True)


if __name__ == "__main__":
    main()

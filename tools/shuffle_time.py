#!/usr/bin/env python
"""Host time of the native np.random.shuffle (mf_legacy_shuffle_i32, branch-free
MT draws, prefetched swaps) on an n-element int32 array, three repetitions,
with a signature of the result (first 1000 elements' sum and the next NumPy
draw) to compare builds.  Usage: python tools/shuffle_time.py [--n 100000000]"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "matrix-factorization_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100_000_000)
    args = ap.parse_args()
    from matrix_factorization import _prep
    ts, sig = [], None
    for _ in range(3):
        a = np.arange(args.n, dtype=np.int32)
        np.random.seed(3)
        t = time.perf_counter()
        _prep.legacy_shuffle_(a)
        ts.append(time.perf_counter() - t)
        sig = int(a[:1000].astype(np.int64).sum()), int(np.random.randint(0, 2**31 - 1))
    print(f"n={args.n}: {ts} s, signature {sig}", flush=True)


if __name__ == "__main__":
    main()

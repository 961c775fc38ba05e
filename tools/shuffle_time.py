#!/usr/bin/env python
"""Host time of the native np.random.shuffle (mf_legacy_shuffle_i32) on a
100M-element int32 array: the pipelined form (default for n >= 2^22) and
the one-thread form (MF_SHUFFLE_SERIAL=1), each checked against the other.
Usage: python tools/shuffle_time.py [--n 100000000]"""
import argparse
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "matrix-factorization_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100_000_000)
    ap.add_argument("--child", action="store_true")
    args = ap.parse_args()
    if not args.child:
        for serial in ("1", None):
            env = dict(os.environ)
            env.pop("MF_SHUFFLE_SERIAL", None)
            if serial:
                env["MF_SHUFFLE_SERIAL"] = serial
            subprocess.run([sys.executable, __file__, "--child", "--n", str(args.n)], env=env,
                           check=True)
        return
    from matrix_factorization import _prep
    ts, sig = [], None
    for rep in range(3):
        a = np.arange(args.n, dtype=np.int32)
        np.random.seed(3)
        t = time.perf_counter()
        _prep.legacy_shuffle_(a)
        ts.append(time.perf_counter() - t)
        sig = int(a[:1000].astype(np.int64).sum()), int(np.random.randint(0, 2**31 - 1))
    print(f"MF_SHUFFLE_SERIAL={os.environ.get('MF_SHUFFLE_SERIAL')}: {ts} s, signature {sig}",
          flush=True)


if __name__ == "__main__":
    main()

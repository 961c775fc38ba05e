#!/usr/bin/env python
"""Host probe: the native np.random.shuffle (mf_legacy_shuffle_i32) of a
100M int32 array in ordinary NumPy memory vs memory madvise'd for
transparent huge pages (the swaps are random accesses over 400 MB: one TLB
miss each with 4-KiB pages).  Prints the THP mode, AnonHugePages before and
after, and the time of each form (same permutation: same signature)."""
import mmap
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "matrix-factorization_amd"))


def anon_huge():
    for line in open("/proc/meminfo"):
        if line.startswith("AnonHugePages"):
            return line.split(":")[1].strip()
    return "?"


def main():
    from matrix_factorization import _prep
    n = 100_000_000
    try:
        print("thp", open("/sys/kernel/mm/transparent_hugepage/enabled").read().strip(),
              "defrag", open("/sys/kernel/mm/transparent_hugepage/defrag").read().strip())
    except OSError as e:
        print("thp ?", e)
    print("AnonHugePages before", anon_huge(), flush=True)
    keep = []
    for label in ("plain", "huge", "plain", "huge"):
        if label == "plain":
            a = np.arange(n, dtype=np.int32)
        else:
            mm = mmap.mmap(-1, n * 4, flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
            mm.madvise(mmap.MADV_HUGEPAGE)
            a = np.frombuffer(mm, dtype=np.int32, count=n)
            a[:] = np.arange(n, dtype=np.int32)
            keep.append(mm)
            print("AnonHugePages with the huge buffer", anon_huge(), flush=True)
        np.random.seed(3)
        t = time.perf_counter()
        _prep.legacy_shuffle_(a)
        print(f"{label}: {time.perf_counter() - t:.3f} s signature "
              f"{int(a[:1000].astype(np.int64).sum())}", flush=True)
        del a


if __name__ == "__main__":
    main()

"""Host-only timing: two C3 strata plans (the engine's own and one relabelled
plan, as prepare_strata builds them) one after the other vs on two threads
at once.  Prints one JSON line."""
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "matrix-factorization_amd"))

import bench  # noqa: E402
from matrix_factorization.engine import balanced_bounds, sched_strata  # noqa: E402

NU, NI, B, C, NS = 1_000_000, 100_000, 256, 4, 32


def bounds(u, i):
    return balanced_bounds(u, NU, C * B), balanced_bounds(i, NI, B)


def plan(u, i, bnd):
    ub, ib = bnd
    t = time.perf_counter()
    sched_strata(u, i, NU, NI, B, ub, ib, NS, C)
    return time.perf_counter() - t


def main():
    u, i, _ = bench.synth(NU, NI, 100_000_000)
    rs = np.random.RandomState(1)
    pu = rs.permutation(NU).astype(np.int32)
    pi = rs.permutation(NI).astype(np.int32)
    u2, i2 = pu[u], pi[i]
    b1, b2 = bounds(u, i), bounds(u2, i2)
    plan(u, i, b1)                               # page in
    out = {"host_threads": os.environ.get("MF_HOST_THREADS", "default")}
    t = time.perf_counter()
    a, b = plan(u, i, b1), plan(u2, i2, b2)
    out["sequential_s"] = round(time.perf_counter() - t, 3)
    out["sequential_each_s"] = [round(a, 3), round(b, 3)]
    with ThreadPoolExecutor(2) as ex:
        t = time.perf_counter()
        fa, fb = ex.submit(plan, u, i, b1), ex.submit(plan, u2, i2, b2)
        a, b = fa.result(), fb.result()
        out["concurrent_s"] = round(time.perf_counter() - t, 3)
        out["concurrent_each_s"] = [round(a, 3), round(b, 3)]
    print(json.dumps(out))


if __name__ == "__main__":
    main()

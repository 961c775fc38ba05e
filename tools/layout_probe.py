#!/usr/bin/env python
"""Does the id layout of the ratings change the strata sweep's speed?

fit() trains on _preprocess_data's frame (rows shuffled, user / item ids in
order of first appearance); bench.py on synth()'s ids.  Same C3 matrix,
three layouts, each with its own engine and plan, the bench's loop
(epoch_strata + sse_async, hipEvents), median ms of SGD and RMSE:
  bench     synth()'s ids and row order
  rows      rows permuted, ids kept
  firstapp  rows permuted, ids renumbered by first appearance (fit()'s)
  sorted    rows sorted by (user, item), ids kept
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "matrix-factorization_amd"))

import bench  # noqa: E402


def first_appearance(x, n):
    uniq, first = np.unique(x, return_index=True)
    m = np.empty(n, np.int32)
    m[uniq[np.argsort(first)]] = np.arange(len(uniq), dtype=np.int32)
    return m[x]


def main():
    if "--after-bench" in sys.argv:        # bench.py's own run first, in this process
        argv = sys.argv
        sys.argv = ["bench.py", "--cpu-sample", "0", "--steps", "5"]
        bench.main()
        sys.argv = argv
    import torch

    if "--set-device" in sys.argv:         # bench.py's start: torch.cuda.set_device
        torch.cuda.set_device(torch.device("cuda", 0))
    if "--warm-alloc" in sys.argv:         # one big segment in the caching allocator first
        x = torch.empty(6 << 30, dtype=torch.uint8, device="cuda:0")
        del x
    from matrix_factorization.engine import SGDEngine

    nu, ni, nnz, k = 1_000_000, 100_000, 100_000_000, 64
    u, i, r = bench.synth(nu, ni, nnz)
    mu = float(np.mean(r, dtype=np.float64))
    rs = np.random.RandomState(7)
    P0 = rs.normal(0.0, 0.1, (nu, k)).astype(np.float32)
    Q0 = rs.normal(0.0, 0.1, (ni, k)).astype(np.float32)
    only = [x for x in sys.argv[1:] if not x.startswith("-")]
    perm = np.random.RandomState(1).permutation(nnz)
    layouts = {
        "bench": lambda: (u, i, r),
        "rows": lambda: (u[perm], i[perm], r[perm]),
        "firstapp": lambda: (first_appearance(u[perm], nu), first_appearance(i[perm], ni), r[perm]),
        "sorted": lambda: tuple(a[np.lexsort((i, u))] for a in (u, i, r)),
    }
    out = {}
    names = [n for n in layouts if not only or n in only]
    if "--twice" in sys.argv:              # the same layout twice: a second engine and plan
        names = names + names
    for name in names:
        make = layouts[name]
        lu, li, lr_ = make()
        eng = SGDEngine(lu, li, lr_, nu, ni, k, "linear", "float32", "cuda:0", gamma=1.0 / k,
                        min_rating=1.0, max_rating=5.0, global_mean=mu)
        if "--plan-first" in sys.argv:      # bench.py's order: plan, then the parameters
            plan = eng.prepare_strata()
            eng.load_params(P0, Q0, np.zeros(nu), np.zeros(ni))
        else:
            eng.load_params(P0, Q0, np.zeros(nu), np.zeros(ni))
            plan = eng.prepare_strata()
        eng._ensure_sse_slots(8)
        if "--p-contiguous" in sys.argv:   # P in hipExtMallocWithFlags(hipDeviceMallocContiguous)
            import ctypes
            hip = ctypes.CDLL("libamdhip64.so")
            ptr = ctypes.c_void_p()
            nb = nu * k * 4
            rc = hip.hipExtMallocWithFlags(ctypes.byref(ptr), ctypes.c_size_t(nb), ctypes.c_uint(4))
            assert rc == 0, rc

            class _Buf:
                __cuda_array_interface__ = {"shape": (nu, k), "typestr": "<f4",
                                            "data": (ptr.value, False), "version": 2,
                                            "strides": None}
            P2 = torch.as_tensor(_Buf(), device="cuda:0")
            assert P2.data_ptr() == ptr.value
            P2.copy_(eng.P)
            eng.P = P2
            print("contiguous P at", hex(ptr.value), file=sys.stderr)
        arena = [a for a in sys.argv if a.startswith("--p-arena=")]
        if arena:                          # P as a view at the start of a larger allocation
            gb = float(arena[0].split("=")[1])
            buf = torch.empty(int(gb * (1 << 30)) // 4, dtype=torch.float32, device="cuda:0")
            P2 = buf[: nu * k].view(nu, k)
            P2.copy_(eng.P)
            eng.P = P2
        ev = []
        if "--timing-first" in sys.argv:   # bench.py's first warmup epoch: timing=True
            eng.epoch_strata(bench.strata_seq(99, plan.B), bench.strata_rot(99), 0.01, 0.02,
                             timing=True)
        for ep in range(7):
            a, m_, b = (torch.cuda.Event(enable_timing=True) for _ in range(3))
            a.record()
            eng.epoch_strata(bench.strata_seq(ep, plan.B), bench.strata_rot(ep), 0.01, 0.02)
            m_.record()
            eng.sse_async(ep)
            b.record()
            ev.append((a, m_, b))
        torch.cuda.synchronize()
        sgd = [a.elapsed_time(m_) for a, m_, _ in ev][2:]
        sse = [m_.elapsed_time(b) for _, m_, b in ev][2:]
        name = name if name not in out else name + "_again"
        out[name] = {"sgd_ms": float(np.median(sgd)), "rmse_ms": float(np.median(sse)),
                     "B": int(plan.B), "positions": int(plan.n_positions),
                     "max_steps": int(np.diff(plan.bstep).max())}
        print(name, out[name], file=sys.stderr, flush=True)
        del eng
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()

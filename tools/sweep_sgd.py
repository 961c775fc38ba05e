#!/usr/bin/env python
"""A/B sweep of SGD-kernel variants and the RMSE pass on one workload.

Interleaves every variant over several rounds in ONE process (guide rule 24)
and prints per-variant median kernel time per epoch (hipEvents around each
launch), wall time per epoch, and the RMSE-pass time.
"""

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "matrix-factorization_amd"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c3")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", default="")
    args = ap.parse_args()

    import torch

    import bench
    from matrix_factorization import _lib
    from matrix_factorization.engine import SGDEngine

    nu, ni, nnz, k, kernel, desc = bench.WORKLOADS[args.workload]
    u, i, r = bench.synth(nu, ni, nnz)
    rs = np.random.RandomState(7)
    P0 = rs.normal(0, 0.1, (nu, k)).astype(np.float32)
    Q0 = rs.normal(0, 0.1, (ni, k)).astype(np.float32)
    eng = SGDEngine(u, i, r, nu, ni, k, kernel, "float32", "cuda:0", gamma=1.0 / k,
                    min_rating=1.0, max_rating=5.0, global_mean=float(r.mean()))
    eng.load_params(P0, Q0, np.zeros(nu), np.zeros(ni))
    nb = eng.prepare_colored()
    print(f"# {desc}: {nb} colours", file=sys.stderr, flush=True)
    X, NT, NQ = _lib.MF_FLAG_XCD_SWIZZLE, _lib.MF_FLAG_NT_USER, _lib.MF_FLAG_NT_ITEM
    CL = _lib.MF_FLAG_XCD_CLAIM
    variants = {    # float4 layout, k=64: tile 0 -> S=4 slots (16 ratings/wave),
                    # 1 -> S=2, 2 -> S=8, 3 -> S=1
        "s4_nt": X | NT, "s4_nt_noxcd": NT, "s4": X,
    }
    # user-row cache policies (mf_rows.hpp kPolAux; flags bits 12..15)
    for pol in range(2, 8):
        variants[f"p{pol}"] = X | (pol << 12)
    if args.variants:
        variants = {kk: v for kk, v in variants.items() if kk in args.variants.split(",")}
    res = {kk: {"kernel_ms": [], "wall_ms": [], "wall_nt_ms": []} for kk in variants}
    sse_ms = []
    seq = np.random.RandomState(0).permutation(nb).astype(np.int32)
    dev = torch.device("cuda", 0)
    for rd in range(args.rounds):
        for name, fl in variants.items():
            eng.epoch_colored(seq, 0.01, 0.02, flags=fl)          # warm
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            kms = eng.epoch_colored(seq, 0.01, 0.02, flags=fl, timing=True)
            torch.cuda.synchronize(dev)
            res[name]["wall_ms"].append((time.perf_counter() - t0) * 1e3)
            res[name]["kernel_ms"].append(kms[0])
            t0 = time.perf_counter()
            eng.epoch_colored(seq, 0.01, 0.02, flags=fl)
            torch.cuda.synchronize(dev)
            res[name]["wall_nt_ms"].append((time.perf_counter() - t0) * 1e3)
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        eng.sse_async(0)
        e1.record()
        torch.cuda.synchronize(dev)
        sse_ms.append(e0.elapsed_time(e1))
        print(f"# round {rd} done", file=sys.stderr, flush=True)
    # timing-only probe: the whole epoch as ONE launch (conflicting updates
    # race; numerically meaningless) -> steady-state rate without boundaries
    from matrix_factorization.engine import _np, _tp
    import ctypes
    one = np.array([0, eng.n], np.int64)
    single = []
    for fl in (X, X | NT, X | NT | NQ):
        ms = (ctypes.c_double * 2)()
        for _ in range(2):
            _lib.call("mf_sgd_epoch", _tp(eng.u), _tp(eng.i), _tp(eng.r), eng.n, None,
                      _np(one), 1, None, 0, eng.global_mean, _tp(eng.bu), _tp(eng.bi),
                      _tp(eng.P), _tp(eng.Q), eng.n_users, eng.n_items, eng.k, eng.kcode,
                      eng.dcode, eng.gamma, 0.01, 0.02, 1.0, 5.0, 1, 1, fl, None, 0,
                      eng.stream, ms)
        single.append({"flags": fl, "ms": ms[0], "Gupd_s": nnz / ms[0] / 1e6})
    out = {"single_launch": single}
    for name, d in res.items():
        out[name] = {kk: float(np.median(v)) for kk, v in d.items()}
        km = out[name]["kernel_ms"]
        out[name]["kernel_Gupd_s"] = nnz / km / 1e6
        out[name]["alg_TBs"] = nnz * (16 * k + 28) / km / 1e9
    out["sse_ms"] = float(np.median(sse_ms))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

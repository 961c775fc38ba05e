#!/usr/bin/env python
"""Phase timing of mf_als_sweep per entity (mf_als_sweep_probe): Gramian,
elimination, border + back substitution, for the user and the item
half-sweep of a synthetic workload (bench.py's generator)."""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "matrix-factorization_amd"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c5_small")
    args = ap.parse_args()
    import bench
    from matrix_factorization import _lib
    from matrix_factorization.engine import FactorALS, SGDEngine, _tp

    nu, ni, nnz, k, _, _ = bench.WORKLOADS[args.workload]
    u, i, r = bench.synth(nu, ni, nnz)
    dev = torch.device("cuda", 0)
    eng = SGDEngine(u, i, r, nu, ni, k, "linear", "float32", dev, global_mean=float(r.mean()))
    rs = np.random.RandomState(7)
    eng.load_params(rs.normal(0, .1, (nu, k)), rs.normal(0, .1, (ni, k)), np.zeros(nu), np.zeros(ni))
    als = FactorALS(eng)
    for name, csr, n, ob, oq, b, q in (("users", als.user_csr, nu, eng.bi, eng.Q, eng.bu, eng.P),
                                       ("items", als.item_csr, ni, eng.bu, eng.P, eng.bi, eng.Q)):
        probe = torch.zeros(4 * n, dtype=torch.int64, device=dev)
        for rep in range(2):
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record()
            _lib.call("mf_als_sweep_probe", _tp(csr[0]), _tp(csr[1]), _tp(csr[2]), n,
                      eng.global_mean, _tp(ob), _tp(oq), _tp(b), _tp(q), k, _lib.MF_F32, 1.0,
                      eng.stream, _tp(probe))
            ev[1].record()
            torch.cuda.synchronize()
        t = probe.view(n, 4).cpu().numpy().astype(np.float64) * 10.0     # ns (100 MHz)
        d = np.diff(t, axis=1) / 1e3
        life = (t[:, 3] - t[:, 0]) / 1e3
        span = (t[:, 3].max() - t[:, 0].min()) / 1e6
        print(f"{name}: {n} entities, kernel {ev[0].elapsed_time(ev[1]):.2f} ms (span {span:.2f} ms); "
              f"per entity us: gram {d[:, 0].mean():.1f}  elim {d[:, 1].mean():.1f}  "
              f"backsub {d[:, 2].mean():.1f}  total {life.mean():.1f} (p99 {np.percentile(life, 99):.1f}); "
              f"concurrent WGs ~ {life.sum() / 1e3 / span:.0f}", flush=True)


if __name__ == "__main__":
    main()

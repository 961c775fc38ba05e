"""Time the training-SSE pass (mf_sse) at C3 for kernel variants and grid
sizes (MF_SSE_VARIANT / MF_SSE_BLOCKS, read by the launcher at every call).
Usage: python tools/sse_probe.py [variant:blocks ...]   (0 = library default;
variant 1 = k_sse_stream, 2 = k_sse_owned without the uniform skip)"""

import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "matrix-factorization_amd"))

import numpy as np
import torch

import bench
from matrix_factorization.engine import SGDEngine


def main():
    runs = [tuple(int(y) for y in x.split(":")) for x in sys.argv[1:]] or [(0, 0)]
    nu, ni, nnz, k = 1_000_000, 100_000, 100_000_000, 64
    import matrix_factorization.engine as E
    E.N_SLICES = int(os.environ.get("SSE_PROBE_SLICES", E.N_SLICES))   # evaluation slices
    u, i, r = bench.synth(nu, ni, nnz)
    dt = os.environ.get("SSE_PROBE_DTYPE", "float32")
    eng = SGDEngine(u, i, r, nu, ni, k, "linear", dt, "cuda:0",
                    global_mean=float(r.mean()), min_rating=1, max_rating=5)
    rs = np.random.RandomState(0)
    eng.load_params(rs.normal(0, 0.1, (nu, k)).astype(dt),
                    rs.normal(0, 0.1, (ni, k)).astype(dt),
                    np.zeros(nu, dt), np.zeros(ni, dt))
    ref = None
    for var, g in runs:
        for key, val in (("MF_SSE_VARIANT", var), ("MF_SSE_BLOCKS", g)):
            if val:
                os.environ[key] = str(val)
            else:
                os.environ.pop(key, None)
        for _ in range(3):
            eng.sse_async(0)
        torch.cuda.synchronize()
        reps = int(os.environ.get("SSE_PROBE_REPS", "20"))
        t0 = torch.cuda.Event(enable_timing=True)
        t1 = torch.cuda.Event(enable_timing=True)
        t0.record()
        for s in range(reps):
            eng.sse_async(s)
        t1.record()
        torch.cuda.synchronize()
        ms = t0.elapsed_time(t1) / reps
        sse = eng.sse_values(1)[0]
        ref = sse if ref is None else ref
        print(f"dtype={dt} slices={E.N_SLICES} variant={var} blocks={g or 'default'} sse_ms={ms:.3f} sse={sse:.6f} "
              f"rel_to_first={abs(sse - ref) / ref:.2e}", flush=True)


if __name__ == "__main__":
    main()

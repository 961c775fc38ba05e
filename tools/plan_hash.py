"""Hash the strata planner's output (sched + block step offsets) over a few
configurations, so that a change to mf_strata_sched.cpp can be checked to
leave every plan bit-identical:

    python tools/plan_hash.py > /tmp/before.json   # old build
    python tools/plan_hash.py > /tmp/after.json    # new build; diff the two

Host code only (no GPU).  Sizes: C3 at full scale (10^8 ratings) plus small
ragged and skewed cases."""
import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "matrix-factorization_amd"))

import bench  # noqa: E402
from matrix_factorization.engine import balanced_bounds, sched_strata  # noqa: E402


def one(name, u, i, nu, ni, B, C, ns):
    ub = balanced_bounds(u, nu, C * B)
    ib = balanced_bounds(i, ni, B)
    t = time.time()
    sched, bstep = sched_strata(u, i, nu, ni, B, ub, ib, ns, C)
    dt = time.time() - t
    h = hashlib.sha256(sched.tobytes())
    h.update(bstep.tobytes())
    return {"case": name, "B": B, "C": C, "ns": ns, "positions": int(len(sched)),
            "sha256": h.hexdigest(), "s": round(dt, 3)}


def main():
    out = []
    rng = np.random.default_rng(7)
    for (nu, ni, n, B, C, ns) in [(500, 300, 20000, 8, 1, 64), (500, 300, 20000, 8, 3, 32),
                                  (40000, 9000, 600000, 32, 4, 128),
                                  (40000, 9000, 600000, 48, 2, 256)]:
        u = rng.integers(0, nu, n).astype(np.int32)
        # skewed items (a few heavy ones)
        i = np.minimum((rng.pareto(1.2, n) * 50).astype(np.int64), ni - 1).astype(np.int32)
        out.append(one(f"rand{n}", u, i, nu, ni, B, C, ns))
    if "--small" not in sys.argv:
        u, i, _ = bench.synth(1_000_000, 100_000, 100_000_000)
        out.append(one("c3", u, i, 1_000_000, 100_000, 256, 4, 32))
    for r in out:
        print(json.dumps(r))


if __name__ == "__main__":
    main()

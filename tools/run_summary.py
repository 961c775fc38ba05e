#!/usr/bin/env python
"""One-screen summary of a tools/gpu.sh output directory:
python tools/run_summary.py gpurun_out/TAG [kernel-name-fragment ...]

Prints the pytest tail of each test step, the key fields of each bench JSON
line (ms per step, value, phases, roofline, parity gates) and the rocprofv3
kernel-stats rows whose names contain one of the fragments."""
import csv
import glob
import json
import os
import sys

d = sys.argv[1]
frags = sys.argv[2:] or ["k_"]
for f in sorted(os.listdir(d)):
    p = os.path.join(d, f)
    if f.endswith("_test.log"):
        tail = [ln for ln in open(p).read().splitlines() if "passed" in ln or "failed" in ln]
        print(f, tail[-1] if tail else "(no pytest summary)")
    elif f.endswith(".json") and os.path.getsize(p) > 0:
        lines = [ln for ln in open(p).read().splitlines() if ln.startswith("{")]
        if not lines:
            print(f, "(no JSON line)")
            continue
        j = json.loads(lines[-1])
        roof = j.get("roofline") or {}
        par = j.get("parity") or {}
        gates = {k: v for k, v in par.items() if isinstance(v, (bool, dict)) or "diff" in k}
        print(f, f"ms={j.get('ms_per_step', 0):.4f}", f"value={j.get('value', 0):.4g}",
              "phases=" + json.dumps({k: round(v, 4) for k, v in (j.get("phases") or {}).items()
                                      if isinstance(v, float)}),
              f"roof={roof.get('kernel')}:{roof.get('frac', 0):.3f}", json.dumps(gates)[:300])
    elif os.path.isdir(p):
        for st in glob.glob(os.path.join(p, "*kernel_stats.csv")):
            for row in csv.DictReader(open(st)):
                if any(fr in row["Name"] for fr in frags):
                    print(f"  {f}: {row['Name'][:70]:70s} calls={row['Calls']:>4s} "
                          f"avg_ms={float(row['AverageNs']) / 1e6:.4f}")

"""Summarise an A/B run of tools/gpu.sh bench steps: SGD / RMSE ms per epoch, prev vs new."""
import glob
import json
import os
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ab"
for f in sorted(glob.glob(os.path.join(d, "*.json"))):
    try:
        j = json.load(open(f))
    except Exception as e:          # noqa: BLE001
        print(os.path.basename(f), "unreadable:", e)
        continue
    ph = j.get("phases", {})
    print(f"{os.path.basename(f):22s} value={j['value'] / 1e9:6.3f} G/s  "
          f"sgd={ph.get('sgd_ms_per_epoch', 0):7.3f} ms  rmse={ph.get('rmse_ms_per_epoch', 0):6.3f} ms  "
          f"final_rmse={j.get('final_rmse')}")

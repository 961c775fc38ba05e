#!/usr/bin/env python
"""Turn rocprofv3 PMC passes into measured HBM bytes per SGD launch.

Inputs (directories written by `rocprofv3 --pmc X --kernel-trace
--output-format csv -d DIR -o run`):
  calib FETCH / WRITE passes of tools/calib_fetch (known bytes: 256 MiB read
  by each k_gather dispatch, 256 MiB written by each k_scatter dispatch, in
  the SGD kernels' access shape: one 256-B row per wave-instruction);
  bench FETCH / WRITE passes of bench.py.

The guide (MI355X_MICROARCH.md, HBM) prescribes calibrating FETCH_SIZE and
WRITE_SIZE on a known byte count in your own access pattern: the correction
factors are known / counted from the calibration kernels, applied to the
bench's per-dispatch averages.  Writes profiles/traffic.json.
"""

import argparse
import collections
import csv
import json
import os


def per_kernel(path, counter):
    tot = collections.defaultdict(float)
    cnt = collections.Counter()
    for row in csv.DictReader(open(os.path.join(path, "run_counter_collection.csv"))):
        if row["Counter_Name"] != counter:
            continue
        tot[row["Kernel_Name"]] += float(row["Counter_Value"])
        cnt[row["Kernel_Name"]] += 1
    return {k: (tot[k], cnt[k]) for k in tot}


def pick(d, needle):
    for k, v in d.items():
        if needle in k:
            return v
    raise KeyError(needle)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calib-fetch", required=True)
    ap.add_argument("--calib-write", required=True)
    ap.add_argument("--bench-fetch", required=True)
    ap.add_argument("--bench-write", required=True)
    ap.add_argument("--key", default="c3/strata_persistent/float32/n1",
                    help="workload/schedule/dtype/nN: the key bench.py looks up")
    ap.add_argument("--sgd-kernel", default="k_sgd_batch",
                    help="name fragment of the SGD kernel (k_sgd_batch | k_sgd_strata)")
    ap.add_argument("--kernel-label", default=None,
                    help="kernel name stored with the entry (bench.py matches it against "
                         "the kernel its roofline names); default: --sgd-kernel")
    ap.add_argument("--out", default="profiles/traffic.json")
    ap.add_argument("--shape", default="x4", choices=["x1", "x4"],
                    help="calibration kernels matching the bench kernels' access "
                         "width: x1 = 4 B/lane (k_gather/k_scatter), x4 = 16 B/lane")
    args = ap.parse_args()

    known = 256 * (1 << 20)                       # bytes per calibration dispatch
    g, sc = ("k_gather4", "k_scatter4") if args.shape == "x4" else ("k_gather(", "k_scatter(")
    f_tot, f_n = pick(per_kernel(args.calib_fetch, "FETCH_SIZE"), g)
    w_tot, w_n = pick(per_kernel(args.calib_write, "WRITE_SIZE"), sc)
    cf = known / (f_tot / f_n * 1024.0)
    cw = known / (w_tot / w_n * 1024.0)
    res = {}
    for name, needle in (("sgd", args.sgd_kernel), ("sse", "k_sse_")):
        bf, nf = pick(per_kernel(args.bench_fetch, "FETCH_SIZE"), needle)
        bw, nw = pick(per_kernel(args.bench_write, "WRITE_SIZE"), needle)
        res[name] = {
            "dispatches": nf,
            "fetch_bytes_raw": bf / nf * 1024.0,
            "write_bytes_raw": bw / nw * 1024.0,
            "fetch_bytes": bf / nf * 1024.0 * cf,
            "write_bytes": bw / nw * 1024.0 * cw,
        }
    out = {}
    if os.path.exists(args.out):
        out = json.load(open(args.out))
    out[args.key] = {
        "kernel": args.kernel_label or args.sgd_kernel,
        "hbm_bytes_per_sgd_launch": res["sgd"]["fetch_bytes"] + res["sgd"]["write_bytes"],
        "calibration": {"shape": args.shape, "fetch_factor": cf, "write_factor": cw,
                        "known_bytes_per_dispatch": known},
        "kernels": res,
    }
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    json.dump(out, open(args.out, "w"), indent=1)
    print(json.dumps(out[args.key], indent=1))


if __name__ == "__main__":
    main()

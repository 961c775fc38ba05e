#!/bin/bash
# strata B sweep for the small configs (C2, one rank's share of C3 at N=8)
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/blocks
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 150 python -u bench.py --workload c2 --steps 20 --warmup 2 --cpu-sample 0 > $O/c2_default.json 2> $O/c2_default.log
for b in 128 192 256; do
  timeout -k 10 150 python -u bench.py --workload c2 --steps 20 --warmup 2 --cpu-sample 0 --blocks $b > $O/c2_b$b.json 2> $O/c2_b$b.log
done
for b in 192 224 256; do
  timeout -k 10 150 python -u bench.py --workload c3_shard8 --steps 20 --warmup 2 --cpu-sample 0 --blocks $b > $O/s8_b$b.json 2> $O/s8_b$b.log
done
echo done

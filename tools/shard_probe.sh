#!/bin/bash
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/shard
mkdir -p $O
cd $GRAFT_REPO_ROOT
for w in c3_shard8 c3_shard4 c3_shard2; do
  timeout -k 10 200 python -u bench.py --workload $w --steps 10 --warmup 2 --cpu-sample 0 > $O/$w.json 2> $O/$w.log
done
echo done

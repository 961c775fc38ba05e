#!/bin/bash
# Same-box A/B of the persistent strata pipeline depth (MF_STRATA_DEEP=0/1):
# strata GPU tests first, then the N=8 shard, the N=4 / N=2 shards, C2, C3.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-ab_deep}
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_strata.py -x -q --timeout 120 --timeout-method thread > $O/pytest_strata.log 2>&1
for w in c3_shard8 c3_shard4 c2 c3_shard8 c3; do
  for d in 0 1; do
    MF_STRATA_DEEP=$d timeout -k 10 200 python -u bench.py --workload $w --steps 10 --warmup 2 --cpu-sample 0 > $O/${w}_d${d}_$(date +%s).json 2> $O/${w}_d${d}.log
  done
done
echo done

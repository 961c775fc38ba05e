#!/bin/bash
# GPU suite, default bench, N=8 shard probe.
set -e
TAG=${1:-q}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.log
timeout -k 10 200 python -u bench.py --workload c3_shard8 --steps 10 --warmup 2 --cpu-sample 0 > $O/shard8.json 2> $O/shard8.log
echo done

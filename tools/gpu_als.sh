#!/bin/bash
# First GPU run of the factor ALS: parity tests, then the small and C5 benches.
set -e
TAG=${1:-als}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_als.py -v --timeout 120 --timeout-method thread > $O/pytest_als.log 2>&1
timeout -k 10 300 python -u bench.py --workload c5_small --steps 3 --warmup 1 > $O/bench_c5_small.json 2> $O/bench_c5_small.log
timeout -k 10 600 python -u bench.py --workload c5 --steps 3 --warmup 1 > $O/bench_c5.json 2> $O/bench_c5.log
echo done

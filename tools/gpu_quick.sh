#!/bin/bash
# GPU check after a kernel change: strata parity first, the whole -m gpu
# suite, then the default bench.  Outputs under gpurun_out/$TAG.
set -e
TAG=${1:-quick}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_strata.py -x -v --timeout 120 --timeout-method thread > $O/pytest_strata.log 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 400 python -u bench.py "${@:2}" > $O/bench.json 2> $O/bench.log
echo done

#!/bin/bash
# GPU suite + default bench.
set -e
TAG=${1:-q}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.log
echo done

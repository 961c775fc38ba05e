#!/bin/bash
# GPU tests, default bench, public fit() wall time at C3 (native preprocessing).
set -e
TAG=${1:-r01e}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.log
timeout -k 10 300 python -u tools/fit_walltime.py > $O/fit_walltime_native.json 2> $O/fit_walltime_native.log
echo done

#!/bin/bash
# One GPU call: gpu tests, default bench, rocprofv3 kernel-trace stats and
# FETCH/WRITE PMC passes (+ calibration).  Outputs under gpurun_out/$TAG.
set -e
TAG=${1:-r01b}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python $R/bench.py --steps 5 --warmup 1 --cpu-sample 0 > $O/bench_trace.json 2> $O/bench_trace.log
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/calib_fetch -o run -- $R/tools/calib_fetch > $O/calib_fetch.log 2>&1
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/calib_write -o run -- $R/tools/calib_fetch > $O/calib_write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_fetch -o run -- python $R/bench.py --steps 2 --warmup 1 --cpu-sample 0 --no-phase-timing > $O/pmc_fetch.json 2> $O/pmc_fetch.log
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_write -o run -- python $R/bench.py --steps 2 --warmup 1 --cpu-sample 0 --no-phase-timing > $O/pmc_write.json 2> $O/pmc_write.log
echo done

#!/bin/bash
# GPU tests; public fit() wall time at C3 (native and pandas preprocessing);
# C5 ALS bench + rocprofv3 kernel stats.
set -e
TAG=${1:-r01f}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python -u tools/fit_walltime.py > $O/fit_walltime_native.json 2> $O/fit_walltime_native.log
timeout -k 10 300 python -u tools/fit_walltime.py --pandas-prep > $O/fit_walltime_pandas.json 2> $O/fit_walltime_pandas.log
timeout -k 10 400 python -u bench.py --workload c5 --steps 3 --warmup 1 > $O/bench_c5.json 2> $O/bench_c5.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c5 -o run -- python $R/bench.py --workload c5 --steps 2 --warmup 1 --cpu-sample 0 > $O/bench_c5_trace.json 2> $O/bench_c5_trace.log
echo done

#!/bin/bash
# first GPU run of the stratified sweep: parity tests, then small + c3 benches
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s1; mkdir -p $O
cd $R
timeout -k 10 300 python -m pytest tests/test_gpu_strata.py -x -q > $O/pytest_strata.log 2>&1
timeout -k 10 200 python bench.py --workload small --steps 3 --warmup 1 --cpu-sample 1000000 > $O/bench_small_strata.json 2> $O/bench_small_strata.log
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --cpu-sample 2000000 > $O/bench_c3_strata.json 2> $O/bench_c3_strata.log
echo done

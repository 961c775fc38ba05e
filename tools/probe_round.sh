#!/bin/bash
# probes: P-in-MALL workload sweep + re-calibrated PMC for the float4 layout
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/probe; mkdir -p $O
timeout -k 10 400 python $R/tools/sweep_sgd.py --workload c3_u250k --rounds 2 > $O/sweep_u250k.json 2> $O/sweep_u250k.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/calib_fetch -o run -- $R/tools/calib_fetch > $O/calib_fetch.log 2>&1
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/calib_write -o run -- $R/tools/calib_fetch > $O/calib_write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_fetch -o run -- python $R/bench.py --steps 2 --warmup 1 --cpu-sample 0 --no-phase-timing > $O/pmc_fetch.json 2> $O/pmc_fetch.log
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_write -o run -- python $R/bench.py --steps 2 --warmup 1 --cpu-sample 0 --no-phase-timing > $O/pmc_write.json 2> $O/pmc_write.log
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $O/pmc_tcc -o run -- python $R/bench.py --steps 2 --warmup 1 --cpu-sample 0 --no-phase-timing > $O/pmc_tcc.json 2> $O/pmc_tcc.log
echo done

#!/bin/bash
# user-row cache-policy sweep on c3 + L2 hit counters per policy
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/pol; mkdir -p $O
timeout -k 10 500 python $R/tools/sweep_sgd.py --workload c3 --rounds 2 > $O/sweep_c3.json 2> $O/sweep_c3.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $O/pmc_tcc -o run -- python $R/tools/sweep_sgd.py --workload c3 --rounds 1 --variants s4_nt,s4,p3,p4,p6 > $O/pmc_tcc.json 2> $O/pmc_tcc.log
echo done

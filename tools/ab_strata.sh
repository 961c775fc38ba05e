#!/bin/bash
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/ab
mkdir -p $O
cd $GRAFT_REPO_ROOT
PREV=$GRAFT_REPO_ROOT/matrix-factorization_amd/matrix_factorization/libmf_hip_prev.so
for rep in 1 2; do
  MF_HIP_LIB=$PREV timeout -k 10 200 python -u bench.py --workload c3_shard8 --steps 20 --warmup 2 --cpu-sample 0 > $O/s8_prev_$rep.json 2> $O/s8_prev_$rep.log
  timeout -k 10 200 python -u bench.py --workload c3_shard8 --steps 20 --warmup 2 --cpu-sample 0 > $O/s8_new_$rep.json 2> $O/s8_new_$rep.log
done
MF_HIP_LIB=$PREV timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --cpu-sample 0 > $O/c3_prev.json 2> $O/c3_prev.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --cpu-sample 0 > $O/c3_new.json 2> $O/c3_new.log
echo done

#!/bin/bash
# Same-box A/B of the strata sweep: libmf_hip_prev.so (MF_HIP_LIB) vs the
# in-tree build, at the N=8 shard, C3 and C2; GPU strata tests first.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-ab}
mkdir -p $O
cd $GRAFT_REPO_ROOT
PREV=$GRAFT_REPO_ROOT/matrix-factorization_amd/matrix_factorization/libmf_hip_prev.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_strata.py tests/test_gpu_distributed.py -x -q --timeout 120 --timeout-method thread > $O/pytest_strata.log 2>&1
for rep in 1 2; do
  MF_HIP_LIB=$PREV timeout -k 10 200 python -u bench.py --workload c3_shard8 --steps 20 --warmup 2 --cpu-sample 0 > $O/s8_prev_$rep.json 2> $O/s8_prev_$rep.log
  timeout -k 10 200 python -u bench.py --workload c3_shard8 --steps 20 --warmup 2 --cpu-sample 0 > $O/s8_new_$rep.json 2> $O/s8_new_$rep.log
done
for w in c3 c2; do
  MF_HIP_LIB=$PREV timeout -k 10 300 python -u bench.py --workload $w --steps 10 --warmup 2 --cpu-sample 0 > $O/${w}_prev.json 2> $O/${w}_prev.log
  timeout -k 10 300 python -u bench.py --workload $w --steps 10 --warmup 2 --cpu-sample 0 > $O/${w}_new.json 2> $O/${w}_new.log
done
echo done

#!/bin/bash
# GPU suite, default bench, and an N=2 rehearsal of bench.py's sharded path
# (gloo, both ranks on cuda:0, C2 so both persistent grids are co-resident).
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r01k}
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --workload c2 --backend gloo --steps 5 --warmup 1 > $O/bench_c2_n2_gloo.json 2> $O/bench_c2_n2_gloo.log
echo done

#!/bin/bash
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/ssepmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
R=$GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU --kernel-trace --output-format csv -d $O/p1 -o run -- python $R/tools/sse_probe.py 3:0 1:0 > $O/p1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $O/p2 -o run -- python $R/tools/sse_probe.py 3:0 1:0 > $O/p2.log 2>&1
echo done

#!/bin/bash
# PMC passes (one counter group per rocprofv3 run) on a short bench run.
# Usage: tools/pmc_sgd.sh OUTDIR [bench args...]
set -e
OUT=$1; shift
cd /tmp && export TMPDIR=/tmp
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"; do
  tag=$(echo $grp | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/pmc_$tag -o run -- python $GRAFT_REPO_ROOT/bench.py --cpu-sample 0 --no-phase-timing "$@" > $OUT/pmc_$tag.json 2> $OUT/pmc_$tag.log
done

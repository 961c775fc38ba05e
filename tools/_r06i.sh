set -e
mkdir -p gpurun_out/r06i
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 rocprofv3 -L > gpurun_out/r06i/avail.txt 2>&1 || true
grep -i -n "pc\|sampl" gpurun_out/r06i/avail.txt | head -50 > gpurun_out/r06i/avail_pc.txt || true
timeout -k 10 400 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles --pc-sampling-interval 1048576 -d gpurun_out/r06i/pcs -o pcs --output-format csv -- python bench.py --workload topk --steps 5 --warmup 2 > gpurun_out/r06i/pcs.log 2>&1

set -e
bash tools/gpu.sh r06g py:tools/shuffle_hugepage_probe.py
bash tools/gpu.sh r06g2 test:tests/test_gpu_bench_multi.py
bash tools/gpu.sh r06g3 dist:2:--workload,c3,--steps,2,--warmup,1

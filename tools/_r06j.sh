set -e
bash tools/gpu.sh r06j bench:--workload,topk,--steps,20,--warmup,3 test:tests/test_gpu_parity.py,-k,topk

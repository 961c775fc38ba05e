set -e
bash tools/gpu.sh r06m test:tests/test_gpu_parity.py,-k,topk bench:--workload,topk,--steps,20,--warmup,3 trace:--workload,topk,--steps,20,--warmup,3

set -e
bash tools/gpu.sh r06b py:tools/sse_tiles_probe.py:--dtype,float64,1,8,1,16d,1,16,4,16,8,16,2,32,4,32,8,8,16,8,1,8
bash tools/gpu.sh r06b2 py:tools/sse_tiles_probe.py:--dtype,float32,1,8,4,16,8,8,1,16
bash tools/gpu.sh r06b3 test:tests/test_gpu_sse.py,tests/test_gpu_distributed.py,tests/test_gpu_recovery.py,tests/test_gpu_bench_multi.py,--durations=20

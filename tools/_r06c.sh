set -e
bash tools/gpu.sh r06c py:tools/sse_tiles_probe.py:--dtype,float64,1x8,1x16d,1x16,4x16,8x16,2x32,4x32,8x8,16x8,1x8
bash tools/gpu.sh r06c2 py:tools/sse_tiles_probe.py:--dtype,float32,1x8,4x16,8x8,1x16,1x8
bash tools/gpu.sh r06c3 py:tools/shuffle_time.py env:MF_SHUFFLE_THREADS=1 py:tools/shuffle_time.py
bash tools/gpu.sh r06c4 py:tools/strata_probe.py:--workload,c2 py:tools/strata_probe.py:--workload,c3,--rotate,8
bash tools/gpu.sh r06c5 test:tests/test_gpu_sse.py,tests/test_gpu_distributed.py,tests/test_gpu_recovery.py,tests/test_gpu_bench_multi.py,--durations=20

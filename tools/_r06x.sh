set -e
bash tools/gpu.sh r06x test:tests/test_gpu_sse.py env:SSE_PROBE_DTYPE=float64 py:tools/sse_probe.py:0:0,0:0 env:SSE_PROBE_DTYPE=float32 py:tools/sse_probe.py:0:0,0:0

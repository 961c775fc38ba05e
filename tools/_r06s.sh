set -e
bash tools/gpu.sh r06s test:tests/test_gpu_sse.py,-k,gs32 env:SSE_PROBE_DTYPE=float64 py:tools/sse_probe.py:0:0,13:0,0:0,13:0 env:SSE_PROBE_DTYPE=float32 py:tools/sse_probe.py:0:0,13:0

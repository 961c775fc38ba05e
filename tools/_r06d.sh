set -e
bash tools/gpu.sh r06d env:SSE_PROBE_DTYPE=float64 py:tools/sse_probe.py:0:0,12:0,0:0,12:0 env:SSE_PROBE_DTYPE=float32 py:tools/sse_probe.py:0:0,12:0,0:0,12:0
bash tools/gpu.sh r06d2 test:tests/test_gpu_sse.py
bash tools/gpu.sh r06d5 py:tools/shuffle_time.py env:MF_SHUFFLE_THREADS=2 py:tools/shuffle_time.py env:MF_SHUFFLE_AHEAD=1024 py:tools/shuffle_time.py
bash tools/gpu.sh r06d3 py:tools/fit_walltime.py:--dtype,float32 py:tools/fit_walltime.py:--schedule,exact,--dtype,float64,--epochs,5
bash tools/gpu.sh r06d4 env:PY_TIMEOUT=1000 py:tools/frontier_probe.py:--designs,rotate,rotprod8,--out,gpurun_out/r06d4/frontier.json

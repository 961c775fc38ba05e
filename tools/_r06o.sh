set -e
bash tools/gpu.sh r06o2 py:tools/fit_walltime.py:--dtype,float32 py:tools/fit_walltime.py:--dtype,float32 py:tools/fit_walltime.py:--dtype,float64 test:tests/test_gpu_parity.py,tests/test_gpu_configs.py

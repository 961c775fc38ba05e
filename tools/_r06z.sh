set -e
bash tools/gpu.sh r06z py:tools/fit_walltime.py:--dtype,float64 py:tools/fit_walltime.py:--dtype,float64 test:tests/test_gpu_strata.py,tests/test_gpu_configs.py,tests/test_gpu_distributed.py

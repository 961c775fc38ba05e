set -e
bash tools/gpu.sh r06t test:tests/test_gpu_shuffle.py py:tools/fit_walltime.py:--dtype,float32 py:tools/fit_walltime.py:--dtype,float32

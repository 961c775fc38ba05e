set -e
bash tools/gpu.sh r06w test:tests/test_gpu_shuffle.py py:tools/exact_probe.py py:tools/fit_walltime.py:--schedule,exact,--dtype,float64,--epochs,5

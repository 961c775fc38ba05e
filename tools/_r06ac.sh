set -e
bash tools/gpu.sh r06ac env:MF_PLAN_TIMING=1 py:tools/plan_concurrency.py env:MF_PLAN_TIMING= py:tools/fit_walltime.py:--dtype,float32 py:tools/fit_walltime.py:--dtype,float32 py:tools/fit_walltime.py:--dtype,float64 test:tests/test_gpu_strata.py,tests/test_gpu_configs.py

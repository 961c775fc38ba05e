set -e
bash tools/gpu.sh r06ae env:MF_PLAN_TIMING=1 py:tools/plan_concurrency.py env:MF_PLAN_TIMING= py:tools/fit_walltime.py:--dtype,float32 test:tests/test_gpu_strata.py,tests/test_gpu_configs.py,tests/test_gpu_distributed.py smoke

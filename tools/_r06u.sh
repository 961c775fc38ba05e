set -e
bash tools/gpu.sh r06u env:MF_PLAN_TIMING=1 py:tools/plan_concurrency.py

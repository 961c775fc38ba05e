set -e
bash tools/gpu.sh r06p py:tools/exact_probe.py

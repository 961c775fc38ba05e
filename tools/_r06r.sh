set -e
bash tools/gpu.sh r06r py:tools/exact_probe.py

set -e
bash tools/gpu.sh r06e py:tools/shuffle_time.py env:MF_SHUFFLE_PF=32 py:tools/shuffle_time.py env:MF_SHUFFLE_PF=96 py:tools/shuffle_time.py env:MF_SHUFFLE_SIMD=0 py:tools/shuffle_time.py
bash tools/gpu.sh r06e2 py:tools/fit_walltime.py:--schedule,exact,--dtype,float64,--epochs,5 py:tools/fit_walltime.py:--dtype,float32
bash tools/gpu.sh r06e3 test:tests,--durations=25 smoke

set -e
bash tools/gpu.sh r06h2 env:MF_SHUFFLE_PAR_TRACE=1 py:tools/shuffle_time.py env:MF_SHUFFLE_PAR_TRACE= py:tools/fit_walltime.py:--schedule,exact,--dtype,float64,--epochs,5 py:tools/fit_walltime.py:--dtype,float32 env:MF_SHUFFLE_PAR=0 py:tools/fit_walltime.py:--schedule,exact,--dtype,float64,--epochs,5 py:tools/fit_walltime.py:--dtype,float32

set -e
bash tools/gpu.sh r06f env:MF_SHUFFLE_PF=96 py:tools/shuffle_time.py env:MF_SHUFFLE_PF=128 py:tools/shuffle_time.py env:MF_SHUFFLE_PF=192 py:tools/shuffle_time.py env:MF_SHUFFLE_PF=248 py:tools/shuffle_time.py
bash tools/gpu.sh r06f2 py:tools/fit_walltime.py:--schedule,exact,--dtype,float64,--epochs,5
bash tools/gpu.sh r06f3 bench:--gpus,1,--steps,20,--warmup,5 trace:--steps,10,--warmup,2,--cpu-sample,0
bash tools/gpu.sh r06f4 bench:--workload,c2,--steps,20,--warmup,5 bench:--emulate-rank,8,--steps,10,--warmup,3

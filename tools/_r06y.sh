set -e
bash tools/gpu.sh r06y test:tests,--durations=25 smoke bench:--gpus,1,--steps,20,--warmup,5 trace:--gpus,1,--steps,20,--warmup,5

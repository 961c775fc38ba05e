set -e
bash tools/gpu.sh r06v test:tests,--durations=25 smoke bench:--gpus,1,--steps,20,--warmup,5

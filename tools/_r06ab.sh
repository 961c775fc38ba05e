set -e
bash tools/gpu.sh r06ab test:tests,--durations=15 smoke bench:--gpus,1,--steps,20,--warmup,5

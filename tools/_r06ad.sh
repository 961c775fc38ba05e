set -e
bash tools/gpu.sh r06ad test:tests,--durations=10 smoke bench:--gpus,1,--steps,20,--warmup,5

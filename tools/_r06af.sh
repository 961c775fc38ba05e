set -e
bash tools/gpu.sh r06af test:tests smoke bench:--gpus,1,--steps,20,--warmup,5

set -e
B=bench:--workload,topk,--steps,20,--warmup,3
bash tools/gpu.sh r06l env:MF_TOPK_MM_DEFER=2 $B env:MF_TOPK_MM_DEFER= env:MF_TOPK_MM_SPLITS=12 $B env:MF_TOPK_MM_SPLITS=4 $B env:MF_TOPK_MM_SPLITS= env:MF_TOPK_MW_FILL=16 $B env:MF_TOPK_MW_FILL= $B

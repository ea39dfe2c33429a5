#!/bin/bash
# Secondary BASELINE configs on one GPU: yolox_l fp16 bs16 inference (configs[3]),
# yolox_x 1280 fp16 train step (configs[4], per-GPU batch), plus every tile variant's
# time for the yolox_s bs32 bf16 forward (YOLOX_AMD_TUNE_ALL=1).
# Usage (from the repo root on the box): bash tools/gpu_configs.sh TAG
set -o pipefail
TAG=${1:-run}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
YOLOX_AMD_TUNE_ALL=1 timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline \
    > gpurun_out/variants_$TAG.json 2> gpurun_out/variants_$TAG.err || exit 1
timeout -k 10 300 python bench.py --model yolox_l --dtype fp16 --batch 16 --cpu-seconds 10 \
    > gpurun_out/bench_l_$TAG.json 2> gpurun_out/bench_l_$TAG.err || exit 1
timeout -k 10 400 python bench.py --workload train --model yolox_x --size 1280 --batch 8 --dtype fp16 \
    --steps 5 --warmup 2 --cpu-seconds 10 > gpurun_out/bench_xtrain_$TAG.json 2> gpurun_out/bench_xtrain_$TAG.err || exit 1
echo "done"

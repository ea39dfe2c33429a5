#!/bin/bash
# GPU box: 16-bit training with the inference kernels as tuner candidates: train tests, configs[4]
# (yolox_x 1280 fp16 bs8) and yolox_s bf16 train bench.  Usage: bash tools/gpu_r3x.sh TAG
set -o pipefail
TAG=${1:-r3x}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_configs.py -q -x --timeout 200 \
    --timeout-method thread -k "train" > gpurun_out/tests_$TAG.log 2>&1 || { tail -30 gpurun_out/tests_$TAG.log; exit 1; }
tail -2 gpurun_out/tests_$TAG.log
timeout -k 10 400 python bench.py --workload train --model yolox_x --size 1280 --dtype fp16 --batch 8 --steps 6 --warmup 3 \
    --no-cpu-baseline > gpurun_out/train_x_$TAG.json 2> gpurun_out/train_x_$TAG.err || exit 1
cat gpurun_out/train_x_$TAG.json
timeout -k 10 300 python bench.py --workload train --dtype bf16 --steps 10 --warmup 3 --no-cpu-baseline \
    > gpurun_out/train_s16_$TAG.json 2> gpurun_out/train_s16_$TAG.err || exit 1
cat gpurun_out/train_s16_$TAG.json

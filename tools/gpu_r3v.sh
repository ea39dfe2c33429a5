#!/bin/bash
# GPU box: smoke + the whole GPU suite, then configs[2] / configs[4] training benches.
set -o pipefail
TAG=${1:-r3v}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_r3_tests.sh $TAG || exit 1
timeout -k 10 300 python bench.py --workload train --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/train_${TAG}_c2.json 2> gpurun_out/train_${TAG}_c2.err || exit 1
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"frac": [0-9.]*' gpurun_out/train_${TAG}_c2.json | tr '\n' ' '; echo " configs2"
timeout -k 10 400 python bench.py --workload train --model yolox_x --size 1280 --dtype fp16 --batch 8 --steps 6 --warmup 3 \
    --no-cpu-baseline > gpurun_out/train_${TAG}_c4.json 2> gpurun_out/train_${TAG}_c4.err || exit 1
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"frac": [0-9.]*' gpurun_out/train_${TAG}_c4.json | tr '\n' ' '; echo " configs4"
YOLOX_AMD_WGRAD_STREAM=0 timeout -k 10 300 python bench.py --workload train --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/train_${TAG}_c2_inline.json 2> gpurun_out/train_${TAG}_c2_inline.err || exit 1
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"frac": [0-9.]*' gpurun_out/train_${TAG}_c2_inline.json | tr '\n' ' '; echo " configs2 wgrad inline"

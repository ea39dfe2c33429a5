#!/bin/bash
# GPU box: nine-tap fp32 wgrad tests + fp32 train bench (configs[2]) with shapes; configs[4] with the
# 16-bit inference tiles as tuner candidates vs the base tiles.  Usage: bash tools/gpu_r3y.sh TAG
set -o pipefail
TAG=${1:-r3y}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -q -x --timeout 150 --timeout-method thread \
    -k "wgrad9t or kmajor or deterministic or train_step_fp32" > gpurun_out/tests_$TAG.log 2>&1 || { tail -30 gpurun_out/tests_$TAG.log; exit 1; }
tail -2 gpurun_out/tests_$TAG.log
timeout -k 10 300 python bench.py --workload train --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/train_$TAG.json 2> gpurun_out/train_$TAG.err || exit 1
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"frac": [0-9.]*\|"host_issue_ms_per_step": [0-9.]*' gpurun_out/train_$TAG.json | tr '\n' ' '; echo " configs2"
for T in all base; do
  YOLOX_AMD_TRAIN_TILES16=$T timeout -k 10 400 python bench.py --workload train --model yolox_x --size 1280 --dtype fp16 \
      --batch 8 --steps 6 --warmup 3 --no-cpu-baseline > gpurun_out/train_x_${TAG}_$T.json 2> gpurun_out/train_x_${TAG}_$T.err || exit 1
  grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"host_issue_ms_per_step": [0-9.]*' gpurun_out/train_x_${TAG}_$T.json | tr '\n' ' '; echo " configs4 tiles=$T"
done
YOLOX_AMD_TRAIN_LOG=gpurun_out/train_log_$TAG.json timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/prof_train_$TAG \
    -o run --output-format csv -- python bench.py --workload train --steps 4 --warmup 3 --no-cpu-baseline \
    > gpurun_out/prof_train_$TAG.json 2> gpurun_out/prof_train_$TAG.log || exit 1
python tools/train_shapes.py gpurun_out/prof_train_$TAG/run_kernel_trace.csv gpurun_out/train_log_$TAG.json \
    > gpurun_out/train_shapes_$TAG.txt 2>&1; head -30 gpurun_out/train_shapes_$TAG.txt
python tools/trace_window.py gpurun_out/prof_train_$TAG/run_kernel_trace.csv 3 | head -16

#!/bin/bash
# GPU box: new-kernel tests (conv_pw1f, wgrad1), per-layer inference table (frag weights), training
# step per-launch shapes under rocprofv3, train bench.  Usage: bash tools/gpu_r3t.sh TAG
set -o pipefail
TAG=${1:-r3t}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_train.py -q -x --timeout 150 \
    --timeout-method thread -k "pw1f or kmajor or wgrad9t or deterministic or train_step or stride2 or wgrad_and_dgrad or wgrad_tiles or batched" > gpurun_out/tests_$TAG.log 2>&1 || { tail -30 gpurun_out/tests_$TAG.log; exit 1; }
tail -2 gpurun_out/tests_$TAG.log
timeout -k 10 300 python bench.py --workload train --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/train_$TAG.json 2> gpurun_out/train_$TAG.err || exit 1
cat gpurun_out/train_$TAG.json
YOLOX_AMD_TRAIN_LOG=gpurun_out/train_log_$TAG.json timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/prof_train_$TAG \
    -o run --output-format csv -- python bench.py --workload train --steps 4 --warmup 3 --no-cpu-baseline \
    > gpurun_out/prof_train_$TAG.json 2> gpurun_out/prof_train_$TAG.log || exit 1
python tools/train_shapes.py gpurun_out/prof_train_$TAG/run_kernel_trace.csv gpurun_out/train_log_$TAG.json \
    > gpurun_out/train_shapes_$TAG.txt 2>&1; head -50 gpurun_out/train_shapes_$TAG.txt
timeout -k 10 300 python bench.py --layers --no-cpu-baseline > gpurun_out/bench_${TAG}_layers.json 2> gpurun_out/layers_$TAG.txt || exit 1
tail -66 gpurun_out/layers_$TAG.txt

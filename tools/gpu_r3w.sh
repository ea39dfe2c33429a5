#!/bin/bash
# GPU box: fp32 1x1 wgrad tiles + frag-layout conv tests, then train bench (no profiler) and its profile.
# Usage: bash tools/gpu_r3w.sh TAG
set -o pipefail
TAG=${1:-r3w}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_ops.py -q -x --timeout 150 \
    --timeout-method thread -k "wgrad1 or conv_ws or frag or batched" > gpurun_out/tests_$TAG.log 2>&1 || { tail -30 gpurun_out/tests_$TAG.log; exit 1; }
tail -3 gpurun_out/tests_$TAG.log
timeout -k 10 300 python bench.py --workload train --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/train_$TAG.json 2> gpurun_out/train_$TAG.err || exit 1
cat gpurun_out/train_$TAG.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_train_$TAG -o run --output-format csv \
    -- python bench.py --workload train --steps 8 --warmup 3 --no-cpu-baseline \
    > gpurun_out/prof_train_$TAG.json 2> gpurun_out/prof_train_$TAG.log || exit 1
echo done

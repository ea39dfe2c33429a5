#!/bin/bash
# GPU box: optimizer + training tests, yolox_s train bench, rocprofv3 stats of it.
# Usage: bash tools/gpu_train_q.sh TAG
set -o pipefail
TAG=${1:-run}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_optim.py tests/test_gpu_train.py -x -q --timeout 120 \
    --timeout-method thread -rf > gpurun_out/train_tests_$TAG.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --workload train > gpurun_out/train_bench_$TAG.json 2> gpurun_out/train_bench_$TAG.err || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/trainprof_$TAG -o run --output-format csv \
    -- python bench.py --workload train --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/trainprof_$TAG.log 2>&1
echo "done rc=$?"

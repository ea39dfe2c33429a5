#!/bin/bash
# GPU-box session for the training path: parity tests, then the train bench with the
# by-shape default tiles and with on-device tile tuning.  Usage: bash tools/gpu_train_perf.sh TAG
set -o pipefail
TAG=${1:-run}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_simota.py -m gpu -x -q --timeout 240 \
    --timeout-method thread -rf > gpurun_out/train_tests_$TAG.log 2>&1 || exit $?
YOLOX_AMD_TRAIN_TUNE=0 timeout -k 10 300 python -u bench.py --workload train --steps 10 --warmup 3 --no-cpu-baseline \
    > gpurun_out/train_bench_notune_$TAG.json 2> gpurun_out/train_bench_notune_$TAG.err || exit $?
timeout -k 10 300 python -u bench.py --workload train --steps 10 --warmup 3 --no-cpu-baseline \
    > gpurun_out/train_bench_$TAG.json 2> gpurun_out/train_bench_$TAG.err || exit $?
echo "done"

#!/bin/bash
# GPU box: kernel + model tests, the head probe, then the bench twice (second run reuses the
# tune file: run-to-run spread).  Usage: bash tools/gpu_k3.sh TAG
set -o pipefail
TAG=${1:-run}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py tests/test_gpu_configs.py \
    tests/test_gpu_processor.py -m gpu -x -q --timeout 300 --timeout-method thread -rf > gpurun_out/k3_$TAG.log 2>&1
rc=$?
echo "pytest exit=$rc" >> gpurun_out/k3_$TAG.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 python tools/head_pmc.py > gpurun_out/k3_head_$TAG.txt 2>&1 || exit 1
timeout -k 10 500 python bench.py --layers --no-cpu-baseline --tune-file gpurun_out/tune_$TAG.json \
    > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --tune-file gpurun_out/tune_$TAG.json \
    > gpurun_out/bench2_$TAG.json 2> gpurun_out/bench2_$TAG.err || exit 1
echo "done"

#!/bin/bash
# GPU box: probe + full GPU tests + bench (tune file per tag) + yolox_x train bench.
# Usage: bash tools/gpu_quick.sh TAG
set -o pipefail
TAG=${1:-run}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python tools/pw_probe.py > gpurun_out/probe_$TAG.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -rf \
    > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?
echo "pytest exit=$rc" >> gpurun_out/gpu_tests_$TAG.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python bench.py --layers > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 1
timeout -k 10 400 python bench.py --workload train --model yolox_x --size 1280 --batch 8 --dtype fp16 \
    --steps 5 --warmup 2 --cpu-seconds 10 > gpurun_out/bench_xtrain_$TAG.json 2> gpurun_out/bench_xtrain_$TAG.err
echo "done"

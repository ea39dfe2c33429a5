#!/bin/bash
# GPU box: conv_ws probe + its parity tests, then all GPU tests and the bench.
# Usage: bash tools/gpu_ws.sh TAG
set -o pipefail
TAG=${1:-run}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ws_probe.py > gpurun_out/ws_probe_$TAG.txt 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k conv_ws -x -q --timeout 120 --timeout-method thread -rf \
    > gpurun_out/ws_tests_$TAG.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -rf \
    > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?
echo "pytest exit=$rc" >> gpurun_out/gpu_tests_$TAG.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python bench.py --layers --no-cpu-baseline --tune-file gpurun_out/tune_$TAG.json \
    > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 1
echo "done"

#!/bin/bash
# GPU box, round 3: new-kernel tests first, then the whole GPU suite, then bench variants.
set -o pipefail
TAG=${1:-r3b}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -k "stem_s2" -x -q \
    --timeout 120 --timeout-method thread > gpurun_out/s2_tests_$TAG.log 2>&1
rc=$?; echo "s2 tests exit=$rc" >> gpurun_out/s2_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread -rf --durations=10 \
    > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?
echo "pytest exit=$rc" >> gpurun_out/gpu_tests_$TAG.log
[ $rc -le 1 ] || exit $rc
TF=gpurun_out/tune_$TAG.json
timeout -k 10 300 python bench.py --no-cpu-baseline --layers --tune-file $TF > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --tune-file gpurun_out/tune_${TAG}_16.json --chunk 16 --par-chunks > gpurun_out/bench_${TAG}_par2.json 2> gpurun_out/bench_${TAG}_par2.err || exit 1
for v in "" _par2; do python -c "import json,sys; d=json.load(open('gpurun_out/bench_${TAG}$v.json')); print('$v', d['value'], d['roofline']['forward_ms'])"; done

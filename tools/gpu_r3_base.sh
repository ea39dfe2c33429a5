#!/bin/bash
# GPU box, round 3 baseline: smoke, every GPU test, one default bench line.
set -o pipefail
TAG=${1:-r3base}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -rf --durations=15 \
    > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?
echo "pytest exit=$rc" >> gpurun_out/gpu_tests_$TAG.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 1
cat gpurun_out/bench_$TAG.json

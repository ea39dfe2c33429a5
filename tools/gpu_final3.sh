#!/bin/bash
# GPU box, end of round 2: smoke, all GPU tests, bench (default: CPU baseline + per-layer table,
# tune file written), rocprofv3 kernel stats of the same command, PMC traffic passes.
# Usage: bash tools/gpu_final3.sh TAG
set -o pipefail
TAG=${1:-run}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -rf \
    > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?
echo "pytest exit=$rc" >> gpurun_out/gpu_tests_$TAG.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python bench.py --layers --tune-file gpurun_out/tune_$TAG.json > gpurun_out/bench_$TAG.json \
    2> gpurun_out/bench_$TAG.err || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv \
    -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --tune-file gpurun_out/tune_$TAG.json \
    > gpurun_out/prof_$TAG.log 2>&1 || exit 1
bash tools/pmc_traffic.sh $TAG gpurun_out/tune_$TAG.json || exit 1
echo "done"

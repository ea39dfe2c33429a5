#!/bin/bash
# One GPU-box session: parity tests, benchmark (+ per-op table), rocprofv3 kernel stats.
# Usage (from the repo root on the box): bash tools/gpu_check.sh TAG
set -o pipefail
TAG=${1:-run}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q --timeout 300 -rf > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?
echo "pytest exit=$rc" >> gpurun_out/gpu_tests_$TAG.log
# 1 = ordinary test failures; anything else (abort, segfault, timeout) ends the session
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python bench.py --layers --tune-file gpurun_out/tune_$TAG.json > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv \
    -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --tune-file gpurun_out/tune_$TAG.json \
    > gpurun_out/prof_$TAG.log 2>&1
echo "done rc=$?"

#!/bin/bash
# GPU box: bench (tune file) + rocprofv3 kernel-trace stats of the same bench.  Usage: bash tools/gpu_prof.sh TAG
set -o pipefail
TAG=${1:-run}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python bench.py --layers --no-cpu-baseline --tune-file gpurun_out/tune_$TAG.json \
    > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv \
    -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --tune-file gpurun_out/tune_$TAG.json \
    > gpurun_out/prof_$TAG.log 2>&1 || exit 1
echo "done"

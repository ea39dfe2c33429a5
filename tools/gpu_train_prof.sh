#!/bin/bash
# rocprofv3 kernel stats of the training bench (tuned tiles).  Usage: bash tools/gpu_train_prof.sh TAG
set -o pipefail
TAG=${1:-run}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_train_$TAG -o run --output-format csv \
    -- python bench.py --workload train --steps 10 --warmup 3 --no-cpu-baseline \
    > gpurun_out/prof_train_$TAG.json 2> gpurun_out/prof_train_$TAG.log
echo "done rc=$?"

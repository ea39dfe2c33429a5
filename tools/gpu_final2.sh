#!/bin/bash
# GPU box, round-2 evidence: smoke, bench (default, with the CPU baseline), the same with
# Bottleneck fusion off, configs[3] (yolox_l fp16 bs16), rocprofv3 kernel stats of the bench.
# Usage: bash tools/gpu_final2.sh TAG
set -o pipefail
TAG=${1:-run}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --layers --tune-file gpurun_out/tune_$TAG.json > gpurun_out/bench_$TAG.json \
    2> gpurun_out/bench_$TAG.err || exit 1
YOLOX_AMD_FUSE_BOTTLENECK=0 timeout -k 10 400 python bench.py --no-cpu-baseline \
    > gpurun_out/bench_nofuse_$TAG.json 2> gpurun_out/bench_nofuse_$TAG.err || exit 1
timeout -k 10 400 python bench.py --model yolox_l --batch 16 --dtype fp16 --no-cpu-baseline \
    > gpurun_out/bench_l_$TAG.json 2> gpurun_out/bench_l_$TAG.err || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv \
    -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --tune-file gpurun_out/tune_$TAG.json \
    > gpurun_out/prof_$TAG.log 2>&1 || exit 1
echo "done"

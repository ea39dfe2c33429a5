#!/bin/bash
# GPU box (round 3, session 2): bench, launch-cost probes, then smoke + the whole GPU suite.
# Usage: bash tools/gpu_r3s.sh TAG
set -o pipefail
TAG=${1:-r3s}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 1
cat gpurun_out/bench_$TAG.json
timeout -k 10 200 python tools/batch_probe.py "3 40 128 128 171" "3 80 64 64 166" "3 80 128 256 185" \
    "3 20 256 256 176" "1 40 128 128 103" "1 80 128 128 203" "1 80 64 64 97" "1 20 1024 512 99" \
    > gpurun_out/batch_probe_$TAG.txt 2>&1 || exit 1
cat gpurun_out/batch_probe_$TAG.txt
bash tools/gpu_r3_tests.sh $TAG

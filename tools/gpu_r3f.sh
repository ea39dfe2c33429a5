#!/bin/bash
# GPU box: fragment-major weight A/B: launch-cost probe (both layouts), bench with and without.
# Usage: bash tools/gpu_r3f.sh TAG
set -o pipefail
TAG=${1:-r3f}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python tools/batch_probe.py "3 40 128 128 171" "3 80 64 64 166" "3 80 128 256 185" \
    "3 20 256 256 176" "1 80 128 128 203" "1 40 256 256 205" "3 160 32 32 178" \
    > gpurun_out/batch_probe_$TAG.txt 2>&1 || exit 1
cat gpurun_out/batch_probe_$TAG.txt
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_${TAG}_frag.json 2> gpurun_out/bench_${TAG}_frag.err || exit 1
YOLOX_AMD_WFRAG=0 timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_${TAG}_row.json 2> gpurun_out/bench_${TAG}_row.err || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_${TAG}_frag2.json 2> gpurun_out/bench_${TAG}_frag2.err || exit 1
grep -o '"value": [0-9.]*\|"forward_ms": [0-9.]*' gpurun_out/bench_${TAG}_*.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_train_$TAG -o run --output-format csv \
    -- python bench.py --workload train --steps 8 --warmup 3 --no-cpu-baseline \
    > gpurun_out/prof_train_$TAG.json 2> gpurun_out/prof_train_$TAG.log || exit 1
python tools/trace_window.py $(ls gpurun_out/prof_train_$TAG/*/run_kernel_trace.csv gpurun_out/prof_train_$TAG/run_kernel_trace.csv 2>/dev/null | head -1) 5 \
    > gpurun_out/train_window_$TAG.txt 2>&1; cat gpurun_out/train_window_$TAG.txt

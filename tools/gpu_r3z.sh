#!/bin/bash
# GPU box: configs[4] diagnostics -- per-kernel-family step breakdown under rocprofv3.
set -o pipefail
TAG=${1:-r3z}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 rocprofv3 --kernel-trace -d gpurun_out/prof_trainx_$TAG -o run --output-format csv \
    -- python bench.py --workload train --model yolox_x --size 1280 --dtype fp16 --batch 8 --steps 3 --warmup 2 \
    --no-cpu-baseline > gpurun_out/prof_trainx_$TAG.json 2> gpurun_out/prof_trainx_$TAG.log || exit 1
python tools/trace_window.py gpurun_out/prof_trainx_$TAG/run_kernel_trace.csv 2 | head -30
YOLOX_AMD_BATCH_PACK=0 timeout -k 10 400 python bench.py --workload train --model yolox_x --size 1280 --dtype fp16 \
    --batch 8 --steps 6 --warmup 3 --no-cpu-baseline > gpurun_out/train_x_${TAG}_nobatch.json 2>&1 || exit 1
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"host_issue_ms_per_step": [0-9.]*\|"last_loss": [0-9.]*' gpurun_out/train_x_${TAG}_nobatch.json | tr '\n' ' '; echo " no batch pack"

#!/bin/bash
# round 5: per-stream step windows of the current tree (configs[4] and configs[2] captured) + train PMC traffic
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
C4="--workload train --model yolox_x --size 1280 --dtype fp16 --batch 8 --no-cpu-baseline"
YOLOX_AMD_TRAIN_GRAPH=1 timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_train_r5s_c4 -o run --output-format csv \
    -- python bench.py $C4 --steps 4 --warmup 3 > gpurun_out/prof_train_r5s_c4.json 2> gpurun_out/prof_train_r5s_c4.log || exit 1
python tools/trace_streams.py gpurun_out/prof_train_r5s_c4/run_kernel_trace.csv 3 > gpurun_out/train_streams_r5s_c4.txt && head -30 gpurun_out/train_streams_r5s_c4.txt
python tools/trace_window.py gpurun_out/prof_train_r5s_c4/run_kernel_trace.csv 3 > gpurun_out/train_window_r5s_c4.txt && head -3 gpurun_out/train_window_r5s_c4.txt
YOLOX_AMD_TRAIN_GRAPH=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_train_r5s_c2 -o run --output-format csv \
    -- python bench.py --workload train --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/prof_train_r5s_c2.json 2> gpurun_out/prof_train_r5s_c2.log || exit 1
python tools/trace_streams.py gpurun_out/prof_train_r5s_c2/run_kernel_trace.csv 5 > gpurun_out/train_streams_r5s_c2.txt && head -24 gpurun_out/train_streams_r5s_c2.txt
python -c "import json; d=json.load(open('gpurun_out/prof_train_r5s_c4.json')); print('c4 under tracer', d['ms_per_step']); d=json.load(open('gpurun_out/prof_train_r5s_c2.json')); print('c2 under tracer', d['ms_per_step'])"

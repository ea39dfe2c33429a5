#!/bin/bash
# round 5: per-shape time of every conv / data-gradient / weight-gradient launch of one configs[4]
# step (weight gradients inline, so the trace order is the issue order the launch log records)
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
C4="--workload train --model yolox_x --size 1280 --dtype fp16 --batch 8 --no-cpu-baseline"
YOLOX_AMD_WGRAD_STREAM=0 YOLOX_AMD_TRAIN_LOG=gpurun_out/launch_log_r5f_c4.json timeout -k 10 900 rocprofv3 --kernel-trace \
    -d gpurun_out/prof_shapes_r5f_c4 -o run --output-format csv -- python bench.py $C4 --steps 2 --warmup 2 \
    > gpurun_out/prof_shapes_r5f_c4.log 2>&1 || { tail -5 gpurun_out/prof_shapes_r5f_c4.log; exit 1; }
python tools/train_shapes.py gpurun_out/prof_shapes_r5f_c4/run_kernel_trace.csv gpurun_out/launch_log_r5f_c4.json \
    > gpurun_out/train_shapes_r5f_c4.txt && head -60 gpurun_out/train_shapes_r5f_c4.txt

#!/bin/bash
# round 5: conv_pwf's fp32-gradient epilogue (1x1 data gradients of the 16-bit step): tests, configs[4]
# captured bench, per-shape table of one step
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -k "dgrad_1x1_conv_pwf or dgrad_conv_ws or dgrad_s2_parity" -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/tests_r5h.log 2>&1 || { grep -E "^E |Error|FAILED|passed|failed" gpurun_out/tests_r5h.log | head -30; exit 1; }
tail -1 gpurun_out/tests_r5h.log
C4="--workload train --model yolox_x --size 1280 --dtype fp16 --batch 8 --no-cpu-baseline"
YOLOX_AMD_TRAIN_GRAPH=1 timeout -k 10 600 python -u bench.py $C4 --steps 6 --warmup 3 > gpurun_out/train_r5h_c4_graph.json 2> gpurun_out/train_r5h_c4_graph.err || { tail -5 gpurun_out/train_r5h_c4_graph.err; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], 'img/s', d['ms_per_step'], 'ms/step frac', d['roofline']['frac'])" gpurun_out/train_r5h_c4_graph.json
YOLOX_AMD_WGRAD_STREAM=0 YOLOX_AMD_TRAIN_LOG=gpurun_out/launch_log_r5h_c4.json timeout -k 10 900 rocprofv3 --kernel-trace \
    -d gpurun_out/prof_shapes_r5h_c4 -o run --output-format csv -- python bench.py $C4 --steps 2 --warmup 2 \
    > gpurun_out/prof_shapes_r5h_c4.log 2>&1 || { tail -5 gpurun_out/prof_shapes_r5h_c4.log; exit 1; }
python tools/train_shapes.py gpurun_out/prof_shapes_r5h_c4/run_kernel_trace.csv gpurun_out/launch_log_r5h_c4.json \
    > gpurun_out/train_shapes_r5h_c4.txt && grep -E "last step|dgrad +k1" gpurun_out/train_shapes_r5h_c4.txt | head -20

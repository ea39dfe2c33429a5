#!/bin/bash
# round 5: head lanes hoisted next to their inputs (engine.hoist_lanes) and the 16-bit parity-class
# stride-2 data gradient (dgrad_s2h, tiles 217-220): tests, inference bench A/B against the neck-first
# capture order (YOLOX_AMD_LANE_HOIST=0), configs[4] training bench (captured), kernel trace + timeline
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TESTS="tests/test_gpu_model.py tests/test_gpu_train.py -k 'dgrad_s2_parity or dgrad_conv_ws or graph_forms or graph_replay or chunk'" \
AB="YOLOX_AMD_LANE_HOIST=0 DEFAULT=1 YOLOX_AMD_LANE_HOIST=0 DEFAULT=1" bash tools/gpu_iter.sh r5d || exit 1
C4="--workload train --model yolox_x --size 1280 --dtype fp16 --batch 8 --no-cpu-baseline"
YOLOX_AMD_TRAIN_GRAPH=1 timeout -k 10 600 python -u bench.py $C4 --steps 6 --warmup 3 > gpurun_out/train_r5d_c4_graph.json 2> gpurun_out/train_r5d_c4_graph.err || { tail -5 gpurun_out/train_r5d_c4_graph.err; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], 'img/s', d['ms_per_step'], 'ms/step frac', d['roofline']['frac'])" gpurun_out/train_r5d_c4_graph.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r5d -o run --output-format csv \
    -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof_r5d.log 2>&1 || exit 1
python tools/forward_timeline.py gpurun_out/prof_r5d/run_kernel_trace.csv > gpurun_out/timeline_r5d.txt 2>&1 || true
tail -30 gpurun_out/timeline_r5d.txt

#!/bin/bash
# round 5 training evidence: configs[4] (yolox_x 1280 fp16 bs8) and configs[2] (yolox_s 640 fp32 bs8) benches,
# eager and captured (YOLOX_AMD_TRAIN_GRAPH=1), and a rocprofv3 kernel trace of each captured bench whose
# per-step window (tools/trace_window.py) is compared with the bench's ms_per_step
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TUNE4=gpurun_out/tune_train_c4.json
C4="--workload train --model yolox_x --size 1280 --dtype fp16 --batch 8 --no-cpu-baseline"
C2="--workload train --no-cpu-baseline"
summ() { python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], 'img/s', d['ms_per_step'], 'ms/step frac', d['roofline']['frac'], 'host', d.get('host_issue_ms_per_step'))" $1; }
timeout -k 10 600 python -u bench.py $C4 --steps 6 --warmup 3 > gpurun_out/train_r5_c4.json 2> gpurun_out/train_r5_c4.err || { tail -5 gpurun_out/train_r5_c4.err; exit 1; }
summ gpurun_out/train_r5_c4.json
YOLOX_AMD_TRAIN_GRAPH=1 timeout -k 10 600 python -u bench.py $C4 --steps 6 --warmup 3 > gpurun_out/train_r5_c4_graph.json 2> gpurun_out/train_r5_c4_graph.err || { tail -5 gpurun_out/train_r5_c4_graph.err; exit 1; }
summ gpurun_out/train_r5_c4_graph.json
timeout -k 10 300 python -u bench.py $C2 --steps 10 --warmup 3 > gpurun_out/train_r5_c2.json 2> gpurun_out/train_r5_c2.err || { tail -5 gpurun_out/train_r5_c2.err; exit 1; }
summ gpurun_out/train_r5_c2.json
YOLOX_AMD_TRAIN_GRAPH=1 timeout -k 10 300 python -u bench.py $C2 --steps 10 --warmup 3 > gpurun_out/train_r5_c2_graph.json 2> gpurun_out/train_r5_c2_graph.err || { tail -5 gpurun_out/train_r5_c2_graph.err; exit 1; }
summ gpurun_out/train_r5_c2_graph.json
YOLOX_AMD_TRAIN_GRAPH=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_train_r5_c2 -o run --output-format csv \
    -- python bench.py $C2 --steps 10 --warmup 3 > gpurun_out/prof_train_r5_c2.json 2> gpurun_out/prof_train_r5_c2.log || exit 1
python tools/trace_window.py gpurun_out/prof_train_r5_c2/run_kernel_trace.csv 5 > gpurun_out/train_window_r5_c2.txt && head -12 gpurun_out/train_window_r5_c2.txt
YOLOX_AMD_TRAIN_GRAPH=1 timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_train_r5_c4 -o run --output-format csv \
    -- python bench.py $C4 --steps 4 --warmup 3 > gpurun_out/prof_train_r5_c4.json 2> gpurun_out/prof_train_r5_c4.log || exit 1
python tools/trace_window.py gpurun_out/prof_train_r5_c4/run_kernel_trace.csv 3 > gpurun_out/train_window_r5_c4.txt && head -16 gpurun_out/train_window_r5_c4.txt

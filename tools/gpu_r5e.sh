#!/bin/bash
# round 5: BatchNorm reduction occupancy (BWD unroll 2, <= 512 blocks), separable SPP backward,
# 16-bit parity-class stride-2 data gradient: training tests, BN probe (per-kernel split, block cap
# A/B), configs[4] / configs[2] benches and the configs[4] per-stream step window
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/tests_r5e_train.log 2>&1 || { grep -E "^E |Error|FAILED|passed|failed" gpurun_out/tests_r5e_train.log | head -30; exit 1; }
tail -2 gpurun_out/tests_r5e_train.log
for cap in 512 1024; do
  YXH_RED_BLOCKS=$cap timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bn_r5e_$cap -o run --output-format csv \
      -- python tools/bn_probe.py 10 > gpurun_out/bn_probe_r5e_$cap.txt 2>&1 || { tail -5 gpurun_out/bn_probe_r5e_$cap.txt; exit 1; }
  echo "cap $cap"; grep -v "^\[\|^W\|^E" gpurun_out/bn_probe_r5e_$cap.txt | grep "TB/s"
done
C4="--workload train --model yolox_x --size 1280 --dtype fp16 --batch 8 --no-cpu-baseline"
YOLOX_AMD_TRAIN_GRAPH=1 timeout -k 10 600 python -u bench.py $C4 --steps 6 --warmup 3 > gpurun_out/train_r5e_c4_graph.json 2> gpurun_out/train_r5e_c4_graph.err || { tail -5 gpurun_out/train_r5e_c4_graph.err; exit 1; }
YOLOX_AMD_MAIN_PRIORITY=1 YOLOX_AMD_TRAIN_GRAPH=1 timeout -k 10 600 python -u bench.py $C4 --steps 6 --warmup 3 > gpurun_out/train_r5e_c4_graph_prio.json 2> gpurun_out/train_r5e_c4_graph_prio.err || { tail -5 gpurun_out/train_r5e_c4_graph_prio.err; exit 1; }
timeout -k 10 300 python -u bench.py --workload train --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/train_r5e_c2.json 2> gpurun_out/train_r5e_c2.err || { tail -5 gpurun_out/train_r5e_c2.err; exit 1; }
for f in train_r5e_c4_graph train_r5e_c4_graph_prio train_r5e_c2; do
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], 'img/s', d['ms_per_step'], 'ms/step frac', d['roofline']['frac'])" gpurun_out/$f.json
done
YOLOX_AMD_TRAIN_GRAPH=1 timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_train_r5e_c4 -o run --output-format csv \
    -- python bench.py $C4 --steps 4 --warmup 3 > gpurun_out/prof_train_r5e_c4.json 2> gpurun_out/prof_train_r5e_c4.log || exit 1
python tools/trace_streams.py gpurun_out/prof_train_r5e_c4/run_kernel_trace.csv 3 > gpurun_out/train_streams_r5e_c4.txt && head -32 gpurun_out/train_streams_r5e_c4.txt

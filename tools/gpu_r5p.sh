#!/bin/bash
# round 5: benches of the final tree -- the default (configs[1]) line twice, configs[3], configs[4] captured,
# configs[2] eager and captured
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
summ() { python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], d['unit'], d['ms_per_step'], 'ms/step frac', d['roofline']['frac'])" $1; }
for i in 1 2; do
  timeout -k 10 300 python -u bench.py > gpurun_out/bench_r5p_$i.json 2> gpurun_out/bench_r5p_$i.err || { tail -5 gpurun_out/bench_r5p_$i.err; exit 1; }
  summ gpurun_out/bench_r5p_$i.json
done
timeout -k 10 300 python -u bench.py --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/bench_r5p_long.json 2> gpurun_out/bench_r5p_long.err || { tail -5 gpurun_out/bench_r5p_long.err; exit 1; }
summ gpurun_out/bench_r5p_long.json
timeout -k 10 300 python -u bench.py --model yolox_l --batch 16 --dtype fp16 --no-cpu-baseline > gpurun_out/bench_r5p_c3.json 2> gpurun_out/bench_r5p_c3.err || { tail -5 gpurun_out/bench_r5p_c3.err; exit 1; }
summ gpurun_out/bench_r5p_c3.json
C4="--workload train --model yolox_x --size 1280 --dtype fp16 --batch 8 --no-cpu-baseline"
YOLOX_AMD_TRAIN_GRAPH=1 timeout -k 10 600 python -u bench.py $C4 --steps 6 --warmup 3 > gpurun_out/train_r5p_c4_graph.json 2> gpurun_out/train_r5p_c4_graph.err || { tail -5 gpurun_out/train_r5p_c4_graph.err; exit 1; }
summ gpurun_out/train_r5p_c4_graph.json
timeout -k 10 300 python -u bench.py --workload train --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/train_r5p_c2.json 2> gpurun_out/train_r5p_c2.err || { tail -5 gpurun_out/train_r5p_c2.err; exit 1; }
summ gpurun_out/train_r5p_c2.json
YOLOX_AMD_TRAIN_GRAPH=1 timeout -k 10 300 python -u bench.py --workload train --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/train_r5p_c2_graph.json 2> gpurun_out/train_r5p_c2_graph.err || { tail -5 gpurun_out/train_r5p_c2_graph.err; exit 1; }
summ gpurun_out/train_r5p_c2_graph.json

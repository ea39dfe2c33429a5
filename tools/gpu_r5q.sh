#!/bin/bash
# round 5: head-form fusion per level (YOLOX_AMD_HEAD_FUSION) re-measured with the round-5 kernels
cd "${GRAFT_REPO_ROOT:-.}"
AB="DEFAULT=1 YOLOX_AMD_HEAD_FUSION=2 YOLOX_AMD_HEAD_FUSION=1,2 DEFAULT=1 YOLOX_AMD_HEAD_FUSION=2 YOLOX_AMD_HEAD_FUSION=1,2" bash tools/gpu_iter.sh r5q
summ() { python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], d['unit'], d['ms_per_step'], 'ms/step frac', d['roofline']['frac'])" $1; }
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --workload train --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/train_r5q_c2_$i.json 2> gpurun_out/train_r5q_c2_$i.err || { tail -5 gpurun_out/train_r5q_c2_$i.err; exit 1; }
  summ gpurun_out/train_r5q_c2_$i.json
done
C4="--workload train --model yolox_x --size 1280 --dtype fp16 --batch 8 --no-cpu-baseline"
YOLOX_AMD_TRAIN_GRAPH=1 timeout -k 10 600 python -u bench.py $C4 --steps 6 --warmup 3 > gpurun_out/train_r5q_c4_graph.json 2> gpurun_out/train_r5q_c4_graph.err || { tail -5 gpurun_out/train_r5q_c4_graph.err; exit 1; }
summ gpurun_out/train_r5q_c4_graph.json

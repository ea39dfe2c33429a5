#!/bin/bash
# round 5: weight-gradient grid size (YXH_WGRAD_BLOCKS) vs the main stream's BN reductions: configs[4]
# captured and configs[2] eager
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
summ() { python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[1].split('/')[-1], d['value'], d['unit'], d['ms_per_step'], 'ms/step frac', d['roofline']['frac'])" $1 "$2"; }
C4="--workload train --model yolox_x --size 1280 --dtype fp16 --batch 8 --no-cpu-baseline --steps 6 --warmup 3"
for b in 512 256 384 512 256; do
  YXH_WGRAD_BLOCKS=$b YOLOX_AMD_TRAIN_GRAPH=1 timeout -k 10 600 python -u bench.py $C4 > gpurun_out/train_r5t_c4_$b.json 2> gpurun_out/train_r5t_c4_$b.err || { tail -5 gpurun_out/train_r5t_c4_$b.err; exit 1; }
  summ gpurun_out/train_r5t_c4_$b.json "blocks $b"
done
for b in 512 256; do
  YXH_WGRAD_BLOCKS=$b timeout -k 10 300 python -u bench.py --workload train --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/train_r5t_c2_$b.json 2> gpurun_out/train_r5t_c2_$b.err || { tail -5 gpurun_out/train_r5t_c2_$b.err; exit 1; }
  summ gpurun_out/train_r5t_c2_$b.json "blocks $b"
done

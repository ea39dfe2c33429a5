#!/bin/bash
# round 5: configs[3] on the final tree; BN reduction grid cap (YXH_RED_BLOCKS) 256 / 384 vs 512 on
# configs[2] eager and configs[4] captured, alternating
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
summ() { python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['unit'], d['ms_per_step'], 'ms/step frac', d['roofline']['frac'])" $1 "$2"; }
timeout -k 10 300 python -u bench.py --model yolox_l --batch 16 --dtype fp16 --no-cpu-baseline > gpurun_out/bench_r5y_c3.json 2> gpurun_out/bench_r5y_c3.err || { tail -5 gpurun_out/bench_r5y_c3.err; exit 1; }
summ gpurun_out/bench_r5y_c3.json "configs3"
C2="--workload train --no-cpu-baseline --steps 20 --warmup 5"
for b in 512 256 384 512 256 384; do
  YXH_RED_BLOCKS=$b timeout -k 10 300 python -u bench.py $C2 > gpurun_out/train_r5y_c2_$b.json 2> gpurun_out/train_r5y_c2.err || { tail -5 gpurun_out/train_r5y_c2.err; exit 1; }
  summ gpurun_out/train_r5y_c2_$b.json "c2 red $b"
done
C4="--workload train --model yolox_x --size 1280 --dtype fp16 --batch 8 --no-cpu-baseline --steps 6 --warmup 3"
for b in 512 256 512 256; do
  YXH_RED_BLOCKS=$b YOLOX_AMD_TRAIN_GRAPH=1 timeout -k 10 600 python -u bench.py $C4 > gpurun_out/train_r5y_c4_$b.json 2> gpurun_out/train_r5y_c4.err || { tail -5 gpurun_out/train_r5y_c4.err; exit 1; }
  summ gpurun_out/train_r5y_c4_$b.json "c4 red $b"
done

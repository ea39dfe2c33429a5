#!/bin/bash
# round 5: chan_finalize as 64 channels x 16 waves of coalesced partial rows vs the wave-per-channel
# form (ab/libyoloxhip_oldfin.so = HEAD's train.hip), configs[2] eager and configs[4] captured, alternating
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
summ() { python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['unit'], d['ms_per_step'], 'ms/step frac', d['roofline']['frac'])" $1 "$2"; }
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_train.py -k "bn_ or spp or train_step" > gpurun_out/tests_r5v.log 2>&1 || { tail -20 gpurun_out/tests_r5v.log; exit 1; }
tail -1 gpurun_out/tests_r5v.log
OLD=$PWD/ab/libyoloxhip_oldfin.so
C2="--workload train --no-cpu-baseline --steps 20 --warmup 5"
C4="--workload train --model yolox_x --size 1280 --dtype fp16 --batch 8 --no-cpu-baseline --steps 6 --warmup 3"
for i in 1 2; do
  timeout -k 10 300 python -u bench.py $C2 > gpurun_out/train_r5v_c2_new$i.json 2> gpurun_out/train_r5v_c2.err || { tail -5 gpurun_out/train_r5v_c2.err; exit 1; }
  summ gpurun_out/train_r5v_c2_new$i.json "c2 new"
  YOLOX_AMD_LIB=$OLD timeout -k 10 300 python -u bench.py $C2 > gpurun_out/train_r5v_c2_old$i.json 2> gpurun_out/train_r5v_c2.err || { tail -5 gpurun_out/train_r5v_c2.err; exit 1; }
  summ gpurun_out/train_r5v_c2_old$i.json "c2 old"
done
for i in 1 2; do
  YOLOX_AMD_TRAIN_GRAPH=1 timeout -k 10 600 python -u bench.py $C4 > gpurun_out/train_r5v_c4_new$i.json 2> gpurun_out/train_r5v_c4.err || { tail -5 gpurun_out/train_r5v_c4.err; exit 1; }
  summ gpurun_out/train_r5v_c4_new$i.json "c4 new"
  YOLOX_AMD_LIB=$OLD YOLOX_AMD_TRAIN_GRAPH=1 timeout -k 10 600 python -u bench.py $C4 > gpurun_out/train_r5v_c4_old$i.json 2> gpurun_out/train_r5v_c4.err || { tail -5 gpurun_out/train_r5v_c4.err; exit 1; }
  summ gpurun_out/train_r5v_c4_old$i.json "c4 old"
done

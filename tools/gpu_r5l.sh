#!/bin/bash
# round 5: two output slots in the inference serving loop (Plan.capture(slots=2)): graph tests, bench A/B
# against the one-slot pipeline (--one-slot), alternating
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q --timeout 250 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_model.py -k "graph_replay or graph_forms or chunk" > gpurun_out/tests_r5l.log 2>&1 || { grep -E "^E |FAILED" gpurun_out/tests_r5l.log | head; exit 1; }
tail -1 gpurun_out/tests_r5l.log
i=0
for f in "--one-slot" "" "--one-slot" ""; do
  i=$((i + 1))
  timeout -k 10 300 python -u bench.py --no-cpu-baseline $f > gpurun_out/bench_r5l_$i.json 2> gpurun_out/bench_r5l_$i.err || { tail -5 gpurun_out/bench_r5l_$i.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2] or 'two-slot', d['value'], 'img/s', d['ms_per_step'], 'ms/step fwd', d['roofline']['forward_ms'])" gpurun_out/bench_r5l_$i.json "$f"
done
C4="--workload train --model yolox_x --size 1280 --dtype fp16 --batch 8 --no-cpu-baseline"
for e in "YOLOX_AMD_WGRAD_STREAM=0" "DEFAULT=1"; do
  env $e YOLOX_AMD_TRAIN_GRAPH=1 timeout -k 10 600 python -u bench.py $C4 --steps 6 --warmup 3 > gpurun_out/train_r5l_c4_$e.json 2> gpurun_out/train_r5l_c4_$e.err || { tail -5 gpurun_out/train_r5l_c4_$e.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], 'img/s', d['ms_per_step'], 'ms/step frac', d['roofline']['frac'])" gpurun_out/train_r5l_c4_$e.json $e
done

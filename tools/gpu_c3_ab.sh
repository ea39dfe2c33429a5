#!/bin/bash
# GPU box: configs[3] (yolox_l fp16 bs16) bench with the in-tree library vs $BASE_LIB (a previous build),
# alternating REPS times, after the op tests named by K (pytest -k) on the in-tree library.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-c3ab}
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -m gpu -x -q --timeout 300 --timeout-method thread \
      -p no:cacheprovider -k "$K" > gpurun_out/ops_$T.log 2>&1 || { tail -30 gpurun_out/ops_$T.log; exit 1; }
  tail -1 gpurun_out/ops_$T.log
fi
for i in $(seq 1 ${REPS:-2}); do
  for v in new base; do
    if [ $v = base ]; then LIBV="$PWD/$BASE_LIB"; else LIBV=""; fi
    env ${LIBV:+YOLOX_AMD_LIB=$LIBV} timeout -k 10 400 python -u bench.py --no-cpu-baseline --model yolox_l --batch 16 \
        --dtype fp16 --layers > gpurun_out/bench_${T}_${v}_$i.json 2> gpurun_out/bench_${T}_${v}_$i.err \
        || { tail -5 gpurun_out/bench_${T}_${v}_$i.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], 'img/s fwd', d['roofline']['forward_ms'], 'frac', d['roofline']['frac'])" gpurun_out/bench_${T}_${v}_$i.json $v
  done
done
grep -a "tune op" gpurun_out/bench_${T}_new_1.err | grep "k3" | head -40

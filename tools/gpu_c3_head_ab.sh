#!/bin/bash
# GPU box: configs[3] with the 256-channel head_pred2 + score records (in-tree library) vs $BASE_LIB with the row filter
# (--no-scores), alternating, after the head / scored-filter tests.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-c3h}
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_postprocess.py -m gpu -x -q --timeout 300 \
    --timeout-method thread -p no:cacheprovider -k "head_pred_fused or scored_filter" > gpurun_out/ops_$T.log 2>&1 \
    || { tail -30 gpurun_out/ops_$T.log; exit 1; }
tail -1 gpurun_out/ops_$T.log
B="--no-cpu-baseline --model yolox_l --batch 16 --dtype fp16 --tune-file gpurun_out/tune_$T.json"
rm -f gpurun_out/tune_$T.json
for i in $(seq 1 ${REPS:-3}); do
  for v in new base; do
    if [ $v = base ]; then
      YOLOX_AMD_LIB=$PWD/$BASE_LIB timeout -k 10 400 python -u bench.py $B --no-scores > gpurun_out/bench_${T}_${v}_$i.json 2> gpurun_out/bench_${T}_${v}_$i.err || { tail -5 gpurun_out/bench_${T}_${v}_$i.err; exit 1; }
    else
      timeout -k 10 400 python -u bench.py $B > gpurun_out/bench_${T}_${v}_$i.json 2> gpurun_out/bench_${T}_${v}_$i.err || { tail -5 gpurun_out/bench_${T}_${v}_$i.err; exit 1; }
    fi
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], 'img/s fwd', d['roofline']['forward_ms'], 'step', d['ms_per_step'], 'frac', d['roofline']['frac'], d['config']['nms_filter'])" gpurun_out/bench_${T}_${v}_$i.json $v
  done
done

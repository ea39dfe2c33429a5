#!/bin/bash
# GPU box: captured training step tests, then the configs[2] / configs[4] train bench eager vs
# hipGraph replay (YOLOX_AMD_TRAIN_GRAPH=1).  Usage: bash tools/gpu_captrain.sh TAG
set -o pipefail
TAG=${1:-cap}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -m gpu -x -v -k "captured or batched" --timeout 200 \
    --timeout-method thread > gpurun_out/captests_$TAG.log 2>&1; rc=$?
grep -E "PASSED|FAILED|Error|passed|failed" gpurun_out/captests_$TAG.log | tail -12
[ $rc -eq 0 ] || exit $rc
run() {  # name, env, args
  local name=$1 envs=$2; shift 2
  env $envs timeout -k 10 400 python -u bench.py --workload train --no-cpu-baseline "$@" \
      > gpurun_out/train_${TAG}_$name.json 2> gpurun_out/train_${TAG}_$name.err || return $?
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['config'].get('issue'), d.get('host_issue_ms_per_step'))" gpurun_out/train_${TAG}_$name.json $name
}
run c2_eager "YOLOX_AMD_TRAIN_GRAPH=0" --steps 20 --warmup 3 || exit $?
run c2_graph "YOLOX_AMD_TRAIN_GRAPH=1" --steps 20 --warmup 3 || exit $?
run c4_eager "YOLOX_AMD_TRAIN_GRAPH=0" --model yolox_x --size 1280 --dtype fp16 --batch 8 --steps 6 --warmup 2 || exit $?
run c4_graph "YOLOX_AMD_TRAIN_GRAPH=1" --model yolox_x --size 1280 --dtype fp16 --batch 8 --steps 6 --warmup 2 || exit $?

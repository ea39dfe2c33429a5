#!/bin/bash
# GPU box: graph forms x GPU_MAX_HW_QUEUES (does a head lane share a hardware queue with
# the neck?).  One tune file for all runs.
set -o pipefail
TAG=${1:-r3d}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TF=gpurun_out/tune_${TAG}.json
run() {  # name env... -- bench args
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --tune-file $TF --steps 30 \
      > gpurun_out/bench_${TAG}_$name.json 2> gpurun_out/bench_${TAG}_$name.err || return 1
  python -c "import json; d=json.load(open('gpurun_out/bench_${TAG}_$name.json')); print('$name', d['value'], d['roofline']['forward_ms'])"
}
run lanes_q4 GPU_MAX_HW_QUEUES=4 || exit 1
run lanes_q8 GPU_MAX_HW_QUEUES=8 || exit 1
run lanes_q16 GPU_MAX_HW_QUEUES=16 || exit 1
run dag_q8 GPU_MAX_HW_QUEUES=8 YOLOX_AMD_GRAPH=dag || exit 1
run dag_q16 GPU_MAX_HW_QUEUES=16 YOLOX_AMD_GRAPH=dag || exit 1
env GPU_MAX_HW_QUEUES=8 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_${TAG}_q8 -o run --output-format csv \
    -- python bench.py --steps 6 --warmup 2 --no-cpu-baseline --tune-file $TF > gpurun_out/prof_${TAG}_q8.log 2>&1 || exit 1
echo done

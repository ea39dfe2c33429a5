#!/bin/bash
# GPU box: graph forms tests, then lanes vs streams bench (+ a kernel trace of streams).
set -o pipefail
TAG=${1:-r3e}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -k "graph_forms or submodules or stem" -x -q \
    --timeout 120 --timeout-method thread > gpurun_out/e_tests_$TAG.log 2>&1
rc=$?; echo "exit=$rc" >> gpurun_out/e_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
TF=gpurun_out/tune_${TAG}.json
for mode in lanes streams lanes streams; do
  YOLOX_AMD_GRAPH=$mode timeout -k 10 300 python bench.py --no-cpu-baseline --tune-file $TF --steps 30 \
      > gpurun_out/bench_${TAG}_$mode.json 2> gpurun_out/bench_${TAG}_$mode.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/bench_${TAG}_$mode.json')); print('$mode', d['value'], d['roofline']['forward_ms'])"
done
YOLOX_AMD_GRAPH=streams timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_${TAG}_streams -o run --output-format csv \
    -- python bench.py --steps 6 --warmup 2 --no-cpu-baseline --tune-file $TF > gpurun_out/prof_${TAG}_streams.log 2>&1 || exit 1
echo done

#!/bin/bash
# GPU box, round 3: smoke, every GPU test, then bench variants of the graph form
# (dag default, lanes, parallel chunks 2 / 4) sharing one tune file.
set -o pipefail
TAG=${1:-r3a}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread -rf --durations=15 \
    > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?
echo "pytest exit=$rc" >> gpurun_out/gpu_tests_$TAG.log
[ $rc -le 1 ] || exit $rc
TF=gpurun_out/tune_$TAG.json
timeout -k 10 300 python bench.py --no-cpu-baseline --tune-file $TF > gpurun_out/bench_${TAG}_dag.json 2> gpurun_out/bench_${TAG}_dag.err || exit 1
YOLOX_AMD_GRAPH=lanes timeout -k 10 300 python bench.py --no-cpu-baseline --tune-file $TF > gpurun_out/bench_${TAG}_lanes.json 2> gpurun_out/bench_${TAG}_lanes.err || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --tune-file $TF --chunk 16 --par-chunks > gpurun_out/bench_${TAG}_par2.json 2> gpurun_out/bench_${TAG}_par2.err || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --tune-file gpurun_out/tune_${TAG}_8.json --chunk 8 --par-chunks > gpurun_out/bench_${TAG}_par4.json 2> gpurun_out/bench_${TAG}_par4.err || exit 1
for v in dag lanes par2 par4; do python -c "import json,sys; d=json.load(open('gpurun_out/bench_${TAG}_$v.json')); print('$v', d['value'], d['roofline']['forward_ms'])"; done

#!/bin/bash
# GPU box: targeted tests (fp32 1x1 wgrad tiles, conv_ws / ws1 incl. frag, batched repack), inference
# bench with / without the L2 weight prefetch, train bench.  Usage: bash tools/gpu_r3w.sh TAG
set -o pipefail
TAG=${1:-r3w}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_ops.py tests/test_gpu_model.py -q -x \
    --timeout 150 --timeout-method thread -k "wgrad1 or conv_ws or frag or batched or model" \
    > gpurun_out/tests_$TAG.log 2>&1 || { tail -30 gpurun_out/tests_$TAG.log; exit 1; }
tail -3 gpurun_out/tests_$TAG.log
for v in 1 0 1; do
  YOLOX_AMD_PREFETCH=$v timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_${TAG}_pf$v.json \
      2> gpurun_out/bench_${TAG}_pf$v.err || exit 1
  grep -o '"value": [0-9.]*\|"forward_ms": [0-9.]*' gpurun_out/bench_${TAG}_pf$v.json | tr '\n' ' '; echo " pf=$v"
done
timeout -k 10 300 python bench.py --workload train --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/train_$TAG.json 2> gpurun_out/train_$TAG.err || exit 1
cat gpurun_out/train_$TAG.json

#!/bin/bash
# GPU box: captured (hipGraph) training step: parity test, then configs[2] / configs[4] graph vs eager issue.
set -o pipefail
TAG=${1:-r3g}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_train.py \
    -k "captured or batched_weight" -m gpu > gpurun_out/captest_${TAG}.log 2>&1 || { tail -40 gpurun_out/captest_${TAG}.log; exit 1; }
tail -3 gpurun_out/captest_${TAG}.log
B="python bench.py --workload train --no-cpu-baseline"
timeout -k 10 300 $B --steps 10 --warmup 3 > gpurun_out/train_${TAG}_c2.json 2> gpurun_out/train_${TAG}_c2.err || { tail -20 gpurun_out/train_${TAG}_c2.err; exit 1; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"frac": [0-9.]*\|"issue": "[a-zA-Z ]*"' gpurun_out/train_${TAG}_c2.json | tr '\n' ' '; echo " configs2"
YOLOX_AMD_TRAIN_GRAPH=0 timeout -k 10 300 $B --steps 10 --warmup 3 > gpurun_out/train_${TAG}_c2_eager.json 2> gpurun_out/train_${TAG}_c2_eager.err || exit 1
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"frac": [0-9.]*\|"host_issue_ms_per_step": [0-9.]*' gpurun_out/train_${TAG}_c2_eager.json | tr '\n' ' '; echo " configs2 eager"
timeout -k 10 400 $B --model yolox_x --size 1280 --dtype fp16 --batch 8 --steps 6 --warmup 3 \
    > gpurun_out/train_${TAG}_c4.json 2> gpurun_out/train_${TAG}_c4.err || { tail -20 gpurun_out/train_${TAG}_c4.err; exit 1; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"frac": [0-9.]*\|"issue": "[a-zA-Z ]*"' gpurun_out/train_${TAG}_c4.json | tr '\n' ' '; echo " configs4"

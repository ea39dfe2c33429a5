#!/bin/bash
# GPU box: conv/train parity tests, then the fp32 (configs[2]) and bf16 train benches and a
# kernel trace of the fp32 one.  Usage: bash tools/gpu_train_k.sh TAG
set -o pipefail
TAG=${1:-run}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_train.py tests/test_gpu_optim.py \
    tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread -rf \
    -k "r3 or train or optim or configs2" > gpurun_out/tk_$TAG.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --workload train --steps 10 --warmup 3 --no-cpu-baseline \
    > gpurun_out/tk_fp32_$TAG.json 2> gpurun_out/tk_fp32_$TAG.err || exit $?
timeout -k 10 400 python -u bench.py --workload train --dtype bf16 --steps 10 --warmup 3 --no-cpu-baseline \
    > gpurun_out/tk_bf16_$TAG.json 2> gpurun_out/tk_bf16_$TAG.err || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tk_$TAG -o run --output-format csv \
    -- python bench.py --workload train --steps 10 --warmup 3 --no-cpu-baseline \
    > gpurun_out/prof_tk_$TAG.json 2> gpurun_out/prof_tk_$TAG.log || exit $?
echo "done"

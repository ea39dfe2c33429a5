#!/bin/bash
# GPU box: the N=2 bench path (torchrun, 2 ranks sharing the one GPU over gloo) for
# inference and training, plus the bf16-vs-fp32 training test.  Usage: bash tools/gpu_rehearse.sh TAG
set -o pipefail
TAG=${1:-run}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_train.py -q --timeout 120 --timeout-method thread -rf \
    -k "autocast" > gpurun_out/autocast_$TAG.log 2>&1 || exit 1
export YOLOX_AMD_BENCH_BACKEND=gloo
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/rehearse_infer_$TAG.json \
    2> gpurun_out/rehearse_infer_$TAG.err || exit 1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29512 bench.py --gpus 2 --workload train --steps 3 --warmup 2 > gpurun_out/rehearse_train_$TAG.json \
    2> gpurun_out/rehearse_train_$TAG.err || exit 1
echo done

#!/bin/bash
# GPU box: tests/test_gpu_ops.py (-k $K) against an alternative library build ($LIB, YOLOX_AMD_LIB); non-zero on failure
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
YOLOX_AMD_LIB=$PWD/$LIB timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -m gpu -x -q --timeout 200 \
    --timeout-method thread -k "${K:-ws1 or no_activation or pw}" > gpurun_out/ops_$TAG.log 2>&1
rc=$?
tail -3 gpurun_out/ops_$TAG.log
exit $rc

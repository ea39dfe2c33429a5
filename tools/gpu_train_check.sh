#!/bin/bash
# GPU-box session for the training path: its parity tests (+ the ABI / ops suites).
set -o pipefail
TAG=${1:-run}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_simota.py -m gpu -x -v --timeout 240 --timeout-method thread -rf > gpurun_out/train_tests_$TAG.log 2>&1
rc=$?
echo "pytest exit=$rc" >> gpurun_out/train_tests_$TAG.log
exit $rc

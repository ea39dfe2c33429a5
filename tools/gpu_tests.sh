#!/bin/bash
# GPU box: run selected GPU test files.  Usage: bash tools/gpu_tests.sh TAG test_file...
set -o pipefail
TAG=$1; shift
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest "$@" -m gpu -x -v --timeout 300 --timeout-method thread -rf \
    > gpurun_out/tests_$TAG.log 2>&1
rc=$?
echo "pytest exit=$rc" >> gpurun_out/tests_$TAG.log
tail -5 gpurun_out/tests_$TAG.log
exit $rc

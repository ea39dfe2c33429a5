#!/bin/bash
# GPU box: smoke + the whole GPU suite (as the driver runs them).
set -o pipefail
TAG=${1:-r3t}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread -rf --durations=10 \
    > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?
echo "pytest exit=$rc" >> gpurun_out/gpu_tests_$TAG.log
tail -15 gpurun_out/gpu_tests_$TAG.log
exit $rc

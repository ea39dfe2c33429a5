#!/bin/bash
# GPU box: CapturedTrainStep diagnostics, one variant per step, stop at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { echo "== $1"; env $2 timeout -k 10 120 python -u tools/cap_debug.py > gpurun_out/capdbg_$1.log 2>&1; rc=$?; grep "^[0-9] \|plan" gpurun_out/capdbg_$1.log; return $rc; }
run seg_inline "YOLOX_AMD_WGRAD_STREAM=0" &&
run seg_side "YOLOX_AMD_WGRAD_GROUP=1" &&
run seg_side_g6 "YOLOX_AMD_WGRAD_GROUP=6"

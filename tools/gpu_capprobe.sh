#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
YOLOX_AMD_WGRAD_STREAM=0 timeout -k 10 120 python -u tools/cap_probe.py interleave > gpurun_out/capprobe_interleave.log 2>&1; rc=$?
grep "^[0-9]\|captured" gpurun_out/capprobe_interleave.log; echo "interleave rc=$rc"
[ $rc -eq 0 ] || exit $rc
YOLOX_AMD_WGRAD_STREAM=0 timeout -k 10 120 python -u tools/cap_probe.py optstep > gpurun_out/capprobe_optstep.log 2>&1; rc=$?
grep "^[0-9]\|captured" gpurun_out/capprobe_optstep.log; echo "optstep rc=$rc"
exit $rc

#!/bin/bash
# GPU box: new conv_ws variants (FR = 4) vs the tuned picks, per forward 3x3 shape.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/ws_probe2.py "1 80 64 64 332" "1 80 64 64 442" "1 80 64 64 444" "1 80 64 64 446" \
  "1 40 128 128 344" "1 40 128 128 448" "1 40 128 128 450" "1 40 128 128 452" \
  "1 20 256 256 352" "1 20 256 256 454" "1 80 128 256 370" "1 80 128 256 456" "1 80 128 256 458" \
  "1 160 32 32 356" "1 160 32 32 460" "1 40 128 256 362" "1 40 128 256 450" "1 40 128 256 448" \
  "1 20 128 256 350" "1 20 128 256 448" > gpurun_out/ws_new_r3.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/ws_new_r3.txt

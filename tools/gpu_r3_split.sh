#!/bin/bash
# GPU box: conv_ws split probes (full / no stores / no halo DMA / neither) on the 3x3 shapes
# the forward spends most time in, with the tiles the tuner picks.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
SPECS=("1 80 64 64 332" "1 40 128 128 344" "1 20 256 256 352" "1 80 128 256 370" "2 80 128 256 348")
for LIBF in pixeltable-yolox_amd/yolox_amd/_lib/libyoloxhip.so dbg/libws_p1.so dbg/libws_p2.so dbg/libws_p3.so; do
  YOLOX_AMD_LIB=$LIBF timeout -k 10 120 python tools/ws_probe2.py "${SPECS[@]}" >> gpurun_out/ws_split_r3.txt 2>&1 || exit 1
done
cat gpurun_out/ws_split_r3.txt | grep -v amdgpu.ids

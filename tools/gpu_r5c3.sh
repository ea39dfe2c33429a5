#!/bin/bash
# round 5, final tree: configs[3] (yolox_l fp16 bs 16) profile -- bench + trace/stats + PMC traffic + SQ
cd "${GRAFT_REPO_ROOT:-.}"
bash tools/gpu_profile.sh r5f_c3 --model yolox_l --batch 16 --dtype fp16

#!/bin/bash
# round 5: HBM traffic per training step on the final tree, configs[4] and configs[2]
cd "${GRAFT_REPO_ROOT:-.}"
bash tools/gpu_train_traffic.sh r5t2_c4 yolox_x 8 1280 fp16 && bash tools/gpu_train_traffic.sh r5t2_c2 yolox_s 8 640 fp32

#!/bin/bash
# round 5: configs[4] fp16 step parity with the BN reduction block cap at 1024 (round-4 value) and 512
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for cap in 1024 512; do
  YXH_RED_BLOCKS=$cap timeout -k 10 400 python -u -m pytest -q -s --timeout 380 --timeout-method thread -p no:cacheprovider \
    "tests/test_gpu_configs.py::test_configs4_yolox_x_1280_train_step_fp16_derived_bound" > gpurun_out/cfg4_r5j_$cap.log 2>&1
  echo "cap $cap rc $?"; grep -E "configs4 fp16|AssertionError|passed|failed" gpurun_out/cfg4_r5j_$cap.log | cut -c1-400 | head -4
done

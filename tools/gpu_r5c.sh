#!/bin/bash
# round 5: resize bit-exactness, the workload-size configs tests (mAP parity, configs[4] fp16 at batch 8),
# then the headline profile (bench + rocprofv3 trace + PMC traffic + SQ counters)
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -v -s --timeout 150 --timeout-method thread "tests/test_gpu_augment.py" \
  > gpurun_out/tests_r5c.log 2>&1 || { grep -E "^E |FAILED|passed|failed" gpurun_out/tests_r5c.log | head -20; exit 1; }
tail -1 gpurun_out/tests_r5c.log
timeout -k 10 900 python -u -m pytest -v -s --timeout 880 --timeout-method thread \
  "tests/test_gpu_configs.py::test_configs1_yolox_s_640_bf16_batch32" \
  "tests/test_gpu_configs.py::test_configs3_yolox_l_640_fp16_batch16" \
  "tests/test_gpu_configs.py::test_configs4_yolox_x_1280_train_step_fp16_derived_bound" \
  > gpurun_out/tests_r5c_cfg.log 2>&1; rc=$?
grep -E "box mAP|configs4 fp16|passed|failed|^E " gpurun_out/tests_r5c_cfg.log | tail -14
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/gpu_profile.sh r5c || exit 1
python tools/forward_timeline.py gpurun_out/prof_r5c/run_kernel_trace.csv > gpurun_out/timeline_r5c.txt 2>&1 || true
tail -3 gpurun_out/timeline_r5c.txt
head -30 gpurun_out/mfma_util_r5c.txt

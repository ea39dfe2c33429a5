#!/bin/bash
# round 5: the API-edge / nano-training / resize / block train-mode tests, then the workload-size configs tests
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread \
  "tests/test_gpu_model.py::test_decode_in_inference_false" \
  "tests/test_gpu_model.py::test_building_blocks_train_mode" \
  "tests/test_gpu_model.py::test_building_blocks_callable_standalone" \
  "tests/test_gpu_model.py::test_cspdarknet_out_features_and_train_mode" \
  "tests/test_gpu_model.py::test_backbone_stages_callable_standalone" \
  "tests/test_gpu_train.py::test_captured_train_step_fp16_gradscaler_matches_eager" \
  "tests/test_gpu_train.py::test_depthwise_gradients" \
  "tests/test_gpu_train.py::test_train_step_other_widths_match_oracle" \
  "tests/test_gpu_augment.py" \
  > gpurun_out/tests_r5b.log 2>&1 || { grep -E "^E |Error|FAILED|passed|failed" gpurun_out/tests_r5b.log | head -40; exit 1; }
tail -3 gpurun_out/tests_r5b.log
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 880 --timeout-method thread \
  "tests/test_gpu_configs.py::test_configs1_yolox_s_640_bf16_batch32" \
  "tests/test_gpu_configs.py::test_configs3_yolox_l_640_fp16_batch16" \
  "tests/test_gpu_configs.py::test_configs4_yolox_x_1280_train_step_fp16_derived_bound" \
  > gpurun_out/tests_r5b_cfg.log 2>&1 || { grep -E "^E |box mAP|FAILED|passed|failed" gpurun_out/tests_r5b_cfg.log | head -30; exit 1; }
grep -E "box mAP|configs4 fp16|passed|failed" gpurun_out/tests_r5b_cfg.log | tail -12

#!/bin/bash
# round 5: API-edge / nano-training / resize / block train-mode / head_pred2 / wide conv_ws tests, A/B of the
# AGPR-pinned weights + head_pred2, the workload-size configs tests, configs[3] bench
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/resize_probe.py > gpurun_out/resize_probe.txt 2>&1 || { tail -5 gpurun_out/resize_probe.txt; exit 1; }
cat gpurun_out/resize_probe.txt
timeout -k 10 500 python -u -m pytest --deselect "tests/test_gpu_augment.py::test_resize_bilinear_bit_exact_vs_aten_on_device" -x -v -s --timeout 300 --timeout-method thread \
  "tests/test_gpu_model.py::test_decode_in_inference_false" \
  "tests/test_gpu_model.py::test_building_blocks_train_mode" \
  "tests/test_gpu_model.py::test_building_blocks_callable_standalone" \
  "tests/test_gpu_model.py::test_cspdarknet_out_features_and_train_mode" \
  "tests/test_gpu_model.py::test_backbone_stages_callable_standalone" \
  "tests/test_gpu_train.py::test_captured_train_step_fp16_gradscaler_matches_eager" \
  "tests/test_gpu_train.py::test_depthwise_gradients" \
  "tests/test_gpu_train.py::test_train_step_other_widths_match_oracle" \
  "tests/test_gpu_augment.py" \
  "tests/test_gpu_ops.py::test_head_pred_fused_level" \
  "tests/test_gpu_ops.py::test_conv_ws_3x3_wide_channels" \
  "tests/test_gpu_ops.py::test_conv_ws_3x3" \
  "tests/test_gpu_train.py::test_dgrad_conv_ws_fp32_tiles" \
  "tests/test_gpu_model.py::test_fp32_forward_matches_reference" \
  "tests/test_gpu_model.py::test_low_precision_forward" \
  > gpurun_out/tests_r5b.log 2>&1 || { grep -E "^E |Error|FAILED|passed|failed" gpurun_out/tests_r5b.log | head -40; exit 1; }
tail -3 gpurun_out/tests_r5b.log
# A/B: AGPR-pinned weights (current) vs not (dbg/libyoloxhip_nopin.so), head_pred2 vs the tile kernel
TESTS= AB="DEFAULT=1 YOLOX_AMD_LIB=dbg/libyoloxhip_nopin.so YXH_HEAD_V1=1 DEFAULT=1 YOLOX_AMD_LIB=dbg/libyoloxhip_nopin.so YXH_HEAD_V1=1" bash tools/gpu_iter.sh r5b || exit 1
timeout -k 10 300 python bench.py --model yolox_l --batch 16 --dtype fp16 --no-cpu-baseline > gpurun_out/bench_r5b_c3.json 2> gpurun_out/bench_r5b_c3.err || { tail -5 gpurun_out/bench_r5b_c3.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_r5b_c3.json')); print('configs3', d['value'], d['roofline']['forward_ms'], d['roofline']['frac'])"
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 880 --timeout-method thread \
  "tests/test_gpu_configs.py::test_configs1_yolox_s_640_bf16_batch32" \
  "tests/test_gpu_configs.py::test_configs3_yolox_l_640_fp16_batch16" \
  "tests/test_gpu_configs.py::test_configs4_yolox_x_1280_train_step_fp16_derived_bound" \
  > gpurun_out/tests_r5b_cfg.log 2>&1 || { grep -E "^E |box mAP|FAILED|passed|failed" gpurun_out/tests_r5b_cfg.log | head -30; exit 1; }
grep -E "box mAP|configs4 fp16|passed|failed" gpurun_out/tests_r5b_cfg.log | tail -12

cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 280 --timeout-method thread \
  "tests/test_gpu_model.py::test_decode_in_inference_false" \
  "tests/test_gpu_train.py::test_captured_train_step_fp16_gradscaler_matches_eager" \
  > gpurun_out/tests_r5a.log 2>&1 || { tail -30 gpurun_out/tests_r5a.log; exit 1; }
tail -3 gpurun_out/tests_r5a.log
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 880 --timeout-method thread \
  "tests/test_gpu_configs.py::test_configs1_yolox_s_640_bf16_batch32" \
  "tests/test_gpu_configs.py::test_configs3_yolox_l_640_fp16_batch16" \
  "tests/test_gpu_configs.py::test_configs4_yolox_x_1280_train_step_fp16_derived_bound" \
  > gpurun_out/tests_r5a_cfg.log 2>&1 || { tail -30 gpurun_out/tests_r5a_cfg.log; exit 1; }
grep -E "box mAP|configs|passed|failed" gpurun_out/tests_r5a_cfg.log | tail -12

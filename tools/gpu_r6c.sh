cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q -s --timeout 600 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_train.py::test_train_step_bf16_autocast_close_to_fp32 tests/test_gpu_configs.py::test_configs1_yolox_s_640_bf16_batch32 \
  tests/test_gpu_configs.py::test_configs3_yolox_l_640_fp16_batch16 tests/test_gpu_model.py tests/test_gpu_processor.py \
  > gpurun_out/tests_r6c.log 2>&1; rc=$?
grep -E "box mAP|vs fp32 oracle|distances|passed|failed" gpurun_out/tests_r6c.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" gpurun_out/tests_r6c.log | head -30; exit $rc; }

cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_model.py -k "twice or train_mode or out_features" tests/test_gpu_postprocess.py tests/test_gpu_processor.py \
  > gpurun_out/tests_r6a.log 2>&1; rc=$?
tail -3 gpurun_out/tests_r6a.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" gpurun_out/tests_r6a.log | head -30; exit $rc; }
bash tools/gpu_round.sh r6a --no-tests

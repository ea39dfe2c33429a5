cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q -s --timeout 600 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_configs.py -k "configs1 or configs3_yolox_l" > gpurun_out/tests_r6b.log 2>&1; rc=$?
grep -E "box mAP|vs fp32 oracle|passed|failed" gpurun_out/tests_r6b.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" gpurun_out/tests_r6b.log | head -30; exit $rc; }

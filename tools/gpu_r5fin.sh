#!/bin/bash
# round 5: the whole GPU test suite on the current tree, then smoke()
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1050 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/gpu_tests_r5fin.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests_r5fin.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" gpurun_out/gpu_tests_r5fin.log | head -30; exit $rc; }
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r5fin.log 2>&1; rc=$?
tail -2 gpurun_out/smoke_r5fin.log
exit $rc

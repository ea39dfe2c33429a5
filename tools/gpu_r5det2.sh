#!/bin/bash
# round 5: training tuner candidates at the benched shapes, each run twice into a zeroed sink (race detector)
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 800 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_configs.py -k "every_training_candidate" > gpurun_out/tests_r5det2.log 2>&1; rc=$?
grep -E "checked|PASS|FAIL|Error|assert" gpurun_out/tests_r5det2.log | head -20
tail -2 gpurun_out/tests_r5det2.log
exit $rc

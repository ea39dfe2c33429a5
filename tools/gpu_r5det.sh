#!/bin/bash
# round 5: every candidate tile at the benched shapes, three runs each, bit-equal (race detector)
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 800 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_configs.py -k "every_candidate_tile" > gpurun_out/tests_r5det.log 2>&1; rc=$?
grep -E "deterministic|PASS|FAIL|Error|assert" gpurun_out/tests_r5det.log | head -20
tail -2 gpurun_out/tests_r5det.log
exit $rc

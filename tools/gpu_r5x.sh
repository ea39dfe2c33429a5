#!/bin/bash
# round 5: conv_ws1 K-split exchange moved past every row buffer -- the conv_ws1 tests (incl. the
# pipelined 20x20 x 32 shapes), then the whole GPU suite, smoke(), the default bench and the profile
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_ops.py -k "conv_ws1" > gpurun_out/tests_r5x_ws1.log 2>&1 || { grep -E "^E |FAILED" gpurun_out/tests_r5x_ws1.log | head; exit 1; }
tail -1 gpurun_out/tests_r5x_ws1.log
sed -i 's/r5w/r5x/g' tools/gpu_r5w.sh
bash tools/gpu_r5w.sh

#!/bin/bash
# round 5 end: whole GPU suite, smoke(), default bench line on the final tree
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1050 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/gpu_tests_r5end.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests_r5end.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" gpurun_out/gpu_tests_r5end.log | head -30; exit $rc; }
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r5end.log 2>&1 || { tail -5 gpurun_out/smoke_r5end.log; exit 1; }
tail -1 gpurun_out/smoke_r5end.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench_r5end.json 2> gpurun_out/bench_r5end.err || { tail -5 gpurun_out/bench_r5end.err; exit 1; }
cat gpurun_out/bench_r5end.json

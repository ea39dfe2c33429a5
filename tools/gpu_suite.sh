# the whole GPU suite + smoke() on the current tree (TAG names the logs)
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r6s}
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/gpu_tests_$T.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests_$T.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" gpurun_out/gpu_tests_$T.log | head -30; exit $rc; }
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$T.log 2>&1 || { tail -5 gpurun_out/smoke_$T.log; exit 1; }
tail -1 gpurun_out/smoke_$T.log

#!/bin/bash
# GPU box, end of a round (or any full check): the whole GPU test suite, smoke(), the default bench
# line, then the headline profile (tools/gpu_profile.sh: trace + stats, timeline, PMC traffic of the
# timed forwards, SQ counters).  Usage: bash tools/gpu_round.sh TAG [--no-tests] [--no-profile]
set -o pipefail
TAG=${1:-round}
shift
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [[ " $* " != *" --no-tests "* ]]; then
  timeout -k 10 1050 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
      > gpurun_out/gpu_tests_$TAG.log 2>&1; rc=$?
  tail -3 gpurun_out/gpu_tests_$TAG.log
  [ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" gpurun_out/gpu_tests_$TAG.log | head -30; exit $rc; }
  timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
      > gpurun_out/smoke_$TAG.log 2>&1 || { tail -5 gpurun_out/smoke_$TAG.log; exit 1; }
  tail -1 gpurun_out/smoke_$TAG.log
fi
timeout -k 10 300 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err \
    || { tail -5 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
if [[ " $* " != *" --no-profile "* ]]; then
  bash tools/gpu_profile.sh $TAG || exit 1
  cat gpurun_out/timeline_$TAG.txt | tail -2
fi

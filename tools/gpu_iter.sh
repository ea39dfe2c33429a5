#!/bin/bash
# GPU box: a focused test selection, then the default bench (+ optional env A/B of the bench).
# Usage: TESTS="tests/x.py -k y" AB="ENV=0 ENV=1" bash tools/gpu_iter.sh TAG
set -o pipefail
TAG=${1:-it}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  eval timeout -k 10 400 python -u -m pytest $TESTS -m gpu -x -q -s --timeout 200 --timeout-method thread \
      > gpurun_out/tests_$TAG.log 2>&1; rc=$?
  tail -4 gpurun_out/tests_$TAG.log
  [ $rc -eq 0 ] || { grep -E "^E |Error" gpurun_out/tests_$TAG.log | head -20; exit $rc; }
fi
i=0
for e in ${AB:-DEFAULT=1}; do
  i=$((i + 1))
  f=gpurun_out/bench_${TAG}_${i}_${e//\//_}
  env $e timeout -k 10 300 python -u bench.py --no-cpu-baseline --layers > $f.json 2> $f.err || { tail -5 $f.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], 'img/s fwd', d['roofline']['forward_ms'], 'ms frac', d['roofline']['frac'])" $f.json $e
done

# round 6: branch-free conv_ws / conv_ws1 epilogues -- op tests, then two bench runs with the per-layer table
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r6d}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_ops.py -k "conv_ws or ws1 or bit_exact or post or chain" > gpurun_out/tests_$T.log 2>&1; rc=$?
tail -2 gpurun_out/tests_$T.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" gpurun_out/tests_$T.log | head -30; exit $rc; }
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --layers > gpurun_out/bench_${T}_$i.json 2> gpurun_out/bench_${T}_$i.err || { tail -5 gpurun_out/bench_${T}_$i.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], 'img/s fwd', d['roofline']['forward_ms'], 'ms frac', d['roofline']['frac'])" gpurun_out/bench_${T}_$i.json
done

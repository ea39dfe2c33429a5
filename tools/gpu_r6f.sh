# round 6: score-record NMS filter, captured DP step, empty-lane capture, twice-called blocks; then
# the bench with / without the score records (alternating)
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r6f}
timeout -k 10 800 python -u -m pytest -x -q -s --timeout 400 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_postprocess.py tests/test_gpu_dp.py::test_captured_dp_step_matches_eager_dp_step \
  tests/test_gpu_model.py -k "scored or captured_dp or lane or twice or postprocess" > gpurun_out/tests_$T.log 2>&1; rc=$?
tail -3 gpurun_out/tests_$T.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" gpurun_out/tests_$T.log | head -30; exit $rc; }
for i in 1 2; do
  for mode in scores rows; do
    extra=""; [ $mode = rows ] && extra="--no-scores"
    timeout -k 10 300 python -u bench.py --no-cpu-baseline $extra > gpurun_out/bench_${T}_${mode}_$i.json 2> gpurun_out/bench_${T}_${mode}_$i.err || { tail -5 gpurun_out/bench_${T}_${mode}_$i.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], 'img/s step', d['ms_per_step'], 'fwd', d['roofline']['forward_ms'], d['config']['nms_filter'])" gpurun_out/bench_${T}_${mode}_$i.json $mode
  done
done

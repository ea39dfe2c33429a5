#!/bin/bash
# round 5: NMS filter 16-byte tile loads, one mask pass for the bench batch, fewer empty mask blocks:
# postprocess tests (bit-exact vs the C oracle, forced multi-pass budgets) + bench
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_postprocess.py tests/test_gpu_model.py -k "postprocess or nms or filter or processor or graph" > gpurun_out/tests_r5n.log 2>&1 || { grep -E "^E |FAILED" gpurun_out/tests_r5n.log | head; exit 1; }
tail -1 gpurun_out/tests_r5n.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_r5n_$i.json 2> gpurun_out/bench_r5n_$i.err || { tail -5 gpurun_out/bench_r5n_$i.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print('bench', d['value'], 'img/s', d['ms_per_step'], 'ms/step fwd', d['roofline']['forward_ms'])" gpurun_out/bench_r5n_$i.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r5n -o run --output-format csv \
    -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof_r5n.log 2>&1 || exit 1
grep -E "pp_" gpurun_out/prof_r5n/run_kernel_stats.csv | cut -d, -f1-5

#!/bin/bash
# round 5: conv_ws1 6-8-buffer tiles (259-260): tests, bench (tuner picks, per-layer table), configs[3]
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_ops.py -k "conv_ws1" > gpurun_out/tests_r5z.log 2>&1 || { grep -E "^E |FAILED" gpurun_out/tests_r5z.log | head; exit 1; }
tail -1 gpurun_out/tests_r5z.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --layers > gpurun_out/bench_r5z_$i.json 2> gpurun_out/bench_r5z_$i.err || { tail -5 gpurun_out/bench_r5z_$i.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print('bench', d['value'], 'img/s', d['ms_per_step'], 'ms/step fwd', d['roofline']['forward_ms'])" gpurun_out/bench_r5z_$i.json
done
grep -E "tile (25[3-9]|260)" gpurun_out/bench_r5z_1.err | head -20
timeout -k 10 300 python -u bench.py --model yolox_l --batch 16 --dtype fp16 --no-cpu-baseline > gpurun_out/bench_r5z_c3.json 2> gpurun_out/bench_r5z_c3.err || { tail -5 gpurun_out/bench_r5z_c3.err; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); print('configs3', d['value'], 'img/s', d['ms_per_step'], 'ms/step fwd', d['roofline']['forward_ms'])" gpurun_out/bench_r5z_c3.json

#!/bin/bash
# round 5: NMS filter with 8 lanes per row / 32 rows per block vs 4 / 64 (ab/libyoloxhip_oldpp.so)
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_postprocess.py > gpurun_out/tests_r5filt.log 2>&1 || { grep -E "^E |FAILED" gpurun_out/tests_r5filt.log | head; exit 1; }
tail -1 gpurun_out/tests_r5filt.log
summ() { python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], 'img/s', d['ms_per_step'], 'ms/step fwd', d['roofline']['forward_ms'])" $1 "$2"; }
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/filt_new_$i.json 2> gpurun_out/filt.err || { tail -5 gpurun_out/filt.err; exit 1; }
  summ gpurun_out/filt_new_$i.json "filter 8x32"
  YOLOX_AMD_LIB=$PWD/ab/libyoloxhip_oldpp.so timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/filt_old_$i.json 2> gpurun_out/filt.err || { tail -5 gpurun_out/filt.err; exit 1; }
  summ gpurun_out/filt_old_$i.json "filter 4x64"
done

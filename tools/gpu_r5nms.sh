#!/bin/bash
# round 5: NMS filter in order behind the forward + the rest on the side stream (yxh_postprocess_split)
# vs the event form -- postprocess GPU tests, then the bench alternating
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_postprocess.py tests/test_native_lib.py > gpurun_out/tests_r5nms.log 2>&1 || { grep -E "^E |FAILED" gpurun_out/tests_r5nms.log | head; exit 1; }
tail -1 gpurun_out/tests_r5nms.log
summ() { python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], 'img/s', d['ms_per_step'], 'ms/step fwd', d['roofline']['forward_ms'], d['config']['nms_streams'])" $1 "$2"; }
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/nms_split_$i.json 2> gpurun_out/nms_ab.err || { tail -5 gpurun_out/nms_ab.err; exit 1; }
  summ gpurun_out/nms_split_$i.json split
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --nms-event > gpurun_out/nms_event_$i.json 2> gpurun_out/nms_ab.err || { tail -5 gpurun_out/nms_ab.err; exit 1; }
  summ gpurun_out/nms_event_$i.json event
done

#!/bin/bash
# round 5: split NMS streams with and without the forward on a high-priority stream
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
summ() { python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], 'img/s', d['ms_per_step'], 'ms/step fwd', d['roofline']['forward_ms'])" $1 "$2"; }
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/prio_off_$i.json 2> gpurun_out/prio.err || { tail -5 gpurun_out/prio.err; exit 1; }
  summ gpurun_out/prio_off_$i.json "split"
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --fwd-priority > gpurun_out/prio_on_$i.json 2> gpurun_out/prio.err || { tail -5 gpurun_out/prio.err; exit 1; }
  summ gpurun_out/prio_on_$i.json "split+fwd-priority"
done

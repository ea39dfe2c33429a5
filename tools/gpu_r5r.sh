#!/bin/bash
# round 5: two output slots with the forward on a high-priority stream vs the default pipeline
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for f in "" "--two-slot --fwd-priority" "" "--two-slot --fwd-priority"; do
  i=$((i + 1))
  timeout -k 10 300 python -u bench.py --no-cpu-baseline $f > gpurun_out/bench_r5r_$i.json 2> gpurun_out/bench_r5r_$i.err || { tail -5 gpurun_out/bench_r5r_$i.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2] or 'default', d['value'], 'img/s', d['ms_per_step'], 'ms/step fwd', d['roofline']['forward_ms'])" gpurun_out/bench_r5r_$i.json "$f"
done

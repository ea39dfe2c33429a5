#!/bin/bash
# GPU box: the per-op autotune alone vs autotune + the in-graph refinement (bench --refine-tiles).
# Both tunings are written to tune files on their first run, then the bench alternates between
# loading one and the other (REPS rounds), so run-to-run autotune noise stays out of the A/B.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-refab}
rm -f gpurun_out/tune_${T}_base.json gpurun_out/tune_${T}_ref.json
timeout -k 10 300 python -u bench.py --no-cpu-baseline --tune-file gpurun_out/tune_${T}_base.json \
    > gpurun_out/bench_${T}_base_0.json 2> gpurun_out/bench_${T}_base_0.err || { tail -5 gpurun_out/bench_${T}_base_0.err; exit 1; }
timeout -k 10 600 python -u bench.py --no-cpu-baseline --refine-tiles --layers --tune-file gpurun_out/tune_${T}_ref.json \
    > gpurun_out/bench_${T}_ref_0.json 2> gpurun_out/bench_${T}_ref_0.err || { tail -5 gpurun_out/bench_${T}_ref_0.err; exit 1; }
grep -a "^refine" gpurun_out/bench_${T}_ref_0.err | tail -60
for i in $(seq 1 ${REPS:-3}); do
  for f in base ref; do
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --tune-file gpurun_out/tune_${T}_$f.json \
        > gpurun_out/bench_${T}_${f}_$i.json 2> gpurun_out/bench_${T}_${f}_$i.err || { tail -5 gpurun_out/bench_${T}_${f}_$i.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], 'img/s fwd', d['roofline']['forward_ms'])" gpurun_out/bench_${T}_${f}_$i.json $f
  done
done

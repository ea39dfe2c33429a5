#!/bin/bash
# GPU box: the default bench under several tune files (tile choices forced per shape), alternating -- a graph-level
# check of tile choices the per-op autotune makes in isolation.  Usage: FILES="a b" DIR=tools/tune_ab TAG=t bash tools/gpu_tune_ab.sh
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-tuneab}
for i in $(seq 1 ${REPS:-2}); do
  for f in $FILES; do
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --tune-file $DIR/$f.json > gpurun_out/bench_${T}_${f}_$i.json 2> gpurun_out/bench_${T}_${f}_$i.err || { tail -5 gpurun_out/bench_${T}_${f}_$i.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], 'img/s fwd', d['roofline']['forward_ms'])" gpurun_out/bench_${T}_${f}_$i.json $f
  done
done

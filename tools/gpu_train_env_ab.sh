#!/bin/bash
# GPU box: one training config under several environment settings, alternating.  Usage:
#   ENVS="YOLOX_AMD_WGRAD_GROUP=1 YOLOX_AMD_WGRAD_GROUP=4" ARGS="--steps 30 --warmup 5" TAG=t bash tools/gpu_train_env_ab.sh
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-envab}
for i in $(seq 1 ${REPS:-2}); do
  for e in $ENVS; do
    f=gpurun_out/train_${T}_${e//\//_}_$i
    env $e timeout -k 10 400 python -u bench.py --workload train --no-cpu-baseline $ARGS > $f.json 2> $f.err || { tail -5 $f.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['frac'], d['config'].get('issue'))" $f.json $e
  done
done

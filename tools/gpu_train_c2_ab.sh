#!/bin/bash
# GPU box: configs[2] (yolox_s fp32 bs 8) training step, eager vs captured (YOLOX_AMD_TRAIN_GRAPH=1), alternating
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-c2ab}
for i in 1 2; do
  for g in 0 1; do
    YOLOX_AMD_TRAIN_GRAPH=$g timeout -k 10 400 python -u bench.py --workload train --steps 30 --warmup 5 --no-cpu-baseline \
        > gpurun_out/train_${T}_g${g}_$i.json 2> gpurun_out/train_${T}_g${g}_$i.err || { tail -5 gpurun_out/train_${T}_g${g}_$i.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print('graph', sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('host_issue_ms_per_step'))" gpurun_out/train_${T}_g${g}_$i.json $g
  done
done

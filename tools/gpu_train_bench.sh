#!/bin/bash
# GPU box: the training configs -- configs[2] (yolox_s fp32 bs 8) eager, configs[4] (yolox_x 1280 --fp16 bs 8)
# eager and captured.  Usage: TAG=t bash tools/gpu_train_bench.sh
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-train}
YOLOX_AMD_TRAIN_GRAPH=0 timeout -k 10 400 python -u bench.py --workload train --steps 30 --warmup 5 > gpurun_out/train_${T}_c2.json 2> gpurun_out/train_${T}_c2.err || { tail -5 gpurun_out/train_${T}_c2.err; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); print('c2', d['value'], d['ms_per_step'], d['roofline']['frac'], d['config']['issue'])" gpurun_out/train_${T}_c2.json
YOLOX_AMD_TRAIN_GRAPH=0 timeout -k 10 500 python -u bench.py --workload train --model yolox_x --size 1280 --dtype fp16 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/train_${T}_c4.json 2> gpurun_out/train_${T}_c4.err || { tail -5 gpurun_out/train_${T}_c4.err; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); print('c4 eager', d['value'], d['ms_per_step'], d['roofline']['frac'], d['host_issue_ms_per_step'])" gpurun_out/train_${T}_c4.json
YOLOX_AMD_TRAIN_GRAPH=1 timeout -k 10 500 python -u bench.py --workload train --model yolox_x --size 1280 --dtype fp16 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/train_${T}_c4g.json 2> gpurun_out/train_${T}_c4g.err || { tail -5 gpurun_out/train_${T}_c4g.err; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); print('c4 captured', d['value'], d['ms_per_step'], d['roofline']['frac'], d['config']['issue'])" gpurun_out/train_${T}_c4g.json

#!/bin/bash
# GPU box: segmented captured training step: parity tests, configs[2] x wgrad fork group, configs[4], rocprof.
set -o pipefail
TAG=${1:-r3g3}
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_train.py \
    -k "captured or batched_weight" -m gpu > gpurun_out/captest_${TAG}.log 2>&1 || { tail -40 gpurun_out/captest_${TAG}.log; exit 1; }
tail -2 gpurun_out/captest_${TAG}.log
B="python bench.py --workload train --no-cpu-baseline"
P='"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"frac": [0-9.]*\|"issue": "[a-zA-Z ]*"\|"host_issue_ms_per_step": [0-9.]*'
for G in 1 4 12; do
  YOLOX_AMD_TRAIN_GRAPH=1 YOLOX_AMD_WGRAD_GROUP=$G timeout -k 10 300 $B --steps 10 --warmup 3 > gpurun_out/train_${TAG}_c2_g$G.json 2> gpurun_out/train_${TAG}_c2_g$G.err || { tail -20 gpurun_out/train_${TAG}_c2_g$G.err; exit 1; }
  grep -o "$P" gpurun_out/train_${TAG}_c2_g$G.json | tr '\n' ' '; echo " configs2 graph, wgrad group $G"
  YOLOX_AMD_TRAIN_GRAPH=1 YOLOX_AMD_WGRAD_GROUP=$G timeout -k 10 300 $B --steps 10 --warmup 3 > gpurun_out/train_${TAG}_c2_e$G.json 2> gpurun_out/train_${TAG}_c2_e$G.err || exit 1
  grep -o "$P" gpurun_out/train_${TAG}_c2_e$G.json | tr '\n' ' '; echo " configs2 eager, wgrad group $G"
done
C4="--model yolox_x --size 1280 --dtype fp16 --batch 8 --steps 6 --warmup 3"
YOLOX_AMD_TRAIN_GRAPH=1 timeout -k 10 400 $B $C4 > gpurun_out/train_${TAG}_c4.json 2> gpurun_out/train_${TAG}_c4.err || { tail -20 gpurun_out/train_${TAG}_c4.err; exit 1; }
grep -o "$P" gpurun_out/train_${TAG}_c4.json | tr '\n' ' '; echo " configs4 graph"
YOLOX_AMD_TRAIN_GRAPH=1 YOLOX_AMD_WGRAD_GROUP=4 timeout -k 10 400 $B $C4 > gpurun_out/train_${TAG}_c4_g4.json 2> gpurun_out/train_${TAG}_c4_g4.err || exit 1
grep -o "$P" gpurun_out/train_${TAG}_c4_g4.json | tr '\n' ' '; echo " configs4 graph group 4"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${TAG} -o c2g -- \
    python $R/bench.py --workload train --no-cpu-baseline --steps 3 --warmup 2 > $R/gpurun_out/prof_${TAG}.log 2>&1 || exit 1
echo prof done

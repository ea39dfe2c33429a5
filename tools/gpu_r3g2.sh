#!/bin/bash
# GPU box: captured training step x weight-gradient side stream (on/off), configs[2] and configs[4].
set -o pipefail
TAG=${1:-r3g2}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
B="python bench.py --workload train --no-cpu-baseline"
P='"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"frac": [0-9.]*\|"issue": "[a-zA-Z ]*"\|"host_issue_ms_per_step": [0-9.]*'
YOLOX_AMD_WGRAD_STREAM=0 timeout -k 10 300 $B --steps 10 --warmup 3 > gpurun_out/train_${TAG}_c2_inl.json 2> gpurun_out/train_${TAG}_c2_inl.err || exit 1
grep -o "$P" gpurun_out/train_${TAG}_c2_inl.json | tr '\n' ' '; echo " configs2 graph, wgrad inline"
C4="--model yolox_x --size 1280 --dtype fp16 --batch 8 --steps 6 --warmup 3"
YOLOX_AMD_TRAIN_GRAPH=0 timeout -k 10 400 $B $C4 > gpurun_out/train_${TAG}_c4_eager.json 2> gpurun_out/train_${TAG}_c4_eager.err || exit 1
grep -o "$P" gpurun_out/train_${TAG}_c4_eager.json | tr '\n' ' '; echo " configs4 eager"
YOLOX_AMD_WGRAD_STREAM=0 timeout -k 10 400 $B $C4 > gpurun_out/train_${TAG}_c4_inl.json 2> gpurun_out/train_${TAG}_c4_inl.err || exit 1
grep -o "$P" gpurun_out/train_${TAG}_c4_inl.json | tr '\n' ' '; echo " configs4 graph, wgrad inline"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_${TAG} -o c2g -- \
    python $GRAFT_REPO_ROOT/bench.py --workload train --no-cpu-baseline --steps 3 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}.log 2>&1 || exit 1
echo prof done
for G in 4 12; do
  YOLOX_AMD_WGRAD_GROUP=$G timeout -k 10 300 $B --steps 10 --warmup 3 > gpurun_out/train_${TAG}_c2_g$G.json 2> gpurun_out/train_${TAG}_c2_g$G.err || exit 1
  grep -o "$P" gpurun_out/train_${TAG}_c2_g$G.json | tr '\n' ' '; echo " configs2 graph, wgrad group $G"
  YOLOX_AMD_TRAIN_GRAPH=0 YOLOX_AMD_WGRAD_GROUP=$G timeout -k 10 300 $B --steps 10 --warmup 3 > gpurun_out/train_${TAG}_c2_e$G.json 2> gpurun_out/train_${TAG}_c2_e$G.err || exit 1
  grep -o "$P" gpurun_out/train_${TAG}_c2_e$G.json | tr '\n' ' '; echo " configs2 eager, wgrad group $G"
done

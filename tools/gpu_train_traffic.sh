#!/bin/bash
# GPU box: HBM traffic per training step (FETCH_SIZE / WRITE_SIZE in separate rocprofv3 --pmc passes,
# MI355X_MICROARCH.md HBM section) of bench.py --workload train, summarised by tools/traffic_train.py.
# Usage: bash tools/gpu_train_traffic.sh TAG MODEL BATCH SIZE DTYPE
set -o pipefail
TAG=$1; MODEL=$2; B=$3; S=$4; DT=$5
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp  # tuning runs in step 0, outside the measured window
mkdir -p gpurun_out
ARGS="--workload train --model $MODEL --batch $B --size $S --dtype $DT --no-cpu-baseline"
for CNT in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $CNT -d gpurun_out/pmc_${TAG}_$CNT -o run --output-format csv \
      -- python bench.py $ARGS --steps 3 --warmup 1 > gpurun_out/pmc_${TAG}_$CNT.log 2>&1 || exit 1
done
python tools/traffic_train.py gpurun_out/pmc_$TAG gpurun_out/traffic_$TAG.json $MODEL $B $S $DT || exit 1
echo "train traffic $TAG done"

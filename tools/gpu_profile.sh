#!/bin/bash
# GPU box: evidence for one bench configuration -- bench (+ per-layer table, tune file), rocprofv3
# kernel trace + stats of the same bench, PMC HBM traffic (FETCH_SIZE / WRITE_SIZE in separate
# passes, MI355X_MICROARCH.md HBM section) and an SQ / GRBM pass for MFMA utilisation per kernel.
# Usage: [TRAFFIC_ARGS='yolox_l 16 640 fp16'] bash tools/gpu_profile.sh TAG [bench args...]
#        (e.g. --model yolox_l --batch 16 --dtype fp16; TRAFFIC_ARGS names the workload in the traffic JSON)
set -o pipefail
TAG=${1:-run}
shift
ARGS="$*"
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TUNE=gpurun_out/tune_$TAG.json
timeout -k 10 300 python bench.py $ARGS --layers --tune-file $TUNE > gpurun_out/bench_$TAG.json \
    2> gpurun_out/bench_$TAG.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv \
    -- python bench.py $ARGS --steps 10 --warmup 3 --no-cpu-baseline --tune-file $TUNE \
    > gpurun_out/prof_$TAG.log 2>&1 || exit 1
for CNT in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $CNT -d gpurun_out/pmc_${TAG}_$CNT -o run --output-format csv \
      -- python bench.py $ARGS --steps 4 --warmup 1 --no-cpu-baseline --tune-file $TUNE \
      > gpurun_out/pmc_${TAG}_$CNT.log 2>&1 || exit 1
done
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE \
    -d gpurun_out/pmc_${TAG}_SQ -o run --output-format csv \
    -- python bench.py $ARGS --steps 4 --warmup 1 --no-cpu-baseline --tune-file $TUNE \
    > gpurun_out/pmc_${TAG}_SQ.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS \
    SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE \
    -d gpurun_out/pmc_${TAG}_SQ2 -o run --output-format csv \
    -- python bench.py $ARGS --steps 4 --warmup 1 --no-cpu-baseline --tune-file $TUNE \
    > gpurun_out/pmc_${TAG}_SQ2.log 2>&1 || exit 1
python tools/forward_timeline.py gpurun_out/prof_$TAG/run_kernel_trace.csv > gpurun_out/timeline_$TAG.txt || exit 1
# HBM bytes of exactly the 4 timed forwards of the PMC passes, launch list reconciled with the trace
python tools/traffic.py gpurun_out/pmc_$TAG gpurun_out/traffic_$TAG.json $TRAFFIC_ARGS --replays 4 \
    --timeline gpurun_out/timeline_$TAG.txt || exit 1
python tools/mfma_util.py gpurun_out/pmc_${TAG}_SQ/run_counter_collection.csv --last 3 \
    --stalls gpurun_out/pmc_${TAG}_SQ2/run_counter_collection.csv --json gpurun_out/mfma_util_$TAG.json \
    > gpurun_out/mfma_util_$TAG.txt || exit 1
echo "profile $TAG done"

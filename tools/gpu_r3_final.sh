#!/bin/bash
# GPU box, end-of-session evidence (round 3): yolox_s bench (+ per-layer table), rocprofv3 kernel
# trace / stats + forward timeline, PMC HBM traffic (separate FETCH_SIZE / WRITE_SIZE passes, one tune
# file for every pass), configs[3] yolox_l fp16 bs16, configs[2] and configs[4] training.
# Usage: bash tools/gpu_r3_final.sh TAG
set -o pipefail
TAG=${1:-r3fin}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TS=gpurun_out/tune_${TAG}_s.json
timeout -k 10 300 python bench.py --layers --tune-file $TS > gpurun_out/bench_${TAG}_s.json 2> gpurun_out/layers_${TAG}_s.txt || exit 1
cat gpurun_out/bench_${TAG}_s.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_s -o run --output-format csv \
    -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --tune-file $TS > gpurun_out/prof_${TAG}_s.log 2>&1 || exit 1
python tools/forward_timeline.py gpurun_out/prof_${TAG}_s/run_kernel_trace.csv > gpurun_out/timeline_${TAG}_s.txt 2>&1
tail -2 gpurun_out/timeline_${TAG}_s.txt
for CNT in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $CNT -d gpurun_out/pmc_${TAG}_s_$CNT -o run --output-format csv \
      -- python bench.py --steps 4 --warmup 1 --no-cpu-baseline --tune-file $TS \
      > gpurun_out/pmc_${TAG}_s_$CNT.log 2>&1 || exit 1
done
echo "pmc done"
LARGS="--model yolox_l --batch 16 --dtype fp16"
timeout -k 10 300 python bench.py $LARGS --no-cpu-baseline --tune-file gpurun_out/tune_${TAG}_l.json \
    > gpurun_out/bench_${TAG}_l.json 2> gpurun_out/bench_${TAG}_l.err || exit 1
grep -o '"value": [0-9.]*\|"forward_ms": [0-9.]*\|"frac": [0-9.]*' gpurun_out/bench_${TAG}_l.json | tr '\n' ' '; echo " configs3"
timeout -k 10 300 python bench.py --workload train --steps 10 --warmup 3 > gpurun_out/train_${TAG}_c2.json 2> gpurun_out/train_${TAG}_c2.err || exit 1
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"frac": [0-9.]*' gpurun_out/train_${TAG}_c2.json | tr '\n' ' '; echo " configs2"
timeout -k 10 400 python bench.py --workload train --model yolox_x --size 1280 --dtype fp16 --batch 8 --steps 6 --warmup 3 \
    --no-cpu-baseline > gpurun_out/train_${TAG}_c4.json 2> gpurun_out/train_${TAG}_c4.err || exit 1
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"frac": [0-9.]*' gpurun_out/train_${TAG}_c4.json | tr '\n' ' '; echo " configs4"
echo "final evidence done"

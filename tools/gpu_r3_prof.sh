#!/bin/bash
# GPU box, round 3 evidence: quick tests of new kernels, yolox_s bench (+ per-layer table),
# rocprofv3 kernel trace / stats, PMC HBM traffic; then configs[3] (yolox_l fp16 bs16):
# bench, kernel trace, PMC traffic and an SQ/GRBM pass for MFMA utilisation per kernel.
# Usage: bash tools/gpu_r3_prof.sh TAG
set -o pipefail
TAG=${1:-r3c}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -k "stem" -x -q \
    --timeout 120 --timeout-method thread > gpurun_out/quick_tests_$TAG.log 2>&1 || exit 1
TS=gpurun_out/tune_${TAG}_s.json
timeout -k 10 300 python bench.py --layers --tune-file $TS > gpurun_out/bench_${TAG}_s.json 2> gpurun_out/bench_${TAG}_s.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_s -o run --output-format csv \
    -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --tune-file $TS > gpurun_out/prof_${TAG}_s.log 2>&1 || exit 1
bash tools/pmc_traffic.sh ${TAG}_s $TS || exit 1
TL=gpurun_out/tune_${TAG}_l.json
LARGS="--model yolox_l --batch 16 --dtype fp16"
timeout -k 10 300 python bench.py $LARGS --no-cpu-baseline --tune-file $TL > gpurun_out/bench_${TAG}_l.json 2> gpurun_out/bench_${TAG}_l.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_l -o run --output-format csv \
    -- python bench.py $LARGS --steps 6 --warmup 2 --no-cpu-baseline --tune-file $TL > gpurun_out/prof_${TAG}_l.log 2>&1 || exit 1
for CNT in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $CNT -d gpurun_out/pmc_${TAG}_l_$CNT -o run --output-format csv \
      -- python bench.py $LARGS --steps 4 --warmup 1 --no-cpu-baseline --tune-file $TL \
      > gpurun_out/pmc_${TAG}_l_$CNT.log 2>&1 || exit 1
done
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE \
    -d gpurun_out/pmc_${TAG}_l_SQ -o run --output-format csv \
    -- python bench.py $LARGS --steps 4 --warmup 1 --no-cpu-baseline --tune-file $TL \
    > gpurun_out/pmc_${TAG}_l_SQ.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE \
    -d gpurun_out/pmc_${TAG}_s_SQ -o run --output-format csv \
    -- python bench.py --steps 4 --warmup 1 --no-cpu-baseline --tune-file $TS \
    > gpurun_out/pmc_${TAG}_s_SQ.log 2>&1 || exit 1
echo "prof done"

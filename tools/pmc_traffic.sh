#!/bin/bash
# HBM traffic of one forward (bench workload) from rocprofv3 PMC counters, one
# counter group per pass (MI355X_MICROARCH.md HBM section: FETCH_SIZE x2 on gfx950).
# Usage (GPU box, repo root): bash tools/pmc_traffic.sh TAG TUNE_FILE
set -o pipefail
TAG=${1:-run}
TUNE=${2:-profiles/r01/tune_yolox_s_bs32_bf16.json}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for CNT in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $CNT -d gpurun_out/pmc_${TAG}_$CNT -o run --output-format csv \
      -- python bench.py --steps 4 --warmup 1 --no-cpu-baseline --tune-file $TUNE \
      > gpurun_out/pmc_${TAG}_$CNT.log 2>&1 || exit 1
done
echo "pmc done"

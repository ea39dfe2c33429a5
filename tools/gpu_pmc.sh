#!/bin/bash
# GPU box: SQ stall / instruction-mix counters for one 1x1 conv (tools/pw_pmc.py), one
# counter group per pass.  Usage: bash tools/gpu_pmc.sh TAG
set -o pipefail
TAG=${1:-run}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU"
P3="TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum"
i=0
for CNT in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $CNT -d gpurun_out/pwpmc_${TAG}_$i -o run --output-format csv \
      -- python tools/pw_pmc.py 12 > gpurun_out/pwpmc_${TAG}_$i.log 2>&1 || exit 1
done
echo "pmc done"

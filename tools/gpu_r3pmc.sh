#!/bin/bash
# GPU box: SQ counters for 3x3 conv shapes (tools/r3_pmc.py), one counter group per pass.
# Usage: bash tools/gpu_r3pmc.sh TAG "S H CIN COUT TILE" ["S H CIN COUT TILE" ...]
set -o pipefail
TAG=${1:-run}
shift
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU"
P3="SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL"
j=0
for SHAPE in "$@"; do
  j=$((j+1))
  i=0
  for CNT in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    timeout -s KILL 60 rocprofv3 --pmc $CNT -d gpurun_out/r3pmc_${TAG}_${j}_$i -o run --output-format csv \
        -- python tools/r3_pmc.py $SHAPE > gpurun_out/r3pmc_${TAG}_${j}_$i.log 2>&1 || exit 1
  done
done
echo "pmc done"

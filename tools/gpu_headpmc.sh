#!/bin/bash
# GPU box: time + SQ counters of yxh_head_pred at yolox_s level 0 (tools/head_pmc.py).
set -o pipefail
TAG=${1:-run}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python tools/head_pmc.py > gpurun_out/headpmc_${TAG}_time.txt 2>&1 || exit 1
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU"
i=0
for CNT in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $CNT -d gpurun_out/headpmc_${TAG}_$i -o run --output-format csv \
      -- python tools/head_pmc.py > gpurun_out/headpmc_${TAG}_$i.log 2>&1 || exit 1
done
echo "pmc done"

#!/bin/bash
# GPU box: where a conv_ws tile's time goes -- HIP-event timing of the given tiles with the
# shipped library and the probe builds of tools/ws_split.sh (p1 no epilogue stores, p2 no halo
# DMA after the first tile, p3 both), then two SQ counter passes over one shape.
# Usage: bash tools/gpu_ws_probe.sh TAG "S H CIN COUT TILE" tile-codes...
set -o pipefail
TAG=$1
PMC_SHAPE=$2
shift 2
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=gpurun_out/wsprobe_$TAG.txt
: > $OUT
for P in shipped p1 p2 p3; do
  if [ $P = shipped ]; then LIBV=""; else LIBV="$PWD/dbg/libws_$P.so"; fi
  echo "== $P" >> $OUT
  env ${LIBV:+YOLOX_AMD_LIB=$LIBV} timeout -k 10 240 python -u tools/ws_probe.py "$@" >> $OUT 2>&1 || exit 1
done
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA \
    SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS -d gpurun_out/wspmc_${TAG}_a -o run --output-format csv \
    -- python tools/r3_pmc.py $PMC_SHAPE > gpurun_out/wspmc_${TAG}_a.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE \
    -d gpurun_out/wspmc_${TAG}_b -o run --output-format csv \
    -- python tools/r3_pmc.py $PMC_SHAPE > gpurun_out/wspmc_${TAG}_b.log 2>&1 || exit 1
python tools/pmc_sum.py conv_ws gpurun_out/wspmc_${TAG}_a gpurun_out/wspmc_${TAG}_b >> $OUT
echo "ws probe $TAG done"

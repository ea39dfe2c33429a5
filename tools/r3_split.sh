#!/bin/bash
# Build two probe copies of the library (CPU side): conv_r3 without MFMA (dbg/lib_p1.so)
# and without DMA (dbg/lib_p2.so), for tools/r3_probe.py via YOLOX_AMD_LIB.
set -e
cd "$(dirname "$0")/../pixeltable-yolox_amd"
mkdir -p ../dbg
FLAGS="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -I../include -Icsrc -mcode-object-version=5"
OBJS=$(ls build/*.o | grep -v conv_r3)
for P in 1 2; do
  /opt/rocm/bin/hipcc $FLAGS -DYXH_R3_PROBE=$P -c csrc/conv_r3.hip -o ../dbg/conv_r3_p$P.o &
done
wait
for P in 1 2; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../dbg/lib_p$P.so $OBJS ../dbg/conv_r3_p$P.o
done

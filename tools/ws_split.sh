#!/bin/bash
# Build probe copies of the library (CPU side): conv_ws without epilogue stores
# (dbg/libws_p1.so), without the in-loop halo DMA (p2), without both (p3); for
# tools/ws_probe.py via YOLOX_AMD_LIB.
set -e
cd "$(dirname "$0")/../pixeltable-yolox_amd"
mkdir -p ../dbg
FLAGS="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -I../include -Icsrc -mcode-object-version=5"
OBJS=$(ls build/*.o | grep -v "conv_ws.hip.o")
for P in 1 2 3; do
  /opt/rocm/bin/hipcc $FLAGS -DYXH_WS_PROBE=$P -c csrc/conv_ws.hip -o ../dbg/conv_ws_p$P.o &
done
wait
for P in 1 2 3; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../dbg/libws_p$P.so $OBJS ../dbg/conv_ws_p$P.o
done

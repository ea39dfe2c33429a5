#!/bin/bash
# GPU box: A/B of conv_ws builds (dbg/lib_<v>.so, linked on the CPU side): HIP-event timing of the plain
# conv_ws tiles on the given shapes per build, then the default bench alternating over the builds.
# Usage: VARIANTS="base x" WS_SHAPES="1,80,128,128" TAG=t bash tools/gpu_ws_ab.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-wsab}
OUT=gpurun_out/wsab_$T.txt
: > $OUT
for v in $VARIANTS; do
  echo "== $v" >> $OUT
  YOLOX_AMD_LIB=$PWD/dbg/lib_$v.so timeout -k 10 200 python -u tools/ws_probe.py $WS_TILES >> $OUT 2>&1 || { tail -5 $OUT; exit 1; }
done
cat $OUT
for i in $(seq 1 ${REPS:-2}); do
  for v in $VARIANTS; do
    YOLOX_AMD_LIB=$PWD/dbg/lib_$v.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --layers > gpurun_out/bench_${T}_${v}_$i.json 2> gpurun_out/bench_${T}_${v}_$i.err || { tail -5 gpurun_out/bench_${T}_${v}_$i.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], 'img/s fwd', d['roofline']['forward_ms'])" gpurun_out/bench_${T}_${v}_$i.json $v
  done
done

#!/bin/bash
# round 5 A/B: conv_ws / conv_ws1 epilogue SiLU as scalar fp32 ops (ab/libyoloxhip_silus.so, built with
# -DYXH_SILU4_SCALAR -fno-slp-vectorize) vs the packed-fp32 silu4, yolox_s bench alternating
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
summ() { python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], 'img/s fwd', d['roofline']['forward_ms'])" $1 "$2"; }
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/ab_silu_pk_$i.json 2> gpurun_out/ab_silu.err || { tail -5 gpurun_out/ab_silu.err; exit 1; }
  summ gpurun_out/ab_silu_pk_$i.json "packed"
  YOLOX_AMD_LIB=$PWD/ab/libyoloxhip_silus.so timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/ab_silu_sc_$i.json 2> gpurun_out/ab_silu.err || { tail -5 gpurun_out/ab_silu.err; exit 1; }
  summ gpurun_out/ab_silu_sc_$i.json "scalar"
done

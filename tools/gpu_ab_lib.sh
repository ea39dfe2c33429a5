# A/B of two libyoloxhip builds on one box: the in-tree library vs $ALT (YOLOX_AMD_LIB), alternating,
# the default bench with the per-layer table.  Usage: ALT=dbg/libyoloxhip_x.so TAG=t bash tools/gpu_ab_lib.sh
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-ab}
for i in 1 2; do
  for v in base alt; do
    if [ $v = alt ]; then export YOLOX_AMD_LIB=$PWD/$ALT; else unset YOLOX_AMD_LIB; fi
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --layers > gpurun_out/bench_${T}_${v}_$i.json 2> gpurun_out/bench_${T}_${v}_$i.err || { tail -5 gpurun_out/bench_${T}_${v}_$i.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], 'img/s fwd', d['roofline']['forward_ms'])" gpurun_out/bench_${T}_${v}_$i.json $v
  done
done
unset YOLOX_AMD_LIB

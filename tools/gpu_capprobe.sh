#!/bin/bash
# GPU box: tools/cap_probe.py in both modes (inline weight gradients, then the side stream), then one bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
TAG=${1:-r4a}
for m in ${MODES:-snap noopt}; do
  YOLOX_AMD_WGRAD_STREAM=0 timeout -k 10 150 python -u tools/cap_probe.py $m > gpurun_out/capprobe_${TAG}_$m.log 2>&1
  rc=$?; grep -v Warning gpurun_out/capprobe_${TAG}_$m.log | grep "replay\|eager\|captured\|Error" ; echo "$m rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
[ -n "$NOBENCH" ] && exit 0
timeout -k 10 200 python -u bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err; rc=$?
tail -c 600 gpurun_out/bench_${TAG}.json; exit $rc

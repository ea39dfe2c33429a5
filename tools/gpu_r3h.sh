#!/bin/bash
# GPU box: head-lane scheduling A/B on the bench (one tune file): graph lanes (default), per-level
# streams forked at each level's neck op, and streams with the level-0 head's grids capped to a CU share.
set -o pipefail
TAG=${1:-r3h}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TS=gpurun_out/tune_$TAG.json
timeout -k 10 300 python bench.py --no-cpu-baseline --tune-file $TS > gpurun_out/bench_${TAG}_lanes.json 2>&1 || exit 1
grep -o '"value": [0-9.]*\|"forward_ms": [0-9.]*' gpurun_out/bench_${TAG}_lanes.json | tr '\n' ' '; echo " lanes"
for CFG in "streams:" "streams:1:128" "streams:1:160" "streams:1:96" "lanes:1:128" "streams:1:128,2:64"; do
  G=${CFG%%:*}; C=${CFG#*:}
  YOLOX_AMD_GRAPH=$G YOLOX_AMD_LANE_CUS=$C timeout -k 10 300 python bench.py --no-cpu-baseline --tune-file $TS \
      > gpurun_out/bench_${TAG}_${G}_${C}.json 2>&1 || exit 1
  grep -o '"value": [0-9.]*\|"forward_ms": [0-9.]*' gpurun_out/bench_${TAG}_${G}_${C}.json | tr '\n' ' '; echo " $G cus=$C"
done
# cold-cache autotune (weights evicted from the XCD L2s before every timed candidate launch)
TC=gpurun_out/tune_${TAG}_cold.json
YOLOX_AMD_TUNE_COLD=1 timeout -k 10 400 python bench.py --no-cpu-baseline --tune-file $TC \
    > gpurun_out/bench_${TAG}_cold.json 2>&1 || exit 1
grep -o '"value": [0-9.]*\|"forward_ms": [0-9.]*' gpurun_out/bench_${TAG}_cold.json | tr '\n' ' '; echo " lanes cold-tuned"

#!/bin/bash
# round 5: head lanes hoisted next to their inputs (engine.hoist_lanes) -- graph tests, bench A/B
# against the neck-first capture order (YOLOX_AMD_LANE_HOIST=0), kernel trace + timeline
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TESTS="tests/test_gpu_model.py -k 'graph or chunk or lanes or uint8'" \
AB="YOLOX_AMD_LANE_HOIST=0 DEFAULT=1 YOLOX_AMD_LANE_HOIST=0 DEFAULT=1" bash tools/gpu_iter.sh r5d || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r5d -o run --output-format csv \
    -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof_r5d.log 2>&1 || exit 1
python tools/forward_timeline.py gpurun_out/prof_r5d/run_kernel_trace.csv > gpurun_out/timeline_r5d.txt 2>&1 || true
tail -30 gpurun_out/timeline_r5d.txt

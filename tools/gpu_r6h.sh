# round 6: kernel trace of the serving step (score-record filter) -> the step beyond the forward
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r6h}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$T -o run --output-format csv \
    -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof_$T.log 2>&1 || { tail -5 gpurun_out/prof_$T.log; exit 1; }
python tools/serving_gap.py gpurun_out/prof_$T/run_kernel_trace.csv 4 | tee gpurun_out/serving_gap_$T.txt
python tools/forward_timeline.py gpurun_out/prof_$T/run_kernel_trace.csv > gpurun_out/timeline_$T.txt && tail -1 gpurun_out/timeline_$T.txt

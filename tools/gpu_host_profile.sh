#!/bin/bash
# GPU box: cProfile of the eager training step's host issue path (configs[2] by default), top functions by
# own time and by cumulative time.  Usage: TAG=t [ARGS="..."] bash tools/gpu_host_profile.sh
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-hostprof}
YOLOX_AMD_TRAIN_GRAPH=0 BENCH_HOST_PROFILE=gpurun_out/host_$T.pstats timeout -k 10 400 python -u bench.py --workload train --steps 10 --warmup 5 \
    --no-cpu-baseline $ARGS > gpurun_out/host_$T.json 2> gpurun_out/host_$T.err || { tail -5 gpurun_out/host_$T.err; exit 1; }
python -c "
import pstats, sys
s = pstats.Stats(sys.argv[1])
s.sort_stats('tottime').print_stats(45)
s.sort_stats('cumulative').print_stats(45)
" gpurun_out/host_$T.pstats > gpurun_out/host_$T.txt 2>&1
head -70 gpurun_out/host_$T.txt

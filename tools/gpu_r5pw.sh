#!/bin/bash
# round 5: 1x1 time vs pixel count (fixed cost vs per-pixel cost) for the 256- and 512-channel tiles
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
PW_SHAPES="3200,256,256;6400,256,256;12800,256,256;25600,256,256;51200,256,256;102400,256,256;204800,256,256" \
  timeout -k 10 300 python -u tools/pw_probe.py 486 410 506 194 > gpurun_out/pw_sweep_256.txt 2>&1 || { tail -5 gpurun_out/pw_sweep_256.txt; exit 1; }
cat gpurun_out/pw_sweep_256.txt
PW_SHAPES="1600,512,512;3200,512,512;6400,512,512;12800,512,512;25600,512,512;51200,512,512" \
  timeout -k 10 300 python -u tools/pw_probe.py 510 414 492 198 > gpurun_out/pw_sweep_512.txt 2>&1 || { tail -5 gpurun_out/pw_sweep_512.txt; exit 1; }
cat gpurun_out/pw_sweep_512.txt

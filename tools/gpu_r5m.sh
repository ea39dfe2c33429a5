#!/bin/bash
# round 5: configs[3] (yolox_l 640 fp16 bs16) evidence: bench, kernel trace, PMC traffic, SQ counters, timeline
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for f in "" "--fwd-priority" "" "--fwd-priority"; do
  i=$((i + 1))
  timeout -k 10 300 python -u bench.py --no-cpu-baseline $f > gpurun_out/bench_r5m_$i.json 2> gpurun_out/bench_r5m_$i.err || { tail -5 gpurun_out/bench_r5m_$i.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2] or 'default', d['value'], 'img/s', d['ms_per_step'], 'ms/step fwd', d['roofline']['forward_ms'])" gpurun_out/bench_r5m_$i.json "$f"
done
bash tools/gpu_profile.sh r5m_c3 --model yolox_l --batch 16 --dtype fp16 || exit 1
python tools/forward_timeline.py gpurun_out/prof_r5m_c3/run_kernel_trace.csv > gpurun_out/timeline_r5m_c3.txt 2>&1 || true
tail -2 gpurun_out/timeline_r5m_c3.txt
python -c "import json; d=json.load(open('gpurun_out/bench_r5m_c3.json')); print('configs3', d['value'], d['ms_per_step'], d['roofline']['forward_ms'], d['roofline']['frac'])"
head -24 gpurun_out/mfma_util_r5m_c3.txt

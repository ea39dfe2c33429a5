#!/bin/bash
# GPU box: configs[3] A/B of the 20-wide stride-2 conv_r3h tile (r3 id 39 = tile 151) against the previous choices
# for the same shapes (130 for 512->1024, 139 for 512->512), everything else from one tune file: the first run
# tunes and writes it, the second file differs only in those two shapes.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-c3t}
B="--no-cpu-baseline --model yolox_l --batch 16 --dtype fp16"
rm -f gpurun_out/tune_${T}_new.json
timeout -k 10 400 python -u bench.py $B --tune-file gpurun_out/tune_${T}_new.json > gpurun_out/bench_${T}_new_0.json \
    2> gpurun_out/bench_${T}_new_0.err || { tail -5 gpurun_out/bench_${T}_new_0.err; exit 1; }
python - "$T" <<'PY' || exit 1
import json, sys
t = sys.argv[1]
d = json.load(open(f"gpurun_out/tune_{t}_new.json"))
out, n = [], 0
for k, v in d:
    # key: dtype, batch, in_h, in_w, out_h, out_w, cin, cout, kh, stride, ...
    if k[4] == 20 and k[6] == 512 and k[8] == 3 and k[9] == 2:
        v = 2 * 130 if k[7] == 1024 else 2 * 139
        n += 1
    out.append([k, v])
json.dump(out, open(f"gpurun_out/tune_{t}_old.json", "w"))
print("shapes changed", n)
PY
for i in $(seq 1 ${REPS:-3}); do
  for v in old new; do
    timeout -k 10 400 python -u bench.py $B --tune-file gpurun_out/tune_${T}_$v.json > gpurun_out/bench_${T}_${v}_$i.json \
        2> gpurun_out/bench_${T}_${v}_$i.err || { tail -5 gpurun_out/bench_${T}_${v}_$i.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], 'img/s fwd', d['roofline']['forward_ms'], 'frac', d['roofline']['frac'])" gpurun_out/bench_${T}_${v}_$i.json $v
  done
done

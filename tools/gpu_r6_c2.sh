cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r6c2}
for i in 1 2; do
  timeout -k 10 400 python -u bench.py --workload train --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/train_${T}_$i.json 2> gpurun_out/train_${T}_$i.err || { tail -5 gpurun_out/train_${T}_$i.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print('c2', d['value'], d['ms_per_step'], d['roofline']['frac'], 'host', d['host_issue_ms_per_step'])" gpurun_out/train_${T}_$i.json
done

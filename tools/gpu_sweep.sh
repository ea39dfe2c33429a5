#!/bin/bash
# Inference bench sweep: each argument is one quoted set of extra bench.py flags.
# Usage: bash tools/gpu_sweep.sh TAG "" "--chunk 16 --concurrent" ...
set -o pipefail
TAG=$1; shift
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/sweep_$TAG.jsonl
: > $out
for flags in "$@"; do
    timeout -k 10 200 python -u bench.py --no-cpu-baseline $flags --tune-file gpurun_out/tune_$TAG.json \
        >> $out 2>> gpurun_out/sweep_$TAG.err || exit $?
    python -c "import json,sys; d=json.loads(open('$out').read().splitlines()[-1]); print('$flags', d['value'], d['roofline']['forward_ms'])"
done
echo done

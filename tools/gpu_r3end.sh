#!/bin/bash
# GPU box (round-3 end): the whole GPU suite + smoke, then the head-lane / cold-tune inference A/B.
set -o pipefail
TAG=${1:-r3end}
cd "${GRAFT_REPO_ROOT:-.}"
bash tools/gpu_r3_tests.sh $TAG || exit 1
bash tools/gpu_r3h.sh ${TAG}h

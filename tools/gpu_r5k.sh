#!/bin/bash
# round 5: configs[4] fp16 step parity with the oracle's SimOTA routed from the device; the training stem's
# conv_ws tile (289); configs[4] captured bench
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q --timeout 250 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_ops.py -k "conv_ws_3x3_wide" > gpurun_out/tests_r5k_ops.log 2>&1 || { grep -E "^E |FAILED" gpurun_out/tests_r5k_ops.log | head; exit 1; }
tail -1 gpurun_out/tests_r5k_ops.log
timeout -k 10 400 python -u -m pytest -q -s --timeout 380 --timeout-method thread -p no:cacheprovider \
    "tests/test_gpu_configs.py::test_configs4_yolox_x_1280_train_step_fp16_derived_bound" > gpurun_out/cfg4_r5k.log 2>&1
rc=$?; grep -E "configs4 fp16|^E |passed|failed" gpurun_out/cfg4_r5k.log | cut -c1-2500 | head -6; [ $rc -eq 0 ] || exit $rc
C4="--workload train --model yolox_x --size 1280 --dtype fp16 --batch 8 --no-cpu-baseline"
YOLOX_AMD_TRAIN_GRAPH=1 timeout -k 10 600 python -u bench.py $C4 --steps 6 --warmup 3 > gpurun_out/train_r5k_c4_graph.json 2> gpurun_out/train_r5k_c4_graph.err || { tail -5 gpurun_out/train_r5k_c4_graph.err; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], 'img/s', d['ms_per_step'], 'ms/step frac', d['roofline']['frac'])" gpurun_out/train_r5k_c4_graph.json

#!/bin/bash
# GBDT histograms: bit-identity tests, config-5 shard at 100 trees
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gbdt_gpu.py tests/test_gpu_multirank.py tests/test_forest_gpu.py -k "gbdt or cfg5 or multirank or crossfit" > gpurun_out/gbdt_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gbdt_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/gbdt_tests.log | head; exit $rc; }
( while true; do sleep 50; date >> gpurun_out/cfg5_heartbeat.log; done ) &
HB=$!
timeout -k 10 700 python tools/cfg5.py --rows 100000000 --cols 2000 --trees 100 --shard 0/8 > gpurun_out/cfg5_100.log 2>&1
rc=$?; kill $HB; tail -1 gpurun_out/cfg5_100.log | cut -c1-500; exit $rc

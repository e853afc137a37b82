#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_forest_gpu.py -x -q --timeout 200 --timeout-method thread -k "level" > gpurun_out/lv_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/lv_tests.log; exit 1; }
tail -2 gpurun_out/lv_tests.log
ENGINES=level ATE_FOREST_LV_PROF=1 timeout -k 10 300 python -u tools/forest_level_probe.py > gpurun_out/lv_probe.log 2>&1 || { echo run failed; tail -20 gpurun_out/lv_probe.log; exit 1; }
cut -c1-900 gpurun_out/lv_probe.log
timeout -k 10 300 python -u tools/bench_configs.py --configs 3 --panel3 --n3 10000000 --p3 500 --shard3 0/8 --trees3 100 --serial3 > gpurun_out/cfg3_serial.log 2>&1 || { echo cfg3 failed; tail -20 gpurun_out/cfg3_serial.log; exit 1; }
tail -1 gpurun_out/cfg3_serial.log

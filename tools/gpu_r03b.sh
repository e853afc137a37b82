#!/bin/bash
# round 3b: level forest engine bit identity + config-3 per-GPU shard timing
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_forest_gpu.py -x -v --timeout 200 --timeout-method thread -k "level" > gpurun_out/r03b_tests.log 2>&1 || { echo "tests failed"; tail -60 gpurun_out/r03b_tests.log; exit 1; }
tail -3 gpurun_out/r03b_tests.log
timeout -k 10 600 python tools/bench_configs.py --configs 3 --panel3 --n3 10000000 --p3 500 --shard3 0/8 --trees3 100 > gpurun_out/r03b_cfg3.log 2>&1 || { echo cfg3 failed; tail -20 gpurun_out/r03b_cfg3.log; exit 1; }
tail -2 gpurun_out/r03b_cfg3.log
echo done

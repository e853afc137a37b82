#!/bin/bash
# round 3a: captured RCCL collectives, GBDT stepper/dist, graph estimators, bench, cfg5 shard
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_segmented.py tests/test_gbdt_gpu.py tests/test_gpu_multirank.py -x -v --timeout 240 --timeout-method thread > gpurun_out/r03a_tests.log 2>&1 || { echo "tests failed"; tail -60 gpurun_out/r03a_tests.log; exit 1; }
tail -3 gpurun_out/r03a_tests.log
timeout -k 10 300 python bench.py > gpurun_out/r03a_bench.log 2>&1 || { echo bench failed; tail -20 gpurun_out/r03a_bench.log; exit 1; }
tail -1 gpurun_out/r03a_bench.log
timeout -k 10 600 python tools/cfg5.py --rows 100000000 --cols 2000 --trees 100 --shard 0/8 > gpurun_out/r03a_cfg5.log 2>&1 || { echo cfg5 failed; tail -20 gpurun_out/r03a_cfg5.log; exit 1; }
tail -1 gpurun_out/r03a_cfg5.log
echo done

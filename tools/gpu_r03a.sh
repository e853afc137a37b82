#!/bin/bash
# round 3a: captured RCCL collectives (segmented + dist estimators), graph estimators, bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_segmented.py tests/test_gpu_graph_estimators.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r03a_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r03a_tests.log; exit 1; }
tail -3 gpurun_out/r03a_tests.log
timeout -k 10 300 python bench.py > gpurun_out/r03a_bench.log 2>&1 || { echo bench failed; tail -20 gpurun_out/r03a_bench.log; exit 1; }
tail -1 gpurun_out/r03a_bench.log
echo done

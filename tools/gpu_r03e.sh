#!/bin/bash
# exact-split forest engine on the GPU + the forest suite (predict refactor)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_forest_gpu.py -k exact > gpurun_out/exact_forest.log 2>&1
rc=$?; tail -8 gpurun_out/exact_forest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_forest_gpu.py > gpurun_out/forest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/forest_gpu.log; exit $rc

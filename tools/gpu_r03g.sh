#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_forest_gpu.py -k exact > gpurun_out/exact_forest.log 2>&1
rc=$?; tail -3 gpurun_out/exact_forest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/exact_forest_prof.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/exact_forest_prof.log
timeout -k 10 300 python -u tools/exact_forest_probe.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/exact_forest_probe.log
TREES=3 timeout -k 10 900 bash tools/gbdt_modes.sh 2>&1 | tee gpurun_out/gbdt_modes.log

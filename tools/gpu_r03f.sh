#!/bin/bash
# forest estimators (exact-split default at tutorial scale) on the GPU: graphs, determinism,
# segmented/RCCL capture, plus timing of aipw_rf / double_ml exact vs binned
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_forest_gpu.py tests/test_gpu_graph_estimators.py tests/test_gpu_determinism.py \
  tests/test_gpu_segmented.py > gpurun_out/est_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/est_gpu.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/est_gpu.log | head -20; exit $rc; }
timeout -k 10 300 python -u tools/exact_rf_timing.py 2>&1 | tee gpurun_out/exact_rf_timing.log

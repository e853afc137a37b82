#!/bin/bash
# GBDT H-atomic ablation, tutorial table pattern test, replicate timing
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_tutorial_table.py > gpurun_out/table_test.log 2>&1
rc=$?; tail -3 gpurun_out/table_test.log; [ $rc -eq 0 ] || { grep -E "assert|Error" gpurun_out/table_test.log | head; }
timeout -k 10 300 python -u tools/replicate_timing.py --passes 2 > gpurun_out/replicate_timing.jsonl 2>&1; tail -3 gpurun_out/replicate_timing.jsonl | cut -c1-300
MODES="0 8 16" TREES=3 timeout -k 10 600 bash tools/gbdt_modes.sh

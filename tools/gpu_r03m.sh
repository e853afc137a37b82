#!/bin/bash
# lookback-free scans in the forest level engine / AIPW cross-fit: scan + forest GPU tests,
# then the config-3 per-GPU shard at forest concurrency 5 (twice) and 3
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_scan.py tests/test_forest_gpu.py > gpurun_out/scan_forest_tests.log 2>&1
rc=$?; tail -3 gpurun_out/scan_forest_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/scan_forest_tests.log | head; exit $rc; }
for C in 5 5 3; do
  ATE_CF_CONCURRENT=$C timeout -k 10 240 python -u tools/bench_configs.py --configs 3 --panel3 --n3 10000000 --p3 500 --shard3 0/8 --trees3 100 > gpurun_out/cfg3s_c$C.log 2>&1 || { echo "cfg3 c$C failed"; tail -5 gpurun_out/cfg3s_c$C.log; exit 1; }
  echo "concurrent $C: $(tail -1 gpurun_out/cfg3s_c$C.log | grep -o '"seconds": [0-9.]*\|"ate": [0-9.]*' | tr '\n' ' ')"
done

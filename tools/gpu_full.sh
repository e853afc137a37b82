#!/bin/bash
# full GPU test suite + smoke + 1-GPU bench (round-end rehearsal)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_full.log 2>&1
rc=$?; tail -5 gpurun_out/gpu_tests_full.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/gpu_tests_full.log | head; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1
rc=$?; tail -2 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err
rc=$?; tail -1 gpurun_out/bench_full.json | cut -c1-600; exit $rc

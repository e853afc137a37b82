#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_graph_estimators.py tests/test_gpu_glm.py tests/test_forest_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03c_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r03c_tests.log; exit 1; }
tail -2 gpurun_out/r03c_tests.log
for mode in eager graph; do REPS=6 timeout -k 10 120 python -u tools/arb_profile.py $mode > gpurun_out/arb_$mode.log 2>&1 || { echo arb failed; tail gpurun_out/arb_$mode.log; exit 1; }; echo $mode; cut -c1-200 gpurun_out/arb_$mode.log; done
for C in 5 3 8 5; do
ATE_CF_CONCURRENT=$C timeout -k 10 300 python -u tools/bench_configs.py --configs 3 --panel3 --n3 10000000 --p3 500 --shard3 0/8 --trees3 100 > gpurun_out/cfg3_c$C.log 2>&1 || { echo cfg3 failed; tail -20 gpurun_out/cfg3_c$C.log; exit 1; }
echo "concurrent $C"; tail -1 gpurun_out/cfg3_c$C.log | cut -c 210-290
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_segmented.py -x -q --timeout 240 --timeout-method thread > gpurun_out/r03c_multirank.log 2>&1 || { echo "multirank failed"; tail -40 gpurun_out/r03c_multirank.log; exit 1; }
tail -2 gpurun_out/r03c_multirank.log
timeout -k 10 300 python bench.py --exact 1 > gpurun_out/r03c_bench_exact.log 2>&1 || { echo bench exact failed; tail -20 gpurun_out/r03c_bench_exact.log; exit 1; }
tail -1 gpurun_out/r03c_bench_exact.log | cut -c1-300

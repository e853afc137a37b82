#!/bin/bash
# path-kernel change: enet/DML GPU tests, determinism, bench, cycle profile
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu.py tests/test_gpu_determinism.py tests/test_gpu_graph_estimators.py tests/test_gpu_segmented.py > gpurun_out/r03h_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03h_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r03h_tests.log | head; exit $rc; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r03h_bench.json 2> gpurun_out/r03h_bench.err
rc=$?; python -c "import json; d=json.loads(open('gpurun_out/r03h_bench.json').read().splitlines()[-1]); print('ms', d['ms_per_step'], 'single', d['single_fit_ms'], d['single_fit_ms_all'], 'ate', d['ate_hex'], 'parity', d['parity']['abs_diff_ate'])"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/enet_profile.py > gpurun_out/enet_prof_r03h.json 2> gpurun_out/enet_prof_r03h.err

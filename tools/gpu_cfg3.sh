#!/bin/bash
# Config 3 on HBM panels: parity test, then timings (1e6 x 500 full forests; the per-GPU
# tree shard of N=1e7 x 500 over 8 GPUs). A heartbeat file marks progress of long runs.
set -o pipefail
mkdir -p gpurun_out
( while true; do sleep 50; date >> gpurun_out/cfg3_heartbeat.log; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 300 python -u -m pytest tests/test_forest_gpu.py -x -q --timeout 200 --timeout-method thread -k panel > gpurun_out/cfg3_test.log 2>&1 || { echo test failed; tail -30 gpurun_out/cfg3_test.log; exit 1; }
tail -2 gpurun_out/cfg3_test.log
timeout -k 10 600 python tools/bench_configs.py --configs 3 --panel3 --n3 1000000 --p3 500 --trees3 100 > gpurun_out/cfg3.jsonl 2>&1 || { echo cfg3a failed; tail -20 gpurun_out/cfg3.jsonl; exit 1; }
tail -1 gpurun_out/cfg3.jsonl
timeout -k 10 900 python tools/bench_configs.py --configs 3 --panel3 --n3 10000000 --p3 500 --trees3 100 --shard3 0/8 >> gpurun_out/cfg3.jsonl 2>&1 || { echo cfg3b failed; tail -20 gpurun_out/cfg3.jsonl; exit 1; }
tail -1 gpurun_out/cfg3.jsonl

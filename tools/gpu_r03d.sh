#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err && tail -1 gpurun_out/bench_default.json &&
timeout -k 10 240 python bench.py --steps 20 --warmup 5 --exact 1 > gpurun_out/bench_exact.json 2> gpurun_out/bench_exact.err && tail -1 gpurun_out/bench_exact.json &&
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_multirank.py -k exact 2>&1 | tail -3

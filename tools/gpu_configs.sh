#!/bin/bash
# All BASELINE configs on one GPU (tools/bench_configs.py) + the 14-row driver timing,
# with the package defaults (no environment overrides). Output: gpurun_out/configs.jsonl.
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/configs.jsonl
: > $O
run() { timeout -k 10 "$1" python3 "${@:2}" 2>/dev/null | grep '^{' >> $O || { echo "failed: ${*:2}"; exit 1; }; }
run 200 tools/bench_configs.py --configs 2
run 300 tools/bench_configs.py --configs 3 --panel3 --n3 1000000 --p3 500 --trees3 100
run 400 tools/bench_configs.py --configs 3 --panel3 --n3 10000000 --p3 500 --shard3 0/8
run 200 tools/bench_configs.py --configs 4
run 200 tools/bench_configs.py --configs 5 --panel5 --n5 12500000 --p5 2000 --trees5 10
run 200 tools/replicate_timing.py --passes 3
cut -c1-260 $O

#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for C in 5 3 8 5; do
ATE_CF_CONCURRENT=$C timeout -k 10 300 python -u tools/bench_configs.py --configs 3 --panel3 --n3 10000000 --p3 500 --shard3 0/8 --trees3 100 > gpurun_out/cfg3_c$C.log 2>&1 || { echo cfg3 failed; tail -20 gpurun_out/cfg3_c$C.log; exit 1; }
echo "concurrent $C"; tail -1 gpurun_out/cfg3_c$C.log | cut -c 210-290
done

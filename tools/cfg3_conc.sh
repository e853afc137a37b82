#!/bin/bash
# config-3 per-GPU shard on ONE box at several forest-concurrency caps (ATE_CF_CONCURRENT)
set -o pipefail
mkdir -p gpurun_out
for c in 1 2 3 5; do
  ATE_CF_CONCURRENT=$c timeout -k 10 300 python tools/bench_configs.py --configs 3 --panel3 --n3 10000000 --p3 500 --trees3 100 --shard3 0/8 > gpurun_out/cfg3_conc$c.log 2>&1 || { echo "c=$c failed"; tail -5 gpurun_out/cfg3_conc$c.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/cfg3_conc$c.log').read().splitlines()[-1]); print('concurrency $c', round(d['seconds'], 2), d['ate'])"
done

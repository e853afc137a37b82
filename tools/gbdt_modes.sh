#!/bin/bash
# histogram-kernel ablation on the config-5 shard: 0 full, 1 no LDS atomics, 2 no bins gather,
# 3 neither, 8 G atomics only, 16 H atomics as u32 (timing only; results are meaningless for
# modes != 0)
set -o pipefail
mkdir -p gpurun_out
for m in ${MODES:-0 1 2 3}; do
  ATE_GBDT_HIST_MODE=$m timeout -k 10 300 python tools/cfg5.py --rows 100000000 --cols 2000 --trees ${TREES:-3} --shard 0/8 > gpurun_out/gbdt_mode$m.log 2>&1 || { echo "mode $m failed"; tail -5 gpurun_out/gbdt_mode$m.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/gbdt_mode$m.log').read().splitlines()[-1]); print('mode $m', round(d['seconds'],3))"
done

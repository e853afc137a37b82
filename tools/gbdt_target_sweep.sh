#!/bin/bash
# config-5 shard (3 trees) vs the histogram workgroup target (ATE_GBDT_HIST_TARGET: smaller row
# chunks -> the 8 workgroups sharing a bins line run closer together, more L2 reuse)
set -o pipefail
mkdir -p gpurun_out
for t in ${TARGETS:-512 2048 8192 32768}; do
  ATE_GBDT_HIST_TARGET=$t timeout -k 10 300 python tools/cfg5.py --rows 100000000 --cols 2000 --trees ${TREES:-3} --shard 0/8 > gpurun_out/gbdt_target$t.log 2>&1 || { echo "target $t failed"; tail -5 gpurun_out/gbdt_target$t.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/gbdt_target$t.log').read().splitlines()[-1]); print('target $t', round(d['seconds'], 3), d['ate_hex'])"
done

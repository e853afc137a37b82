#!/bin/bash
# kernel summary of the config-5 per-GPU shard (fewer trees: the per-tree mix is the same)
set -o pipefail
ROOT=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_cfg5" -o cfg5 \
  -- python3 "$ROOT/tools/cfg5.py" --rows 100000000 --cols 2000 --trees ${TREES:-10} --shard 0/8 > "$ROOT/gpurun_out/prof_cfg5.log" 2>&1 || { echo prof failed; tail -20 "$ROOT/gpurun_out/prof_cfg5.log"; exit 1; }
tail -1 "$ROOT/gpurun_out/prof_cfg5.log"
f=$(find $ROOT/gpurun_out/prof_cfg5 -name "*kernel_stats.csv" | head -1)
head -25 "$f"

#!/bin/bash
set -o pipefail
ROOT=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp
ENGINES=level timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_lv" -o lv \
  -- python3 "$ROOT/tools/forest_level_probe.py" > "$ROOT/gpurun_out/prof_lv.log" 2>&1 || { echo prof failed; tail -20 "$ROOT/gpurun_out/prof_lv.log"; exit 1; }
tail -1 "$ROOT/gpurun_out/prof_lv.log"
f=$(find $ROOT/gpurun_out/prof_lv -name "*kernel_stats.csv" | head -1)
cut -c1-200 "$f" | head -24

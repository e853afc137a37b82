#!/bin/bash
# kernel summary of the tutorial driver's passes (tools/replicate_timing.py)
set -o pipefail
ROOT=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_rep" -o rep \
  -- python3 "$ROOT/tools/replicate_timing.py" > "$ROOT/gpurun_out/prof_rep.log" 2>&1 || { echo prof failed; tail -20 "$ROOT/gpurun_out/prof_rep.log"; exit 1; }
f=$(find $ROOT/gpurun_out/prof_rep -name "*kernel_stats.csv" | head -1)
head -30 "$f" | cut -c1-220

#!/bin/bash
# Kernel-level profiles of the headline bench step and of the 14-row driver.
# Run on the GPU box from the repo root; summaries land in gpurun_out/prof_*.
set -o pipefail
ROOT=$(pwd)
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_bench" -o bench \
  -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 > "$ROOT/gpurun_out/prof_bench.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_replicate" -o rep \
  -- python3 "$ROOT/tools/replicate_timing.py" --passes 2 > "$ROOT/gpurun_out/prof_replicate.log" 2>&1 || exit $?
